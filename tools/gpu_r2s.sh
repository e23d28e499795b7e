#!/bin/bash
# jit_treeM staging stores: padded/unconditional vs conditional, same box
set -o pipefail
bash tools/gpu_sweep_env.sh r2s lg08_g4_protein_200k_256 "pad:" "nopad:PLK_JITM_PADSTAGE=0" "pad2:" "nopad2:PLK_JITM_PADSTAGE=0" || exit 1
