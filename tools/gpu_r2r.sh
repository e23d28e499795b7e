#!/bin/bash
# jit_treeM: unconditional P staging stores (padded LDS stride); Y-outer contraction order A/B
set -o pipefail
bash tools/gpu_sweep_env.sh r2r lg08_g4_protein_200k_256 "base:" "youter:PLK_JITM_YOUTER=1" "youter_dm3:PLK_JITM_YOUTER=1,PLK_JITM_DM=3" "youter_w1:PLK_JITM_YOUTER=1,PLK_JITM_MINW=1" || exit 1
bash tools/gpu_tests.sh r2r -k "jit_treeM or bench_mode or subtree_patterns_any" quick || exit 1
PLK_JITM_YOUTER=1 bash tools/gpu_tests.sh r2r_y -k "jit_treeM_vs_oracle" quick || exit 1
