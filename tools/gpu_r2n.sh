#!/bin/bash
# cfg5 after the P stream: remaining P-load cost (same-P) and workgroup size
set -o pipefail
bash tools/gpu_sweep_env.sh r2n nh_gtr_g4_dna_2M_512 "base:" "samep:PLK_DEBUG_SAMEP=1" "g3:PLK_JIT_G=3" "g5:PLK_JIT_G=5" "g6:PLK_JIT_G=6" "pair32:PLK_JIT_PAIR_KB=48" "w2:PLK_JIT_MINW=2" || exit 1
