#!/bin/bash
# cfg5 with split launch: group count x fragment height
set -o pipefail
bash tools/gpu_sweep_env.sh r2p nh_gtr_g4_dna_2M_512 "g8:PLK_JIT_G=8" "g6:PLK_JIT_G=6" "g7:PLK_JIT_G=7" "g8dm5:PLK_JIT_G=8,PLK_JIT_CIW_DM=5" "g8l2:PLK_JIT_G=8,PLK_JIT_L=2" "g8t64:PLK_JIT_G=8,PLK_JIT_TAB_KB=64" "g8p96:PLK_JIT_G=8,PLK_JIT_PAIR_KB=96" || exit 1
bash tools/gpu_sweep_env.sh r2p2 gtr_g4_dna_1M_64 "g2:PLK_JIT_G=2" "g4:PLK_JIT_G=4" "l4:PLK_JIT_L=4" "dm8:PLK_JIT_DM=8" || exit 1
