#!/bin/bash
# cfg5: fragment depth x workgroup size around G=4, DM=6
set -o pipefail
bash tools/gpu_sweep_env.sh r2h nh_gtr_g4_dna_2M_512 "g4dm6:PLK_JIT_G=4,PLK_JIT_CIW_DM=6" "g4dm7:PLK_JIT_G=4,PLK_JIT_CIW_DM=7" "g4dm8:PLK_JIT_G=4,PLK_JIT_CIW_DM=8" "g3dm6:PLK_JIT_G=3,PLK_JIT_CIW_DM=6" "g8dm6:PLK_JIT_G=8,PLK_JIT_CIW_DM=6" "g8dm7:PLK_JIT_G=8,PLK_JIT_CIW_DM=7" "g4dm6l2:PLK_JIT_G=4,PLK_JIT_CIW_DM=6,PLK_JIT_L=2" "g4dm6p32:PLK_JIT_G=4,PLK_JIT_CIW_DM=6,PLK_JIT_PAIR_KB=32" "g4dm6p96:PLK_JIT_G=4,PLK_JIT_CIW_DM=6,PLK_JIT_PAIR_KB=96" "g4dm6t96:PLK_JIT_G=4,PLK_JIT_CIW_DM=6,PLK_JIT_TAB_KB=96" || exit 1
