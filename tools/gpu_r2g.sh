#!/bin/bash
# cfg5 workgroup-size sweep after the hi-word rescale and laundered slot bases
set -o pipefail
bash tools/gpu_sweep_env.sh r2g nh_gtr_g4_dna_2M_512 "base:" "g4:PLK_JIT_G=4" "g4l2:PLK_JIT_G=4,PLK_JIT_L=2" "g6:PLK_JIT_G=6" "g8:PLK_JIT_G=8" "g8l2:PLK_JIT_G=8,PLK_JIT_L=2" "g4dm4:PLK_JIT_G=4,PLK_JIT_CIW_DM=4" "g4dm6:PLK_JIT_G=4,PLK_JIT_CIW_DM=6" "g4w3:PLK_JIT_G=4,PLK_JIT_MINW=3" || exit 1
