#!/bin/bash
# 4-state kernel: cost of the per-workgroup table staging (launch returning after it)
set -o pipefail
bash tools/gpu_sweep_env.sh r2t gtr_g4_dna_1M_64 "base:" "stage:PLK_DEBUG_STAGE_ONLY=1" "empty:PLK_DEBUG_STAGE_ONLY=2" || exit 1
bash tools/gpu_sweep_env.sh r2t5 nh_gtr_g4_dna_2M_512 "base:" "stage:PLK_DEBUG_STAGE_ONLY=1" "empty:PLK_DEBUG_STAGE_ONLY=2" || exit 1
