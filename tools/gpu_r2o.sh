#!/bin/bash
# workgroups split over a tier's fragments (all fragments at once): cfg5 / cfg2 A/B + parity subset
set -o pipefail
bash tools/gpu_sweep_env.sh r2o nh_gtr_g4_dna_2M_512 "split:" "nosplit:PLK_JIT_SPLIT_Y=0" "split_g8:PLK_JIT_G=8" "split_dm7:PLK_JIT_CIW_DM=7" "split_dm5:PLK_JIT_CIW_DM=5" || exit 1
bash tools/gpu_sweep_env.sh r2o2 gtr_g4_dna_1M_64 "split:" "nosplit:PLK_JIT_SPLIT_Y=0" || exit 1
bash tools/gpu_tests.sh r2o -k "jit_tree4 or nonhomogeneous or bench_mode" quick || exit 1
