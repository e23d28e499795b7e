#!/bin/bash
# pipelined P(t) loads for classes-in-wave: parity subset, then cfg5 A/B
set -o pipefail
bash tools/gpu_tests.sh r2l -k "jit_tree4 or nonhomogeneous or scaling or bench_mode" quick || exit 1
bash tools/gpu_sweep_env.sh r2l nh_gtr_g4_dna_2M_512 "ppipe:" "noppipe:PLK_JIT_PPIPE=0" "ppipe_dm5:PLK_JIT_CIW_DM=5" "ppipe_g8:PLK_JIT_G=8" || exit 1
bash tools/gpu_sweep_env.sh r2l2 gtr_g4_dna_1M_64 "base:" || exit 1
