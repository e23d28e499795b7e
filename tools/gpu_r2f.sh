#!/bin/bash
# hi-word rescale decision: jit parity (scaling cases) then cfg5 / cfg3 / cfg2 A/B
set -o pipefail
bash tools/gpu_tests.sh r2f -k "jit or scaling or rescale or fixture" quick || exit 1
bash tools/gpu_sweep_env.sh r2f nh_gtr_g4_dna_2M_512 "base:" "dm4:PLK_JIT_CIW_DM=4" "dm6:PLK_JIT_CIW_DM=6" "l2:PLK_JIT_L=2" "g1:PLK_JIT_G=1" "g4:PLK_JIT_G=4" "minw3:PLK_JIT_MINW=3" "ciw0:PLK_JIT_CIW=0" || exit 1
bash tools/gpu_sweep_env.sh r2f3 lg08_g4_protein_200k_256 "base:" || exit 1
bash tools/gpu_sweep_env.sh r2f2 gtr_g4_dna_1M_64 "base:" || exit 1
