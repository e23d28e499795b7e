#!/bin/bash
# cost of the P(t) scalar loads: every internal branch reading node 0's P (constant address)
set -o pipefail
bash tools/gpu_sweep_env.sh r2k5 nh_gtr_g4_dna_2M_512 "base:" "samep:PLK_DEBUG_SAMEP=1" || exit 1
bash tools/gpu_sweep_env.sh r2k2 gtr_g4_dna_1M_64 "base:" "samep:PLK_DEBUG_SAMEP=1" || exit 1
