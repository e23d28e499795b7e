#!/bin/bash
# new cfg5 defaults (G=4, DM=6): counters list, bench, stall passes for cfg5 and cfg2
set -o pipefail
mkdir -p gpurun_out/r2i
( cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r2i/counters.txt 2>&1 ) || echo "list failed"
bash tools/gpu_sweep_env.sh r2i nh_gtr_g4_dna_2M_512 "cfg5:" || exit 1
bash tools/gpu_stalls.sh cfg5 nh_gtr_g4_dna_2M_512 || exit 1
bash tools/gpu_stalls.sh cfg2 gtr_g4_dna_1M_64 || exit 1
bash tools/gpu_stalls.sh cfg3 lg08_g4_protein_200k_256 || exit 1
