#!/bin/bash
# round-4 stall passes (cfg3, cfg5, cfg2), digested on the box, raw counters removed
set -o pipefail
for c in "cfg3 lg08_g4_protein_200k_256" "cfg5 nh_gtr_g4_dna_2M_512" "cfg2 gtr_g4_dna_1M_64"; do
  set -- $c
  bash tools/gpu_stalls.sh r4_$1 $2 > /dev/null || exit 1
  mkdir -p gpurun_out/r04stalls
  python tools/stalls_digest.py gpurun_out/stalls/r4_$1 --json gpurun_out/r04stalls/$1_stalls.json > /dev/null || exit 1
  rm -rf gpurun_out/stalls/r4_$1; echo "$1 done"
done
