#!/bin/bash
# In-kernel timestamps of the JIT traversal (PLK_DEBUG_TIMES: staging, first super-blocks, end)
set -o pipefail
export PLK_DEBUG_TIMES=1
for a in "--config nh_gtr_g4_dna_2M_512 --patterns 4096" "--config nh_gtr_g4_dna_2M_512" "--config nh_gtr_g4_dna_2M_512 --patterns 2000000" "--patterns 4096" ""; do
  echo "=== $a"
  timeout -k 10 120 python bench.py $a --no-cpu-baseline --no-strong --steps 4 --warmup 3 2>&1 >/dev/null | grep -A 8 "plk times" || exit 1
done
