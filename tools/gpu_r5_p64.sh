#!/bin/bash
# Stall counters of cfg4's two small kernels (pmat64s_kernel, cherry_table_kernel<64>)
set -o pipefail
bash tools/gpu_stalls.sh r5p64 yn98_codon_50k_128 lnl > /dev/null || exit 1
mkdir -p gpurun_out/r5p64
for k in pmat64s_kernel cherry_table_kernel treeM_kernel; do
  python tools/stalls_digest.py gpurun_out/stalls/r5p64 $k --json gpurun_out/r5p64/$k.json || exit 1
done
rm -rf gpurun_out/stalls/r5p64
