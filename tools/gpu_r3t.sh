#!/bin/bash
# Round-3 session T: 64-state P(t) kernel writing the transposed copy (no transpose launch):
# 64-state tests, cfg4 line and kernel trace.
set -o pipefail
T=${1:-r3t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  -k "64 or yn98 or codon or pmat or treeM" > gpurun_out/$T/focus.log 2>&1 || { echo "focus failed"; tail -30 gpurun_out/$T/focus.log; exit 1; }
tail -1 gpurun_out/$T/focus.log
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/k_cfg4 -o run -- \
  python3 $R/bench.py --config yn98_codon_50k_128 --no-cpu-baseline --steps 10 --warmup 2 > $R/gpurun_out/$T/k_cfg4.json 2> $R/gpurun_out/$T/k_cfg4.err ) || { echo "trace failed"; exit 1; }
cut -d, -f1-4 gpurun_out/$T/k_cfg4/run_kernel_stats.csv | head -8
bash tools/ab_bench.sh $T/ab yn98_codon_50k_128 "a:" "b:" || exit 1
