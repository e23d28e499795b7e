#!/bin/bash
# Round-3 session Q: kernel trace of config 5 as BASELINE states it (2 M patterns, strong
# scaling, N = 1), for the roofline of the 2 M line.
set -o pipefail
T=${1:-r3q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/k_cfg5_2M -o run -- \
  python3 $R/bench.py --scaling strong --no-cpu-baseline --steps 10 --warmup 2 > $R/gpurun_out/$T/cfg5_2M.json 2> $R/gpurun_out/$T/cfg5_2M.err ) || { echo "trace failed"; tail -5 gpurun_out/$T/cfg5_2M.err; exit 1; }
cut -d, -f1-7 gpurun_out/$T/k_cfg5_2M/run_kernel_stats.csv | head -6
