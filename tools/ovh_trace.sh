#!/bin/bash
# Per-evaluation timeline of the default bench path at a tiny pattern count (fixed costs):
# rocprofv3 kernel trace (start/end of every kernel) -> gaps between the pmat, traversal
# and block-sum kernels and between evaluations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof/${1:-ovh}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --no-cpu-baseline --steps 100 --warmup 10 --patterns ${2:-4096} > $O/bench.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
find $O -name "*kernel_trace.csv" | head -3
