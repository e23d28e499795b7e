#!/bin/bash
# cfg4 dispatch timeline (cherry tables, P(t), traversal tiers)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/cfg3t
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- \
  python3 $R/bench.py --config lg08_g4_protein_200k_256 --no-cpu-baseline --no-strong --steps 6 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
python3 $R/tools/trace_summary.py $O/t/run_kernel_trace.csv 16 && rm -rf $O/t
