#!/bin/bash
# rocprofv3 kernel-trace stats of one bench line:  tools/gpu_r4_prof.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py "$@" > $O/bench.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
echo "profiled $TAG"; head -c 300 $O/bench.json; echo
