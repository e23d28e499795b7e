#!/bin/bash
# Kernel + memory-copy timeline of a short bench run (gaps between GPU operations).
#   tools/gpu_timeline.sh <tag> <config> [bench args]
set -o pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl -o run -- \
  python3 $R/bench.py --config $CFG --steps 6 --warmup 2 --no-cpu-baseline "$@" > $O/bench.json 2> $O/tl.err || { tail -5 $O/tl.err; exit 1; }
echo "timeline $TAG done"
