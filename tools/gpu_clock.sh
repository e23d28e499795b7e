#!/bin/bash
# Effective clock and VALU issue share of the partials kernel of one config, plus the
# generated JIT source / code object (PLK_JIT_DUMP):
#   tools/gpu_clock.sh <tag> <config> [VAR=value ...]   -> gpurun_out/clock/<tag>/
set -o pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/clock/$TAG
mkdir -p $O/jit
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
cd /tmp
B="$R/bench.py --config $CFG --no-cpu-baseline --steps 5 --warmup 2"
PLK_JIT_DUMP=$O/jit timeout -k 10 300 python3 $B > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY --output-format csv -d $O/c1 -o run -- python3 $B > /dev/null 2> $O/c1.err || { tail -5 $O/c1.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $B > /dev/null 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
echo "clock $TAG done"
