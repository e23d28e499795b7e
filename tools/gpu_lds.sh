#!/bin/bash
# LDS / issue counters of the partials kernel: tools/gpu_lds.sh <tag> <config> [VAR=value ...]
set -o pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lds/$TAG
mkdir -p $O
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
cd /tmp
B="$R/bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $O/l1 -o run -- python3 $B > /dev/null 2> $O/l1.err || { tail -5 $O/l1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $O/l2 -o run -- python3 $B > /dev/null 2> $O/l2.err || { tail -5 $O/l2.err; exit 1; }
echo "lds $TAG done"
