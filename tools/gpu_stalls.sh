#!/bin/bash
# Stall breakdown of the traversal kernel for one bench config: two SQ counter passes
# (waits, per-pipe activity) plus the GPU clock counters, and a third for memory latencies
# (SQ_INST_LEVEL_x / SQ_INSTS_x = average cycles in flight per instruction).
#   tools/gpu_stalls.sh <tag> <config> [mode]
set -o pipefail
TAG=$1; CFG=$2; MODE=${3:-lnl}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/stalls/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --config $CFG --mode $MODE --no-cpu-baseline --no-strong --steps 2 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --output-format csv -d $O/a -o run -- \
  python3 $B > /dev/null 2> $O/a.err || { tail -5 $O/a.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/b -o run -- \
  python3 $B > /dev/null 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS \
  SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS --output-format csv -d $O/c -o run -- \
  python3 $B > /dev/null 2> $O/c.err || { tail -5 $O/c.err; exit 1; }
echo "stalls $TAG done"
