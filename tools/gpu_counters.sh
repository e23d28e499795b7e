#!/bin/bash
# PMC counter groups for the partials kernel of one bench config (separate passes):
#   tools/gpu_counters.sh <tag> <config> [VAR=value ...]
# -> gpurun_out/prof/<tag>/{g1,g2,g3}; digest with tools/counters_digest.py <tag>
set -o pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof/$TAG
mkdir -p $O
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
cd /tmp
B="$R/bench.py --config $CFG --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 300 python3 $B > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d $O/g1 -o run -- python3 $B > /dev/null 2> $O/g1.err || { tail -5 $O/g1.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_BRANCH --output-format csv -d $O/g2 -o run -- python3 $B > /dev/null 2> $O/g2.err || { tail -5 $O/g2.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/g3 -o run -- python3 $B > /dev/null 2> $O/g3.err || { tail -3 $O/g3.err; }
echo "counters $TAG done"
