#!/bin/bash
# Profiling session on the GPU box: kernel-trace stats and separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ instruction mix) for one config/mode of bench.py.
#   tools/gpu_prof.sh <tag> <config> <mode> [steps]
# Outputs land in gpurun_out/prof/<tag>/ ; tools/traffic_from_pmc.py digests them.
set -o pipefail
TAG=$1; CFG=$2; MODE=$3; STEPS=${4:-10}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --config $CFG --mode $MODE --no-cpu-baseline --no-strong"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $B --steps $STEPS --warmup 2 > $O/bench.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
  python3 $B --steps 2 --warmup 1 > /dev/null 2> $O/fetch.err || { tail -5 $O/fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
  python3 $B --steps 2 --warmup 1 > /dev/null 2> $O/write.err || { tail -5 $O/write.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES \
  SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d $O/sq -o run -- \
  python3 $B --steps 2 --warmup 1 > /dev/null 2> $O/sq.err || { tail -5 $O/sq.err; exit 1; }
echo "profiled $TAG"
cat $O/bench.json
