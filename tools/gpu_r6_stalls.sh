#!/bin/bash
# round 6: stall passes of cfg2's traversal with and without quad units, digested, plus kernel-trace stats
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6stalls
for v in "quad" "noquad JIT_QUAD_KB=0"; do
  set -- $v
  PLK_TUNE="$2" bash tools/gpu_stalls.sh r6_$1 gtr_g4_dna_1M_64 > /dev/null || exit 1
  python tools/stalls_digest.py gpurun_out/stalls/r6_$1 --json gpurun_out/r6stalls/cfg2_$1_stalls.json || exit 1
  rm -rf gpurun_out/stalls/r6_$1
done
cd /tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6stalls/trace -o r6 -- \
  python3 $R/bench.py --no-cpu-baseline --no-strong > $R/gpurun_out/r6stalls/bench_trace.json 2> $R/gpurun_out/r6stalls/trace.err || exit 1
cd $R
f=$(find gpurun_out/r6stalls/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 $f | head -8
