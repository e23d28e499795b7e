#!/bin/bash
# Row f4 profile: rocprofv3 kernel-trace stats of tools/bench_dr.py on one config.
#   tools/gpu_dr_prof.sh <tag> [config]
set -o pipefail
T=${1:-dr}; CFG=${2:-gtr_g4_dna_1M_64}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof/$T
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/$T/trace -o run -- \
  python3 $R/tools/bench_dr.py --config $CFG --path-branches 16 > $R/gpurun_out/prof/$T/bench.json 2> $R/gpurun_out/prof/$T/trace.err || { tail -5 $R/gpurun_out/prof/$T/trace.err; exit 1; }
cat $R/gpurun_out/prof/$T/bench.json
