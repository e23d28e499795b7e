#!/bin/bash
# HBM traffic of the DR pass: separate FETCH_SIZE / WRITE_SIZE passes over tools/bench_dr.py
# (per-kernel rows in gpurun_out/prof/<tag>/{fetch,write}).
#   tools/gpu_dr_pmc.sh <tag> [config]
set -o pipefail
T=${1:-drpmc}; CFG=${2:-gtr_g4_dna_1M_64}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof/$T
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- \
    python3 $R/tools/bench_dr.py --config $CFG --path-branches 1 --reps 1 > /dev/null 2> $O/$c.err || { tail -3 $O/$c.err; exit 1; }
done
echo "dr pmc $T done"
