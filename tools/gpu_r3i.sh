#!/bin/bash
# Round-3 session I: tests of jit_treeM's XCD-major work order and the early first code fetch
# of jit_tree4; cfg3 A/B of the work order (+ its L2-miss traffic), cfg2 small/large lines.
#   tools/gpu_r3i.sh <tag>
set -o pipefail
T=${1:-r3i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  -k "xcd_order or issue_orders or jit_tree4_bitwise or jit_treeM_vs_oracle" > gpurun_out/$T/focus.log 2>&1 || { echo "focus failed"; tail -30 gpurun_out/$T/focus.log; exit 1; }
tail -1 gpurun_out/$T/focus.log
bash tools/ab_bench.sh $T/cfg3 lg08_g4_protein_200k_256 "xcd1:" "xcd0:JITM_XCD=0" "xcd1b:" "xcd0b:JITM_XCD=0" || exit 1
export TMPDIR=/tmp
for v in "xcd1:" "xcd0:JITM_XCD=0"; do
  n=${v%%:*}; e=${v#*:}
  ( cd /tmp && PLK_TUNE="$e" timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/$T/fetch_$n -o run -- \
      python3 $R/bench.py --config lg08_g4_protein_200k_256 --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2> $R/gpurun_out/$T/fetch_$n.err ) || { echo "fetch $n failed"; exit 1; }
  ( cd /tmp && PLK_TUNE="$e" timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/$T/l2_$n -o run -- \
      python3 $R/bench.py --config lg08_g4_protein_200k_256 --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2> $R/gpurun_out/$T/l2_$n.err ) || { echo "l2 $n failed"; exit 1; }
done
bash tools/gpu_sweep.sh $T/sweep gtr_g4_dna_1M_64 "4096 1000000" "base:" || exit 1
