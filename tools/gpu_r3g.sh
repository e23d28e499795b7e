#!/bin/bash
# Round-3 session G: DR tests + cfg3/cfg4 DR lines after the batched matrix staging of the
# 20-state fused preorder; kernel traces of small cfg2 traversals (fixed cost per launch).
#   tools/gpu_r3g.sh <tag>
set -o pipefail
T=${1:-r3g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dr.py \
  > gpurun_out/$T/dr_tests.log 2>&1 || { echo "dr tests failed"; tail -30 gpurun_out/$T/dr_tests.log; exit 1; }
tail -1 gpurun_out/$T/dr_tests.log
for v in "default:" "levelwise:DR_PRE=0"; do
  n=${v%%:*}; e=${v#*:}
  PLK_TUNE="$e" timeout -k 10 300 python tools/bench_dr.py --config lg08_g4_protein_200k_256 --reps 3 --path-branches 4 \
    > gpurun_out/$T/dr_cfg3_$n.json 2> gpurun_out/$T/dr_cfg3_$n.err || { tail -5 gpurun_out/$T/dr_cfg3_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/$T/dr_cfg3_$n.json'));print('cfg3 DR $n',round(d['dr_ms'],2),'ms',d['dr_path'],d['max_rel_diff_dr_vs_path'])"
done
for P in 4096 65536; do
  ( export TMPDIR=/tmp; cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/k$P -o run -- \
    python3 $R/bench.py --patterns $P --no-cpu-baseline --steps 20 --warmup 3 > $R/gpurun_out/$T/k$P.json 2> $R/gpurun_out/$T/k$P.err ) || { echo "trace $P failed"; exit 1; }
  head -4 gpurun_out/$T/k$P/run_kernel_stats.csv | cut -d, -f1-4
done
