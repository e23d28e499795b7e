#!/bin/bash
# DR pass A/B on one GPU: tests of the fused preorder and the C++ mirror, then
# tools/bench_dr.py per config with the default DR path, the levelwise one (DR_PRE=0) and the
# fused preorder (DR_PRE=1), and the mirror bench lines.
#   tools/gpu_dr_ab.sh <prefix> [configs...]
set -o pipefail
P=${1:-dr}; shift
CFGS=${@:-lg08_g4_protein_200k_256 yn98_codon_50k_128}
mkdir -p gpurun_out/$P
timeout -k 10 600 python -u -m pytest tests/test_gpu_dr.py tests/test_gpu_host.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/$P/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$P/pytest.log; exit 1; }
tail -1 gpurun_out/$P/pytest.log
for c in $CFGS; do
  for v in "default:" "levelwise:DR_PRE=0" "fused:DR_PRE=1"; do
    n=${v%%:*}; e=${v#*:}
    PLK_TUNE="$e" timeout -k 10 300 python tools/bench_dr.py --config $c --reps 3 --path-branches 4 > gpurun_out/$P/${c}_$n.json 2> gpurun_out/$P/${c}_$n.err || { tail -5 gpurun_out/$P/${c}_$n.err; exit 1; }
    python3 -c "
import json
d=json.load(open('gpurun_out/$P/${c}_$n.json')); print('$c', '$n', round(d['dr_ms'],3), 'ms', d.get('dr_path'), 'maxrel', d['max_rel_diff_dr_vs_path'])"
  done
done
for c in cfg2 cfg3; do
  timeout -k 10 200 bpp-phyl_amd/host/bin/bench_mirror $c > gpurun_out/$P/mirror_$c.json || exit 1
  cat gpurun_out/$P/mirror_$c.json
done
