#!/bin/bash
# 4-state P(t) with a 1 KB kernel-argument request (<= 64 branches) vs the 2.5 KB one (PLK_TUNE PSMALL=0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5psmall
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "pmat4 or evaluate_equals or pmat_request or random_vs_oracle or reference_goldens" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "PSMALL=0" "PSMALL=1" "PSMALL=0" "PSMALL=1" "PSMALL=0" "PSMALL=1" "PSMALL=0" "PSMALL=1"; do
  PLK_TUNE=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-strong > $O/line.json 2> $O/line.err || { tail -5 $O/line.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/line.json'));print('$v', round(d['ms_per_step'],5), round(d['roofline']['frac'],3), d.get('host_us_per_eval'))"
done
