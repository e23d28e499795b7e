#!/bin/bash
# round 6: one wave per quad in the quad build -- parity (quads bitwise, root rules, cfg2 at
# config shape), then cfg2 lines and the prologue stamps
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r6qb}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "quads_bitwise or bitwise_equals_interpreter or root_rules" tests/test_gpu_root_rules.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/line_$r.json 2> $O/err_$r.log || { tail -5 $O/err_$r.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/line_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('line', d['ms_per_step'], r['traversal_ms']*1e3, r['frac'])"
done
TAG=${TAG:-r6qb}/pro PATS=1000000 TUNES=default bash tools/gpu_r6_prologue.sh
