#!/bin/bash
# round 6 session runner: TAG=name PYT="pytest args" BENCH="bench args;bench args2" tools/gpu_r6_run.sh
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r6}
mkdir -p $O
export TMPDIR=/tmp
rc=0
if [ -n "$PYT" ]; then
  timeout -k 10 ${PYT_TIMEOUT:-600} python -u -m pytest -x -v --timeout 120 --timeout-method thread $PYT > $O/pytest.log 2>&1
  rc=$?
  tail -5 $O/pytest.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $O/pytest.log | head -20; exit $rc; }
fi
if [ -n "$BENCH" ]; then
  i=0
  IFS=';' read -ra BS <<< "$BENCH"
  for b in "${BS[@]}"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py $b > $O/bench_$i.json 2> $O/bench_$i.err || { echo "bench $i failed"; tail -20 $O/bench_$i.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench $i: $b |', d['config']['workload'][:40], '| ms/step %.4f value %.3e frac %.3f trav %.1f us' % (d['ms_per_step'], d['value'], r['frac'], r['traversal_ms']*1e3), d.get('kernel_path'))"
  done
fi
exit $rc
