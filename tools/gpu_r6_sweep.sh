#!/bin/bash
# round 6: A/B sweep of PLK_TUNE settings on one box: SWEEP="tune1;tune2;..." ARGS="bench args"
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r6sweep}
mkdir -p $O
export TMPDIR=/tmp
IFS=';' read -ra TS <<< "$SWEEP"
for rep in ${REPS:-1}; do :; done
for r in $(seq 1 ${REPS:-1}); do
for t in "${TS[@]}"; do
  n=$(echo "$t" | tr ',=' '__')
  [ -z "$n" ] && n=default
  PLK_TUNE="$t" timeout -k 10 300 python bench.py --no-cpu-baseline --no-strong $ARGS > $O/b_${n}_$r.json 2> $O/b_${n}_$r.err || { echo "FAIL $t"; tail -5 $O/b_${n}_$r.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/b_${n}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']
print('%-40s ms/step %.4f trav %.1f us frac %.3f' % ('$t' or 'default', d['ms_per_step'], r['traversal_ms']*1e3, r['frac']))"
done
done
if [ -n "$PROF" ]; then
  cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o r6 -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-strong $ARGS > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
  cd $GRAFT_REPO_ROOT
  f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 $f | head -12
fi
