#!/bin/bash
# default bench line: steps / warmup sensitivity on one box (alternating)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5warm
mkdir -p $O
for v in "20 3" "20 50" "200 20" "20 3" "20 50" "200 20" "20 3"; do
  set -- $v
  timeout -k 10 200 python3 bench.py --steps $1 --warmup $2 > $O/l_$1_$2.json 2> $O/l.err || { tail -5 $O/l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/l_$1_$2.json'));print('steps $1 warmup $2', round(d['ms_per_step'],5), d['roofline']['frac'], d.get('host_us_per_eval'))"
done
