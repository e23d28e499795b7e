#!/bin/bash
# round 6: same-box A/B of cfg2 bench lines, this tree's libplk against another build (PLK_LIB),
# alternating (driver window)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r6libab}
B=$1
shift
mkdir -p $O
export TMPDIR=/tmp PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache_ab
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-strong "$@" > $O/new_$i.json 2> $O/new_$i.err || exit 1
  PLK_LIB=$PWD/$B timeout -k 10 300 python bench.py --no-cpu-baseline --no-strong "$@" > $O/old_$i.json 2> $O/old_$i.err || exit 1
done
python3 - <<PY
import json
for v in ("new", "old"):
    for i in (1, 2, 3):
        r = json.loads(open(f"$O/{v}_{i}.json").read().strip().splitlines()[-1])
        print(v, i, "%.4f" % r["ms_per_step"], "%.1f" % (r["roofline"]["traversal_ms"] * 1e3), r["host_us_per_eval"])
PY
