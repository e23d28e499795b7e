#!/bin/bash
# Same-box A/B of bench lines: this tree's libplk against an A/B build (PLK_LIB=$2), alternating.
set -o pipefail
O=gpurun_out/${1:-r5ab}
B=$2
shift 2
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/new_$i.json 2> $O/new_$i.err || exit $?
  PLK_LIB=$PWD/$B timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/old_$i.json 2> $O/old_$i.err || exit $?
done
python - <<PY
import json
for v in ("new", "old"):
    for i in (1, 2, 3):
        r = json.load(open(f"$O/{v}_{i}.json"))
        s = r.get("strong", {})
        print(v, i, "%.4f" % r["ms_per_step"], "%.4f" % r["roofline"]["traversal_ms"], "strong %.4f %.4f" % (s.get("ms_per_step", 0), s.get("traversal_ms", 0)), r["host_us_per_eval"])
PY
