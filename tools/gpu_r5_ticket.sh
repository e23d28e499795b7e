#!/bin/bash
# A/B of the exit ticket (PLK_TUNE JIT_TICKET 0/1/2) against the round-4 library, same box.
set -o pipefail
O=gpurun_out/${1:-r5t}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
for i in 1 2; do
  for v in 0 1 2 old; do
    if [ $v = old ]; then
      PLK_LIB=$PWD/ab/libplk_r4.so timeout -k 10 300 python bench.py --no-cpu-baseline > $O/t${v}_$i.json 2> $O/t${v}_$i.err || exit $?
    else
      PLK_TUNE=JIT_TICKET=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/t${v}_$i.json 2> $O/t${v}_$i.err || exit $?
    fi
  done
done
python - <<PY
import json
for v in ("0", "1", "2", "old"):
    for i in (1, 2):
        r = json.load(open(f"$O/t{v}_{i}.json"))
        s = r.get("strong", {})
        print(v, i, "%.4f" % r["ms_per_step"], "%.4f" % r["roofline"]["traversal_ms"], "strong %.4f %.4f" % (s.get("ms_per_step", 0), s.get("traversal_ms", 0)), r["host_us_per_eval"]["blocks_call"])
PY
