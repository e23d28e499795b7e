#!/bin/bash
# round 6: how long the one-class-per-workgroup traversal's prologue (code fetch, table staging,
# quad build) takes, from PLK_DEBUG_CLOCK=2 stamps (end stamp where the super-block loop starts)
# against the whole-kernel stamps (=1); cfg2 at 1M and 65536 patterns, quads on / off
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r6pro}
mkdir -p $O
export TMPDIR=/tmp
for pat in ${PATS:-1000000 65536}; do
for tune in ${TUNES:-default JIT_QUAD_KB=0}; do
for m in 2 1; do
  t=$tune; [ "$t" = default ] && t=""
  n=${pat}_$(echo "${tune}" | tr ',=' '__')_m$m
  PLK_TUNE="$t" PLK_DEBUG_CLOCK=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-strong --patterns $pat \
    --clock-json $O/clk_$n.json > $O/line_$n.json 2> $O/err_$n.log || { echo "FAIL $n"; tail -5 $O/err_$n.log; exit 1; }
  python - <<PY
import json, statistics as st
d = json.load(open("$O/clk_$n.json"))
rows = [e for e in d["evaluations"] if e[6] == "timed"]
span = [e[3] for e in rows]
mhz = [e[0] for e in rows]
wg = rows[0][4]
l = json.loads(open("$O/line_$n.json").read().strip().splitlines()[-1])
print("%-40s span median %.1f us (min %.1f max %.1f) MHz %.0f wg %d traversal %.1f us" % ("$n", st.median(span), min(span), max(span), st.median(mhz), wg, l["roofline"]["traversal_ms"] * 1e3))
PY
done
done
done
