#!/bin/bash
# cfg5 250k line: per-class scaling (JIT_PCS=1, DM 6 cut) vs classes in the wave, alternating.
set -o pipefail
O=gpurun_out/${1:-r5p2}
mkdir -p $O
shift
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
for i in 1 2; do
  for v in 0 1; do
    PLK_TUNE=JIT_PCS=$v$EXTRA timeout -k 10 300 python bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong "$@" > $O/cfg5_pcs${v}_$i.json 2> $O/cfg5_pcs${v}_$i.err || exit $?
  done
done
python - <<PY
import json
for v in ("0", "1"):
    for i in (1, 2):
        r = json.load(open(f"$O/cfg5_pcs{v}_{i}.json"))
        print("pcs", v, i, "250k %.4f trav %.4f frac %.3f" % (r["ms_per_step"], r["roofline"]["traversal_ms"], r["roofline"]["frac"]), r["partials_launches_per_step"], r["lnl"])
PY
