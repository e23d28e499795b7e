#!/bin/bash
# Host turnaround between evaluations (cfg2 default line): runtime wait modes, alternating.
set -o pipefail
O=gpurun_out/${1:-r5e}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-strong --steps 40 > $O/$tag.json 2> $O/$tag.err || exit $?; }
for i in 1 2; do
  run base_$i X=1
  run intr0_$i HSA_ENABLE_INTERRUPT=0
  run spin_$i ROC_ACTIVE_WAIT_TIMEOUT=100000
done
python - <<PY
import json
for t in ("base", "intr0", "spin"):
    for i in (1, 2):
        r = json.load(open(f"$O/{t}_{i}.json"))
        print(t, i, "%.4f" % r["ms_per_step"], "%.4f" % r["roofline"]["traversal_ms"], r["host_us_per_eval"])
PY
