#!/bin/bash
# Same-box A/B of cfg5 lines (250k shard and the 2M strong line) over PLK_TUNE variants given
# as arguments ("-" = no PLK_TUNE), two alternating rounds:
#   tools/gpu_r5_tune_ab.sh <tag> - JIT_LR=4 ...
set -o pipefail
O=gpurun_out/${1:-r5tab}
shift
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
for i in 1 2; do
  for v in "$@"; do
    t=$(echo $v | tr '=,' '__'); tv=$v; [ "$v" = "-" ] && tv=""
    PLK_TUNE=$tv timeout -k 10 300 python bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong > $O/c5_${t}_$i.json 2> $O/c5_${t}_$i.err || exit $?
    PLK_TUNE=$tv timeout -k 10 300 python bench.py --scaling strong --no-cpu-baseline --steps 10 > $O/c5s_${t}_$i.json 2> $O/c5s_${t}_$i.err || exit $?
  done
done
python - "$O" "$@" <<'PY'
import json, sys
O = sys.argv[1]
for v in sys.argv[2:]:
    t = v.replace("=", "_").replace(",", "_")
    for i in (1, 2):
        r = json.load(open(f"{O}/c5_{t}_{i}.json")); s = json.load(open(f"{O}/c5s_{t}_{i}.json"))
        print(v, i, "250k %.4f trav %.4f frac %.3f" % (r["ms_per_step"], r["roofline"]["traversal_ms"], r["roofline"]["frac"]),
              "| 2M %.4f trav %.4f" % (s["ms_per_step"], s["roofline"]["traversal_ms"]), r["lnl"], s["lnl"])
PY
