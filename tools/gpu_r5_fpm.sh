#!/bin/bash
# Round 5: P(t) request computed in the jit_tree4 traversal's prologue (JIT_FPM) -- the
# evaluate / pmat / jit tests, then cfg2 default lines with PLK_TUNE JIT_FPM=0 / 1,
# alternating, and the 8-shard one-process fan-out rehearsal.
set -o pipefail
O=gpurun_out/${1:-r5fpm}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "evaluate or pmat4 or jit_tree4 or dynamic" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_fpm.log 2>&1
rc=$?; tail -3 $O/pytest_fpm.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/pytest_fpm.log | head -30; exit $rc; }
for i in 1 2 3; do
  for v in 0 1; do
    PLK_TUNE=JIT_FPM=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-strong > $O/c2_fpm${v}_$i.json 2> $O/c2_fpm${v}_$i.err || exit $?
  done
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for v in ("0", "1"):
    for i in (1, 2, 3):
        r = json.load(open(f"{O}/c2_fpm{v}_{i}.json"))
        print("fpm", v, i, "%.4f trav %.4f" % (r["ms_per_step"], r["roofline"]["traversal_ms"]), r["host_us_per_eval"], r["lnl"])
PY
for v in 0 1; do
  PLK_TUNE=JIT_FPM=$v timeout -k 10 300 python bench.py --gpus 8 --devices 0,0,0,0,0,0,0,0 --no-cpu-baseline --steps 20 > $O/fan_fpm$v.json 2> $O/fan_fpm$v.err || exit $?
  python -c "
import json;r=json.load(open('$O/fan_fpm$v.json'));f=r['fanout'];s=r['strong']['fanout']
print('fanout fpm $v weak', round(f['launch_spread_mean_us'],2), round(f['launch_spread_max_us'],2), 'strong', round(s['launch_spread_mean_us'],2), round(s['launch_spread_max_us'],2), r['ms_per_step'])"
done
