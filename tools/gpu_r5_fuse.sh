#!/bin/bash
# Round 5: fused root fragment (JIT_FUSE) -- the jit_tree4 / config / multi-device tests, then
# cfg5 lines (250k shard and the 2M strong line) with PLK_TUNE JIT_FUSE=0 / 1, alternating.
set -o pipefail
O=gpurun_out/${1:-r5f}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_root" -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_fused.log 2>&1
rc=$?; tail -6 $O/pytest_fused.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/pytest_fused.log | head -30; exit $rc; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multi.py tests/test_gpu_underflow.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/pytest.log | head -30; exit $rc; }
for i in 1 2; do
  for v in 0 1; do
    PLK_TUNE=JIT_FUSE=$v timeout -k 10 300 python bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong > $O/cfg5_fuse${v}_$i.json 2> $O/cfg5_fuse${v}_$i.err || exit $?
    PLK_TUNE=JIT_FUSE=$v timeout -k 10 300 python bench.py --scaling strong --no-cpu-baseline --steps 10 > $O/cfg5s_fuse${v}_$i.json 2> $O/cfg5s_fuse${v}_$i.err || exit $?
  done
done
python - <<PY
import json
for v in ("0", "1"):
    for i in (1, 2):
        r = json.load(open(f"$O/cfg5_fuse{v}_{i}.json")); s = json.load(open(f"$O/cfg5s_fuse{v}_{i}.json"))
        print("fuse", v, i, "250k %.4f trav %.4f frac %.3f" % (r["ms_per_step"], r["roofline"]["traversal_ms"], r["roofline"]["frac"]),
              "| 2M %.4f trav %.4f" % (s["ms_per_step"], s["roofline"]["traversal_ms"]), r["lnl"], s["lnl"])
PY
