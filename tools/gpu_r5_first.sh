#!/bin/bash
# Round 5, first GPU session: the L2 stale-line micro test (round-4 -inf shard hypothesis), the
# whole -m gpu suite with a fresh JIT cache (new cache key), the default bench line and the
# eight-shard one-process rehearsal (fan-out timestamps).
set -o pipefail
O=gpurun_out/${1:-r5a}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
mkdir -p $PLK_JIT_CACHE
timeout -k 10 120 tools/micro/l2_stale > $O/l2_stale.txt 2>&1 || { echo "l2_stale rc=$?"; exit 1; }
cat $O/l2_stale.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
cat $O/bench_default.json | head -c 600; echo
timeout -k 10 300 python bench.py --gpus 8 --devices 0,0,0,0,0,0,0,0 --no-cpu-baseline --steps 20 > $O/bench_dev8.json 2> $O/bench_dev8.err || exit $?
python -c "import json;r=json.load(open('$O/bench_dev8.json'));print(r['ms_per_step'],json.dumps(r.get('fanout')));print(r['strong']['ms_per_step'],json.dumps(r['strong'].get('fanout')))"
