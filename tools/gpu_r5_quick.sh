#!/bin/bash
# Round 5 quick check: the jit_tree4 / multi-device / config tests, then the default line.
set -o pipefail
O=gpurun_out/${1:-r5b}
mkdir -p $O
shift
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
mkdir -p $PLK_JIT_CACHE
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python -c "
import json;r=json.load(open('$O/bench_default.json'))
print(r['ms_per_step'], r['roofline']['traversal_ms'], r['roofline']['frac'], r['host_us_per_eval'])
print('strong', r['strong']['ms_per_step'], r['strong']['traversal_ms'])"
