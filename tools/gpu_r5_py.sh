#!/bin/bash
set -o pipefail
O=gpurun_out/r5py
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_underflow.py -k "evaluate or multi or underflow or fanout" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/pytest.log | head -30; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-strong > $O/c2_$i.json 2> $O/c2_$i.err || exit $?
  python -c "import json;d=json.load(open('$O/c2_$i.json'));print($i, round(d['ms_per_step'],4), d['host_us_per_eval'])"
done
