#!/bin/bash
# Round 5: underflow flag tests, the Bio++ mirror's C++ GPU tests (unscaled first with the exact
# fallback) and the mirror's cfg2 line.
set -o pipefail
O=gpurun_out/${1:-r5m}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
timeout -k 10 600 python -u -m pytest tests/test_gpu_underflow.py tests/test_gpu_host.py tests/test_gpu_multi.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bpp-phyl_amd/host/bin/test_likelihood_gpu > $O/test_likelihood_gpu.txt 2>&1 || { echo rc=$?; tail -20 $O/test_likelihood_gpu.txt; exit 1; }
grep -E "taxa|PASS|FAIL" $O/test_likelihood_gpu.txt
for i in 1 2; do
  timeout -k 10 300 bpp-phyl_amd/host/bin/bench_mirror cfg2 > $O/mirror_cfg2_$i.json || exit $?
  cat $O/mirror_cfg2_$i.json
done
