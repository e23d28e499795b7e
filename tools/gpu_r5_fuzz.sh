#!/bin/bash
# Round 5: the random-topology tests against the oracle (tests/test_gpu_parity.py).
set -o pipefail
O=gpurun_out/${1:-r5fuzz}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dr.py -k "random_topologies or subtree or polytomy" -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -20; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest.log | head -30; exit $rc; }
