#!/bin/bash
set -o pipefail
O=gpurun_out/r5pm4
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -k "pmat or evaluate or churn or multi_device or jit_tree4_bitwise" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/pytest.log | head -30; exit $rc; }
bash tools/gpu_r5_ab.sh r5pm4/ab ab/libplk_head.so || exit $?
bash tools/gpu_r5_ab.sh r5pm4/ab5 ab/libplk_head.so --config nh_gtr_g4_dna_2M_512 --no-strong || exit $?
