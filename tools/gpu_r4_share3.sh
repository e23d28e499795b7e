#!/bin/bash
# shape-shared jit_treeM fragments: tests (fresh cache), cfg3 line + compile time
set -o pipefail
export PLK_JIT_CACHE=$PWD/gpurun_out/jc_share3_$$; rm -rf $PLK_JIT_CACHE; mkdir -p $PLK_JIT_CACHE
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multi.py -k "jitm or treeM or lg08 or jit_treeM or s20 or cherry" > gpurun_out/share3_tests.log 2>&1; rc=$?
tail -2 gpurun_out/share3_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|FAIL" gpurun_out/share3_tests.log | head -20; exit $rc; }
rm -rf $PLK_JIT_CACHE/*
PLK_JIT_LOG=1 timeout -k 10 300 python bench.py --config lg08_g4_protein_200k_256 --no-cpu-baseline --no-strong > gpurun_out/sh3.json 2> gpurun_out/sh3.err || { tail -3 gpurun_out/sh3.err; exit 1; }
grep "jit compiled" gpurun_out/sh3.err
python -c "import json; d=json.load(open('gpurun_out/sh3.json')); print('cfg3', round(d['ms_per_step'],4), d['kernel_ms_per_step'], d['lnl'], d['setup_s'])"
