#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pmat64 or pmatrix_kernel or yn98 or treeM" > gpurun_out/p64_tests.log 2>&1; rc=$?
tail -2 gpurun_out/p64_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config yn98_codon_50k_128 --no-cpu-baseline --no-strong > gpurun_out/p64.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/p64.json')); print(round(d['ms_per_step'],4), d['kernel_ms_per_step'], d['roofline']['frac'], d['lnl'])"
bash tools/gpu_r4_cfg4.sh | head -6
