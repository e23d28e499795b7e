#!/bin/bash
set -o pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_host.py tests/test_gpu_configs.py -k "pmat or request or nh or host or drop or config" > gpurun_out/sh_tests.log 2>&1; rc=$?
tail -2 gpurun_out/sh_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/sh_tests.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong > gpurun_out/sh5.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sh5.json')); print('cfg5', round(d['ms_per_step'],4), d['host_us_per_eval'], d['lnl'])"
done
