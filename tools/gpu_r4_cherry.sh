#!/bin/bash
# cherry tables over the occurring code pairs: treeM / jit_treeM / config tests, cfg3 + cfg4 lines, cfg4 trace
set -o pipefail
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "treeM or cherry or jitm or lg08 or yn98 or pmat64" > gpurun_out/ch_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ch_tests.log; [ $rc -eq 0 ] || exit $rc
for c in "lg08_g4_protein_200k_256" "yn98_codon_50k_128"; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-strong > gpurun_out/ch_$c.json 2> gpurun_out/ch_$c.err || { tail -3 gpurun_out/ch_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ch_$c.json')); print('$c', round(d['ms_per_step'],4), d['kernel_ms_per_step'], d['roofline']['frac'], d['lnl'])"
done
bash tools/gpu_r4_cfg4.sh
