#!/bin/bash
# one generated module per tier vs one for all tiers (PLK_DEBUG_ONEMOD): jit tests, cfg5 lines, module register counts
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "jit_tree4 or nh_gtr or full_size or dynamic" > gpurun_out/tm_tests.log 2>&1; rc=$?
tail -2 gpurun_out/tm_tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/t_$tag.json 2> gpurun_out/t_$tag.err || { tail -3 gpurun_out/t_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/t_$tag.json')); print('$tag', round(d['ms_per_step'],4), round(d['kernel_ms_per_step']['partials'],4), d['lnl'])"; }
for i in 1 2; do
  PLK_DEBUG_ONEMOD=1 run one5 --config nh_gtr_g4_dna_2M_512 --no-strong
  run tier5 --config nh_gtr_g4_dna_2M_512 --no-strong
  PLK_DEBUG_ONEMOD=1 run one5s --config nh_gtr_g4_dna_2M_512 --scaling strong --steps 10
  run tier5s --config nh_gtr_g4_dna_2M_512 --scaling strong --steps 10
done
PLK_JIT_CACHE=$PWD/gpurun_out/jitc2 timeout -k 10 120 python bench.py --config nh_gtr_g4_dna_2M_512 --patterns 4096 --no-cpu-baseline --no-strong --steps 2 > /dev/null 2>&1 || exit 1
