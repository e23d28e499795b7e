#!/bin/bash
# staging A/B: jit tests, lines and timestamps
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "jit_tree4" > gpurun_out/st_tests.log 2>&1; rc=$?
tail -3 gpurun_out/st_tests.log; [ $rc -eq 0 ] || exit $rc
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/s_$tag.json 2> gpurun_out/s_$tag.err || { tail -3 gpurun_out/s_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s_$tag.json')); print('$tag', round(d['ms_per_step'],4), round(d['kernel_ms_per_step']['partials'],4), d['lnl'])"; }
for i in 1 2; do
  run cfg2 --no-strong
  run cfg5 --config nh_gtr_g4_dna_2M_512 --no-strong
  run cfg5s --config nh_gtr_g4_dna_2M_512 --scaling strong --steps 10
done
export PLK_DEBUG_TIMES=1
for a in "--config nh_gtr_g4_dna_2M_512" ""; do
  echo "=== $a"
  timeout -k 10 120 python bench.py $a --no-cpu-baseline --no-strong --steps 4 --warmup 3 2>&1 >/dev/null | grep -A 8 "plk times" || exit 1
done
