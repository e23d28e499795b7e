#!/bin/bash
# Dynamic super-blocks: parity tests, then A/B lines (PLK_TUNE JIT_DYN=0 / default) and timestamps
set -o pipefail
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py -k "tree4 or jit or config or full_size" > gpurun_out/dyn_tests.log 2>&1; rc=$?
[ -n "$NOTEST" ] || { tail -3 gpurun_out/dyn_tests.log; [ $rc -eq 0 ] || exit $rc; }
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/d_$tag.json 2> gpurun_out/d_$tag.err || { tail -3 gpurun_out/d_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/d_$tag.json')); print('$tag', round(d['ms_per_step'],4), round(d['kernel_ms_per_step']['partials'],4), d['lnl'])"; }
for v in 0 1 0 1; do
  export PLK_TUNE=JIT_DYN=$v
  run cfg2_$v --no-strong
  run cfg5_$v --config nh_gtr_g4_dna_2M_512 --no-strong
  run cfg5s_$v --config nh_gtr_g4_dna_2M_512 --scaling strong --steps 10
done
unset PLK_TUNE
export PLK_DEBUG_TIMES=1
for a in "--config nh_gtr_g4_dna_2M_512" "--config nh_gtr_g4_dna_2M_512 --patterns 2000000" ""; do
  echo "=== $a"
  timeout -k 10 120 python bench.py $a --no-cpu-baseline --no-strong --steps 4 --warmup 3 2>&1 >/dev/null | grep -A 8 "plk times" || exit 1
done
