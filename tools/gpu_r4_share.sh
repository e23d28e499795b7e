#!/bin/bash
# shape-shared fragment code: jit tests (fresh cache), cfg5 / cfg2 lines, compile times
set -o pipefail
export PLK_JIT_CACHE=$PWD/gpurun_out/jc_share; rm -rf $PLK_JIT_CACHE; mkdir -p $PLK_JIT_CACHE
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "jit_tree4 or nh_gtr or full_size or dynamic or gtr_g4" > gpurun_out/share_tests.log 2>&1; rc=$?
tail -2 gpurun_out/share_tests.log; [ $rc -eq 0 ] || { grep -E "Error|error|FAIL" gpurun_out/share_tests.log | head -20; exit $rc; }
rm -rf $PLK_JIT_CACHE/*
for c in nh_gtr_g4_dna_2M_512 gtr_g4_dna_1M_64; do
  S=$(date +%s%N)
  PLK_JIT_LOG=1 timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-strong > gpurun_out/sh_$c.json 2> gpurun_out/sh_$c.err || { tail -3 gpurun_out/sh_$c.err; exit 1; }
  grep "jit compiled" gpurun_out/sh_$c.err
  python -c "import json; d=json.load(open('gpurun_out/sh_$c.json')); print('$c', round(d['ms_per_step'],4), round(d['kernel_ms_per_step']['partials'],4), d['lnl'], d['setup_s'])"
done
timeout -k 10 200 python bench.py --config nh_gtr_g4_dna_2M_512 --scaling strong --no-cpu-baseline --steps 10 > gpurun_out/sh_5s.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/sh_5s.json')); print('5s', round(d['ms_per_step'],4), d['lnl'])"
