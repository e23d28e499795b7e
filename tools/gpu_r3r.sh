#!/bin/bash
# Round-3 session R: the last tier of jit_tree4 as its own kernel (JIT_TOP): bitwise tests,
# cfg5 A/B (250 k and 2 M patterns) with its lookahead, the cfg2 line (one tier: unchanged).
set -o pipefail
T=${1:-r3r}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  -k "jit_tree4_bitwise or test_bench_mode_vs_oracle or multi_device_handle" > gpurun_out/$T/focus.log 2>&1 || { echo "focus failed"; tail -30 gpurun_out/$T/focus.log; exit 1; }
tail -1 gpurun_out/$T/focus.log
bash tools/ab_bench.sh $T/cfg5 nh_gtr_g4_dna_2M_512 "top:" "one:JIT_TOP=0" "topl3:JIT_TOP_L=3" "topl4:JIT_TOP_L=4" "top2:" "one2:JIT_TOP=0" || exit 1
for v in "top:" "one:JIT_TOP=0"; do
  n=${v%%:*}; e=${v#*:}
  PLK_TUNE="$e" timeout -k 10 300 python bench.py --scaling strong --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/$T/strong_$n.json 2> gpurun_out/$T/strong_$n.err || { tail -5 gpurun_out/$T/strong_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$T/strong_$n.json'));r=d['roofline'];print('strong $n',round(r['traversal_ms'],4),round(r['frac'],3),'ms/step',round(d['ms_per_step'],4))"
done
