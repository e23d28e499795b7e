#!/bin/bash
# cfg5 shape A/B with dynamic super-blocks: JIT_G / JIT_L
set -o pipefail
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --config nh_gtr_g4_dna_2M_512 "$@" > gpurun_out/g_$tag.json 2> gpurun_out/g_$tag.err || { tail -3 gpurun_out/g_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/g_$tag.json')); print('$tag', round(d['ms_per_step'],4), round(d['kernel_ms_per_step']['partials'],4), d['lnl'])"; }
for t in "" "JIT_G=4" "JIT_L=3" "JIT_G=6" ""; do
  export PLK_TUNE=$t
  run "250k_$t" --no-strong
  run "2M_$t" --scaling strong --steps 10
done
