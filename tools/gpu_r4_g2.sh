#!/bin/bash
# cfg2 JIT_G / JIT_L A/B under dynamic super-blocks
set -o pipefail
run() { tag=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --no-strong "$@" > gpurun_out/g2_$tag.json 2> gpurun_out/g2_$tag.err || { tail -3 gpurun_out/g2_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/g2_$tag.json')); print('$tag', round(d['ms_per_step'],4), round(d['kernel_ms_per_step']['partials'],4), d['lnl'])"; }
for i in 1 2; do
for t in "" "JIT_G=2" "JIT_G=4" "JIT_L=2" "JIT_L=4"; do
  PLK_TUNE=$t run "cfg2_$t"
done; done
