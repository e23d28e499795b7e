#!/bin/bash
# cfg2: operand lookahead 3 (default) vs 2, alternating pairs at the 200-step window
set -o pipefail
O=gpurun_out/r5l2
mkdir -p $O
for i in 1 2 3 4 5 6; do
  for v in "JIT_L=3" "JIT_L=2"; do
    PLK_TUNE=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-strong > $O/l.json 2> $O/l.err || { tail -5 $O/l.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/l.json'));print('cfg2 [$v]', round(d['ms_per_step'],5), round(d['roofline']['frac'],3), round(d['roofline']['traversal_ms']*1000,1))"
  done
done
