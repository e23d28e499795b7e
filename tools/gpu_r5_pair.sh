#!/bin/bash
# cfg2 / cfg5 cherry pair-table LDS budget at the 200-step window (alternating)
set -o pipefail
O=gpurun_out/r5pair
mkdir -p $O
for v in "JIT_PAIR_KB=64" "JIT_PAIR_KB=48" "JIT_PAIR_KB=80" "JIT_PAIR_KB=64" "JIT_PAIR_KB=48" "JIT_PAIR_KB=80"; do
  PLK_TUNE=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-strong > $O/l.json 2> $O/l.err || { tail -5 $O/l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/l.json'));print('cfg2 [$v]', round(d['ms_per_step'],5), round(d['roofline']['frac'],3))"
done
for v in "JIT_PAIR_KB=64" "JIT_PAIR_KB=48" "JIT_PAIR_KB=80" "JIT_PAIR_KB=64" "JIT_PAIR_KB=48" "JIT_PAIR_KB=80"; do
  PLK_TUNE=$v timeout -k 10 200 python3 bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong > $O/l.json 2> $O/l.err || { tail -5 $O/l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/l.json'));print('cfg5 [$v]', round(d['ms_per_step'],5), round(d['roofline']['frac'],3))"
done
