#!/bin/bash
# cfg2 / cfg5 generated-kernel shapes at the 200-step window (alternating)
set -o pipefail
O=gpurun_out/r5gl
mkdir -p $O
for v in "" "JIT_L=2" "JIT_L=4" "JIT_G=2" "JIT_G=4" "" "JIT_L=2" "JIT_L=4"; do
  PLK_TUNE=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-strong > $O/l.json 2> $O/l.err || { tail -5 $O/l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/l.json'));print('cfg2 [$v]', round(d['ms_per_step'],5), round(d['roofline']['frac'],3))"
done
for v in "" "JIT_L=3" "JIT_G=6" "" "JIT_L=3"; do
  PLK_TUNE=$v timeout -k 10 200 python3 bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong > $O/l.json 2> $O/l.err || { tail -5 $O/l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/l.json'));print('cfg5 [$v]', round(d['ms_per_step'],5), round(d['roofline']['frac'],3))"
done
