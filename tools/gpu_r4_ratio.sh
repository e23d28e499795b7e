#!/bin/bash
# cfg5 2 M / 250 k step ratio, three alternating pairs
set -o pipefail
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong > gpurun_out/ra_250k_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --config nh_gtr_g4_dna_2M_512 --scaling strong --no-cpu-baseline --steps 20 > gpurun_out/ra_2M_$i.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('gpurun_out/ra_250k_$i.json'))['ms_per_step']; b=json.load(open('gpurun_out/ra_2M_$i.json'))['ms_per_step']; print('pair $i', round(a,4), round(b,4), round(b/a,3))"
done
