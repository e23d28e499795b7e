#!/bin/bash
set -o pipefail
for r in 64 256 128; do
  for c in "lg08_g4_protein_200k_256" "yn98_codon_50k_128"; do
    PLK_TUNE=CHERRY_ROWS=$r timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-strong > gpurun_out/rw.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/rw.json')); print('$r $c', round(d['ms_per_step'],4), round(d['kernel_ms_per_step']['tables']*1000,1), d['lnl'])"
  done
done
