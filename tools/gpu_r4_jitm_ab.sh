#!/bin/bash
# cfg3 jit_treeM shapes with shared fragment code
set -o pipefail
for t in "" "JITM_L=2" "JITM_DM=5" "JITM_DM=3" ""; do
  PLK_TUNE=$t timeout -k 10 300 python bench.py --config lg08_g4_protein_200k_256 --no-cpu-baseline --no-strong > gpurun_out/jm.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/jm.json')); print('$t', round(d['ms_per_step'],4), round(d['roofline']['frac'],3), d['lnl'])"
done
