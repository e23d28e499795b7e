#!/bin/bash
# Round-4 DR pass per configuration (default path), checked against the path derivatives
set -o pipefail
mkdir -p gpurun_out/r4dr
for c in gtr_g4_dna_1M_64 lg08_g4_protein_200k_256 yn98_codon_50k_128 nh_gtr_g4_dna_2M_512; do
  timeout -k 10 300 python tools/bench_dr.py --config $c --reps 3 --path-branches 4 > gpurun_out/r4dr/$c.json 2> gpurun_out/r4dr/$c.err || { tail -5 gpurun_out/r4dr/$c.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/r4dr/$c.json')); print('$c', round(d['dr_ms'],3), 'ms', d.get('dr_path'), 'maxrel', d['max_rel_diff_dr_vs_path'])"
done
