#!/bin/bash
# Row f4 at the round's close: all-branch derivatives per configuration (default DR path)
set -o pipefail
O=gpurun_out/r5dr
mkdir -p $O
for c in gtr_g4_dna_1M_64 lg08_g4_protein_200k_256 yn98_codon_50k_128 nh_gtr_g4_dna_2M_512; do
  timeout -k 10 300 python tools/bench_dr.py --config $c --reps 5 --path-branches 4 > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
  python3 -c "
import json
d=json.load(open('$O/$c.json')); print('$c', round(d['dr_ms'],3), 'ms', d.get('dr_path'), 'vs path x', round(d.get('speedup_vs_path', 0) or 0, 2) if 'speedup_vs_path' in d else '', 'maxrel', d['max_rel_diff_dr_vs_path'])"
done
