#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-dr2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dr.py -x -v --timeout 120 --timeout-method thread > $O/pytest_dr.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_dr.log; exit 1; }
tail -2 $O/pytest_dr.log
for cfg in lg08_g4_protein_200k_256 yn98_codon_50k_128; do
for v in 1 0; do
PLK_DR_MFMA=$v timeout -k 10 200 python tools/bench_dr.py --config $cfg --path-branches 8 > $O/dr_${cfg}_$v.json 2> $O/dr_${cfg}_$v.err || { tail -5 $O/dr_${cfg}_$v.err; exit 1; }
python -c "import json; d=json.load(open('$O/dr_${cfg}_$v.json')); print('$cfg mfma=$v', 'dr_ms %.2f' % d['dr_ms'], 'red_ms %.2f' % d['reduction_kernel_ms'], 'speedup %.1f' % d['speedup_dr_vs_path'], 'maxrel %.1e' % d['max_rel_diff_dr_vs_path'])"
done
done
