#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-drm}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dr.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in lg08_g4_protein_200k_256 yn98_codon_50k_128; do
timeout -k 10 200 python tools/bench_dr.py --config $cfg --path-branches 8 > $O/dr_$cfg.json 2> $O/dr_$cfg.err || { tail -5 $O/dr_$cfg.err; exit 1; }
python -c "import json; d=json.load(open('$O/dr_$cfg.json')); print('$cfg', 'dr_ms %.2f' % d['dr_ms'], 'red_ms %.2f' % d['reduction_kernel_ms'], 'speedup %.2f' % d['speedup_dr_vs_path'], 'maxrel %.1e' % d['max_rel_diff_dr_vs_path'])"
done
