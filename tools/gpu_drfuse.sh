#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-drf}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dr.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0; do
PLK_DR_FUSE=$v timeout -k 10 200 python tools/bench_dr.py --config gtr_g4_dna_1M_64 --path-branches 16 > $O/dr_fuse$v.json 2> $O/dr_fuse$v.err || { tail -5 $O/dr_fuse$v.err; exit 1; }
python -c "import json; d=json.load(open('$O/dr_fuse$v.json')); print('fuse=$v', 'dr_ms %.2f' % d['dr_ms'], 'red_ms %.2f' % d['reduction_kernel_ms'], 'speedup %.2f' % d['speedup_dr_vs_path'], 'maxrel %.1e' % d['max_rel_diff_dr_vs_path'])"
done
