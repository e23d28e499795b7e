#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-spin}; mkdir -p $O
for i in 1 2; do
for v in 0 1; do
  PLK_SPIN=$v timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/spin$v.json 2> $O/spin$v.err || { tail -5 $O/spin$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/spin$v.json')); print('spin$v', '%.4e' % d['value'], 'ms_step %.4f' % d['ms_per_step'], 'kernel_ms %.4f' % d['kernel_ms_per_step']['partials'])"
done
done
PLK_SPIN=0 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-events > $O/noev.json 2> $O/noev.err && python -c "import json; d=json.load(open('$O/noev.json')); print('noevents', '%.4e' % d['value'], 'ms_step %.4f' % d['ms_per_step'])"
