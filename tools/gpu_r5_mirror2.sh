#!/bin/bash
# default line (strong sub-record at 40 steps) and the Bio++ mirror's cfg2 line at 200 steps
set -o pipefail
O=gpurun_out/r5m2
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));s=d.get('strong',{});print('default', round(d['ms_per_step'],5), round(d['roofline']['frac'],3), 'strong', s.get('ms_per_step'), s.get('traversal_frac_fp64'))"
for i in 1 2; do
  timeout -k 10 300 bpp-phyl_amd/host/bin/bench_mirror cfg2 > $O/mirror_cfg2_$i.json || exit $?
  cat $O/mirror_cfg2_$i.json
done
