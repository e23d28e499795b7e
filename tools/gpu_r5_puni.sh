#!/bin/bash
# pmat4_kernel with the request's single model known up front (default) vs through the
# entries (PLK_TUNE PUNI=0): cfg2 under the kernel trace, then alternating bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5puni
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "PUNI=0" "PUNI=1" "PUNI=0" "PUNI=1"; do
  tag=$(echo $v | tr ',=' '__')_$RANDOM
  PLK_TUNE=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-strong --steps 50 --warmup 5 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  s=$(find $O/$tag -name "run_kernel_stats.csv" | head -1)
  python3 - $s "$v" $O/$tag.json <<'PY'
import csv,sys,json
d=json.load(open(sys.argv[3]))
for r in csv.DictReader(open(sys.argv[1])):
    if 'pmat4' in r['Name'] or 'jit_tree4' in r['Name'] or 'wave_sums' in r['Name']:
        print(sys.argv[2], r['Name'][:24], r['Calls'], round(float(r['AverageNs'])/1000,2), round(float(r['MinNs'])/1000,2), 'step', round(d['ms_per_step'],4))
PY
  rm -f $O/$tag/*/*trace.csv
done
for v in "PUNI=0" "PUNI=1" "PUNI=0" "PUNI=1" "PUNI=0" "PUNI=1"; do
  PLK_TUNE=$v timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-strong --steps 200 --warmup 20 > $O/line.json 2> $O/line.err || { tail -5 $O/line.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/line.json'));print('$v', 'line ms/step', round(d['ms_per_step'],5), d.get('host_us_per_eval'))"
done
