#!/bin/bash
# A/B bench lines of one config under libplk tuning variants (PLK_TUNE keys):
#   tools/ab_bench.sh <tag> <config> "<name>:<KEY=v,KEY=v>" ...   ("base:" = defaults)
# Each variant: gpurun_out/<tag>/<name>.json (bench line, no CPU baseline); a summary line each.
set -o pipefail
T=$1; CFG=$2; shift 2
mkdir -p gpurun_out/$T
for v in "$@"; do
  n=${v%%:*}; e=${v#*:}
  PLK_TUNE="$e" timeout -k 10 200 python bench.py --config $CFG --no-cpu-baseline --steps 10 --warmup 2 \
    > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || { echo "$n failed"; tail -5 gpurun_out/$T/$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$T/$n.json'));r=d['roofline'];print('$n',d['kernel_path'],round(r['traversal_ms'],4),round(r['frac'],3),'ms/step',round(d['ms_per_step'],4))"
done
