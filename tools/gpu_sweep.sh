#!/bin/bash
# Env-variant sweep of bench.py lines: tools/gpu_sweep.sh <tag> <config> "<VAR=v ...>" ["<VAR=v ...>" ...]
set -o pipefail
TAG=$1; CFG=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
i=0
for variant in "$@"; do
  i=$((i+1))
  env $variant timeout -k 10 240 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline > $O/v$i.json 2> $O/v$i.err || { echo "variant $variant failed"; tail -5 $O/v$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/v$i.json')); print('$variant |', '%.3e' % d['value'], 'part %.3e' % d['partials_only_updates_per_s'], round(d['kernel_ms_per_step']['partials'],3), d['partials_launches_per_step'])"
done
