#!/bin/bash
# A/B sweep of env settings on one bench config:
#   tools/gpu_sweep_env.sh <tag> <config> "<name>:<VAR=v,VAR=v>" ...   (use "base:" for defaults)
set -o pipefail
TAG=$1; CFG=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$name.json')); print('$name', '%.4e' % d['value'], 'kernel_ms %.4f' % d['kernel_ms_per_step']['partials'], 'part/s %.4e' % d['partials_only_updates_per_s'])"
done
