#!/bin/bash
# Fixed cost of a traversal launch: bench lines of one config over pattern counts, for the
# defaults and optional PLK_TUNE variants; one summary line per run (traversal ms from HIP
# events, step ms).
#   tools/gpu_sweep.sh <tag> <config> "<patterns ...>" "<name>:<KEY=v,...>" ...
set -o pipefail
T=$1; CFG=$2; PS=$3; shift 3
mkdir -p gpurun_out/$T
for v in "$@"; do
  n=${v%%:*}; e=${v#*:}
  for P in $PS; do
    PLK_TUNE="$e" timeout -k 10 200 python bench.py --config $CFG --patterns $P --no-cpu-baseline --steps 20 --warmup 3 \
      > gpurun_out/$T/${n}_$P.json 2> gpurun_out/$T/${n}_$P.err || { echo "$n $P failed"; tail -5 gpurun_out/$T/${n}_$P.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/$T/${n}_$P.json'));r=d['roofline'];print('$n',$P,d['kernel_path'],round(r['traversal_ms']*1e3,2),'us traversal',round(d['ms_per_step']*1e3,2),'us/step')"
  done
done
