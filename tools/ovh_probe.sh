#!/bin/bash
# Fixed per-evaluation costs of the default bench path: ms per step and the host-side
# segments of plk_evaluate (bench line host_us_per_eval) at 1M and 4096 patterns.
#   [CFG=<config>] [SIZES="1000000 4096"] tools/ovh_probe.sh <tag> [ENV=VAL ...]
set -o pipefail
T=${1:-ovh}; shift
mkdir -p gpurun_out
for P in ${SIZES:-1000000 4096}; do
  env "$@" timeout -k 10 120 python bench.py --config ${CFG:-gtr_g4_dna_1M_64} --no-cpu-baseline --steps 200 --warmup 20 --patterns $P > gpurun_out/${T}_${P}.json 2>gpurun_out/${T}_${P}.err || { tail -5 gpurun_out/${T}_${P}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_${P}.json'));print('$T',$P,round(d['ms_per_step'],4),round(d['kernel_ms_per_step']['partials'],4),d['host_us_per_eval'])"
done
