#!/bin/bash
# round 6: stall passes of cfg2's traversal (default shape), digested
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6stalls2
PLK_TUNE="$TUNE" bash tools/gpu_stalls.sh r6_${NAME:-def} gtr_g4_dna_1M_64 > /dev/null || exit 1
python tools/stalls_digest.py gpurun_out/stalls/r6_${NAME:-def} --json gpurun_out/r6stalls2/cfg2_${NAME:-def}_stalls.json > /dev/null || exit 1
rm -rf gpurun_out/stalls/r6_${NAME:-def}
python -c "
import json; d=json.load(open('gpurun_out/r6stalls2/cfg2_${NAME:-def}_stalls.json'))
print({k: round(x,3) for k,x in d['frac_of_wave_cycles'].items()}); t=d['totals']; print({k: '%.3g'%v for k,v in t.items()})"
