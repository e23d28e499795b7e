#!/bin/bash
# First-super-block penalty: timestamps with the first super-block run twice, and with the
# fragment's P(t) range touched during staging (debug switches, wrong results for TWICE)
set -o pipefail
export PLK_DEBUG_TIMES=1
t() { echo "=== $1"; shift; timeout -k 10 120 python bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong --steps 4 --warmup 3 "$@" 2>&1 >/dev/null | grep -A 8 "plk times tier0" || exit 1; }
PLK_TUNE=JIT_DYN=0 t base
PLK_TUNE=JIT_DYN=0 PLK_DEBUG_TWICE=1 t twice
PLK_TUNE=JIT_DYN=0 PLK_DEBUG_PTOUCH=1 t ptouch
PLK_TUNE=JIT_DYN=0 PLK_DEBUG_PTOUCH=1 PLK_DEBUG_TWICE=1 t ptouch_twice
unset PLK_DEBUG_TIMES
for i in 1 2; do
for v in "" 1; do
  if [ -n "$v" ]; then export PLK_DEBUG_PTOUCH=1; else unset PLK_DEBUG_PTOUCH; fi
  timeout -k 10 200 python bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong > gpurun_out/pt.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pt.json')); print('ptouch=$v', round(d['ms_per_step'],4), round(d['kernel_ms_per_step']['partials'],4), d['lnl'])"
done; done
