#!/bin/bash
# pmat4_kernel duration in the cfg2 / cfg5 timelines + P(t) tests
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pmat or pmatrix or bitwise" > gpurun_out/pm4_tests.log 2>&1; rc=$?
tail -2 gpurun_out/pm4_tests.log; [ $rc -eq 0 ] || exit $rc
R=$(pwd); export TMPDIR=/tmp
for c in gtr_g4_dna_1M_64 nh_gtr_g4_dna_2M_512; do
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pm4/$c -o run -- \
    python3 $R/bench.py --config $c --no-cpu-baseline --no-strong --steps 10 > $R/gpurun_out/pm4_$c.json 2> $R/gpurun_out/pm4_$c.err ) || exit 1
  python3 tools/trace_summary.py gpurun_out/pm4/$c/run_kernel_trace.csv 8 | grep -E "pmat|blocks" ; rm -rf gpurun_out/pm4/$c
  python -c "import json; d=json.load(open('gpurun_out/pm4_$c.json')); print('$c', round(d['ms_per_step'],4), d['lnl'])"
done
