#!/bin/bash
# Round-3 session F: tests of the packed unit descriptors (jit_tree4) and the DR defaults, the
# launch fixed-cost sweep again, and the default bench line.
#   tools/gpu_r3f.sh <tag>
set -o pipefail
T=${1:-r3f}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  -k "jit_tree4_bitwise or test_bench_mode or dr_" > gpurun_out/$T/focus.log 2>&1 || { echo "focus failed"; tail -30 gpurun_out/$T/focus.log; exit 1; }
tail -1 gpurun_out/$T/focus.log
bash tools/gpu_sweep.sh $T/sweep gtr_g4_dna_1M_64 "4096 65536 262144 1000000" "base:" || exit 1
bash tools/ab_bench.sh $T/cfg5 nh_gtr_g4_dna_2M_512 "base:" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || { tail -5 gpurun_out/$T/bench_default.err; exit 1; }
cat gpurun_out/$T/bench_default.json
