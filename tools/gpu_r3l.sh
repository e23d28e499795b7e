#!/bin/bash
# Round-3 session L: tests of the workgroup-wide staging of rescaling contribution units
# (jit_tree4), cfg5 lines, then the round's part-2 profiles (tools/gpu_round3.sh <tag> 2).
#   tools/gpu_r3l.sh <tag>
set -o pipefail
T=${1:-r3z}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  -k "jit_tree4_bitwise or test_bench_mode_vs_oracle" > gpurun_out/$T/focus_l.log 2>&1 || { echo "focus failed"; tail -30 gpurun_out/$T/focus_l.log; exit 1; }
tail -1 gpurun_out/$T/focus_l.log
bash tools/ab_bench.sh $T/cfg5 nh_gtr_g4_dna_2M_512 "a:" "b:" || exit 1
bash tools/gpu_round3.sh $T 2
