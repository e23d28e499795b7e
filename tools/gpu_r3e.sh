#!/bin/bash
# Round-3 session E: focused tests of the padded LDS table rows (JIT_RS) and the jit_treeM
# issue-order default, A/B lines of both, then the DR pass A/B (tools/gpu_dr_ab.sh).
#   tools/gpu_r3e.sh <tag>
set -o pipefail
T=${1:-r3e}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  -k "jit_tree4_bitwise or issue_orders or test_bench_mode_vs_oracle" > gpurun_out/$T/focus.log 2>&1 || { echo "focus failed"; tail -30 gpurun_out/$T/focus.log; exit 1; }
tail -1 gpurun_out/$T/focus.log
bash tools/ab_bench.sh $T/cfg5 nh_gtr_g4_dna_2M_512 "rs6:" "rs4:JIT_RS=4" "rs6b:" || exit 1
bash tools/ab_bench.sh $T/cfg2 gtr_g4_dna_1M_64 "rs4:" "rs6:JIT_RS=6" || exit 1
bash tools/ab_bench.sh $T/cfg3 lg08_g4_protein_200k_256 "p2:" "p1:JITM_PIPE=1" "p2b:" || exit 1
bash tools/gpu_stalls.sh ${T}_cfg5 nh_gtr_g4_dna_2M_512 || exit 1
bash tools/gpu_dr_ab.sh ${T}_dr || exit 1
