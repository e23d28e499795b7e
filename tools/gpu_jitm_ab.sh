#!/bin/bash
# jit_treeM issue-order / operand-fetch A/B on one GPU: the bitwise test of the variants,
# the oracle tests of jit_treeM, then cfg3 bench lines per variant and a stall pass.
#   tools/gpu_jitm_ab.sh <tag>
set -o pipefail
T=${1:-jm}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "treeM or jitm or issue_orders" \
  > gpurun_out/$T/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
bash tools/ab_bench.sh $T lg08_g4_protein_200k_256 "base:" "p0l0:JITM_PIPE=0,JITM_LC=0" "p1l0:JITM_LC=0" "p0l3:JITM_PIPE=0" \
  "p2:JITM_PIPE=2" "lc5:JITM_LC=5" "dm3:JITM_DM=3" "w3dm3:JITM_DM=3,JITM_MINW=3" || exit 1
bash tools/gpu_stalls.sh ${T}_cfg3 lg08_g4_protein_200k_256 || exit 1
