#!/bin/bash
# Round-3 session C: the focused tests of this session's changes, the whole -m gpu suite,
# then A/B lines (host-formed block sums, swizzled LDS table rows) and a cfg5 stall pass.
#   tools/gpu_r3c.sh <tag>
set -o pipefail
T=${1:-r3c}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  -k "host_block_sums or treeM_register_depths or issue_orders" > gpurun_out/$T/focus.log 2>&1 || { echo "focus failed"; tail -30 gpurun_out/$T/focus.log; exit 1; }
tail -1 gpurun_out/$T/focus.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/$T/all.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/$T/all.log; exit 1; }
tail -1 gpurun_out/$T/all.log
bash tools/ab_bench.sh $T/cfg2 gtr_g4_dna_1M_64 "base:" "hb:HOST_BLOCKS=1" "noswz:JIT_SWZ=0" "base2:" "hb2:HOST_BLOCKS=1" || exit 1
bash tools/ab_bench.sh $T/cfg5 nh_gtr_g4_dna_2M_512 "base:" "noswz:JIT_SWZ=0" "hb:HOST_BLOCKS=1" || exit 1
bash tools/gpu_stalls.sh ${T}_cfg5 nh_gtr_g4_dna_2M_512 || exit 1
timeout -k 10 150 bpp-phyl_amd/host/bin/bench_mirror cfg2 > gpurun_out/$T/mirror_cfg2.json && cat gpurun_out/$T/mirror_cfg2.json
