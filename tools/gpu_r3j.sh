#!/bin/bash
# Round-3 session J: volatile LDS A-operand reads (ds_read_b64, not ds_read2_b64) in jit_treeM
# and the 20-state DR matvec: tests, cfg3 lines, cfg3 DR line, cfg3 stall pass.
#   tools/gpu_r3j.sh <tag>
set -o pipefail
T=${1:-r3j}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  -k "treeM or jitm or issue_orders or test_bench_mode_vs_oracle or dr_" > gpurun_out/$T/focus.log 2>&1 || { echo "focus failed"; tail -30 gpurun_out/$T/focus.log; exit 1; }
tail -1 gpurun_out/$T/focus.log
bash tools/ab_bench.sh $T/cfg3 lg08_g4_protein_200k_256 "a:" "b:" "c:" || exit 1
timeout -k 10 300 python tools/bench_dr.py --config lg08_g4_protein_200k_256 --reps 3 --path-branches 4 \
  > gpurun_out/$T/dr_cfg3.json 2> gpurun_out/$T/dr_cfg3.err || { tail -5 gpurun_out/$T/dr_cfg3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/$T/dr_cfg3.json'));print('cfg3 DR',round(d['dr_ms'],2),'ms',d['dr_path'],d['max_rel_diff_dr_vs_path'])"
bash tools/gpu_stalls.sh ${T}_cfg3 lg08_g4_protein_200k_256 || exit 1
