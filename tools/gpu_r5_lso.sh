#!/bin/bash
# cfg3 jit_treeM compiled with and without the load/store optimiser (PLK_TUNE JITM_LSO=0:
# single ds_read_b64 A operands instead of ds_read2_b64 pairs), alternating; oracle test first.
set -o pipefail
O=gpurun_out/${1:-r5l}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
PLK_TUNE=JITM_LSO=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "jit_treeM" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    PLK_TUNE=JITM_LSO=$v timeout -k 10 300 python bench.py --config lg08_g4_protein_200k_256 --no-cpu-baseline --no-strong > $O/cfg3_lso${v}_$i.json 2> $O/cfg3_lso${v}_$i.err || exit $?
    python -c "import json; r=json.load(open('$O/cfg3_lso${v}_$i.json')); print('lso $v', round(r['ms_per_step'],4), round(r['roofline']['traversal_ms'],4), round(r['roofline']['frac'],3), r['lnl'])"
  done
done
