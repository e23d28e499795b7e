#!/bin/bash
# jit_treeM prefetch A/B on cfg3
set -o pipefail
bash tools/gpu_tests.sh t7 -k "jit_treeM_register_depths or jit_treeM_vs_oracle" quick || exit 1
O=gpurun_out/r2d; mkdir -p $O
run() {  # name config envs
  env $(echo $3 | tr ',' ' ') timeout -k 10 200 python bench.py --config $2 --steps 10 --warmup 2 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python -c "import json; d=json.load(open('$O/$1.json')); r=d['roofline']; print('$1', d['kernel_path'], '%.4e' % d['value'], 'trav_ms %.4f' % r['traversal_ms'], 'frac %.3f' % r['frac'], 'exec %.3f' % r['executed']['frac'])"
}
C=lg08_g4_protein_200k_256
run dm4 $C "PLK_JITM_DM=4" || exit 1
run dm4h $C "PLK_JITM_DM=4,PLK_JITM_HOIST=1" || exit 1
run dm4p2 $C "PLK_JITM_DM=4,PLK_JITM_PD=2" || exit 1
run dm3p2 $C "PLK_JITM_DM=3,PLK_JITM_PD=2" || exit 1
run dm3p2h $C "PLK_JITM_DM=3,PLK_JITM_PD=2,PLK_JITM_HOIST=1" || exit 1
run dm3h $C "PLK_JITM_DM=3,PLK_JITM_HOIST=1" || exit 1
run dm4l2 $C "PLK_JITM_DM=4,PLK_JITM_L=2" || exit 1
echo done
