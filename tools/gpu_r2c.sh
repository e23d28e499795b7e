#!/bin/bash
# matrix-core tree kernel A/B: 20 states staged vs direct, 4 states (PLK_S4_JITM) and
# 64 states (PLK_JITM64) against the VALU / 16x16 kernels
set -o pipefail
bash tools/gpu_tests.sh t6 -k "jit_treeM or matrix_cores" quick || exit 1
O=gpurun_out/r2c; mkdir -p $O
run() {  # name config envs
  env $(echo $3 | tr ',' ' ') timeout -k 10 200 python bench.py --config $2 --steps 10 --warmup 2 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; return 1; }
  python -c "import json; d=json.load(open('$O/$1.json')); r=d['roofline']; print('$1', d['kernel_path'], '%.4e' % d['value'], 'trav_ms %.4f' % r['traversal_ms'], 'frac %.3f' % r['frac'], 'exec %.3f' % r['executed']['frac'])"
}
run cfg3_staged4 lg08_g4_protein_200k_256 "PLK_JITM_DM=4" || exit 1
run cfg3_direct4 lg08_g4_protein_200k_256 "PLK_JITM_DM=4,PLK_JITM_DIRECT=1" || exit 1
run cfg3_direct3 lg08_g4_protein_200k_256 "PLK_JITM_DM=3,PLK_JITM_DIRECT=1" || exit 1
run cfg4_treeM yn98_codon_50k_128 "PLK_X=0" || exit 1
run cfg4_jitm yn98_codon_50k_128 "PLK_JITM64=1" || exit 1
run cfg4_jitm_direct yn98_codon_50k_128 "PLK_JITM64=1,PLK_JITM_DIRECT=1" || exit 1
run cfg4_jitm_dm2 yn98_codon_50k_128 "PLK_JITM64=1,PLK_JITM_DM=2" || exit 1
run cfg2_jit4 gtr_g4_dna_1M_64 "PLK_X=0" || exit 1
run cfg2_mfma8 gtr_g4_dna_1M_64 "PLK_S4_JITM=1" || exit 1
run cfg2_mfma8d gtr_g4_dna_1M_64 "PLK_S4_JITM=1,PLK_JITM_DIRECT=1" || exit 1
run cfg2_mfma12 gtr_g4_dna_1M_64 "PLK_S4_JITM=1,PLK_JITM_DM=12" || exit 1
run cfg5_jit4 nh_gtr_g4_dna_2M_512 "PLK_X=0" || exit 1
run cfg5_mfma8 nh_gtr_g4_dna_2M_512 "PLK_S4_JITM=1" || exit 1
run cfg5_mfma8d nh_gtr_g4_dna_2M_512 "PLK_S4_JITM=1,PLK_JITM_DIRECT=1" || exit 1
echo done
