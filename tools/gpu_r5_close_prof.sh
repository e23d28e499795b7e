#!/bin/bash
# Round-5 closing profiles at the 200-step window: kernel-trace stats + FETCH/WRITE/SQ passes
# per configuration (digests in gpurun_out/r05close), then the JIT cache entries of the
# random-topology tests (compiled into a copy of .jit_cache under gpurun_out/jitc)
set -o pipefail
p() { tag=$1; cfg=$2; steps=$3
  bash tools/gpu_prof.sh $tag $cfg lnl $steps > /dev/null || exit 1
  python tools/traffic_from_pmc.py $tag $cfg lnl ../gpurun_out/r05close > /dev/null || exit 1
  rm -rf gpurun_out/prof/$tag; echo "$tag done"; }
p r5k_cfg2_lnl gtr_g4_dna_1M_64 200
p r5k_cfg5_lnl nh_gtr_g4_dna_2M_512 200
p r5k_cfg4_lnl yn98_codon_50k_128 100
rm -rf gpurun_out/jitc; cp -r .jit_cache gpurun_out/jitc
PLK_JIT_CACHE=$(pwd)/gpurun_out/jitc timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "random_topologies or polytomy or pmat64" tests > gpurun_out/r05close/pytest_jitc.log 2>&1 || { tail -20 gpurun_out/r05close/pytest_jitc.log; exit 1; }
tail -1 gpurun_out/r05close/pytest_jitc.log; echo "jitc entries $(ls gpurun_out/jitc | wc -l)"
