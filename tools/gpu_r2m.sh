#!/bin/bash
# P(t) load stream across a fragment's contributions: parity subset, then cfg5 A/B
set -o pipefail
mkdir -p gpurun_out/r2m/dump5
PLK_JIT_DUMP=gpurun_out/r2m/dump5 timeout -k 10 200 python bench.py --config nh_gtr_g4_dna_2M_512 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2m/d5.json 2> gpurun_out/r2m/d5.err || { tail -20 gpurun_out/r2m/d5.err; exit 1; }
bash tools/gpu_tests.sh r2m -k "jit_tree4 or nonhomogeneous or scaling or bench_mode" quick || exit 1
bash tools/gpu_sweep_env.sh r2m nh_gtr_g4_dna_2M_512 "stream:" "nopipe:PLK_JIT_PPIPE=0" "g8:PLK_JIT_G=8" "dm5:PLK_JIT_CIW_DM=5" "dm7:PLK_JIT_CIW_DM=7" || exit 1
