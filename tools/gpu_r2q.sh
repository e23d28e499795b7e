#!/bin/bash
# dump the generated 20-state kernel (cfg3) for ISA inspection; subtree bench line with the fixed roofline
set -o pipefail
mkdir -p gpurun_out/r2q/dump3
PLK_JIT_DUMP=gpurun_out/r2q/dump3 timeout -k 10 200 python bench.py --config lg08_g4_protein_200k_256 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2q/cfg3.json 2> gpurun_out/r2q/cfg3.err || { tail -5 gpurun_out/r2q/cfg3.err; exit 1; }
timeout -k 10 200 python bench.py --mode subtree --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2q/cfg2_sub.json 2> gpurun_out/r2q/cfg2_sub.err || { tail -5 gpurun_out/r2q/cfg2_sub.err; exit 1; }
echo ok
