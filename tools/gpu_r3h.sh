#!/bin/bash
# Round-3 session H: the generated kernels of cfg2 / cfg3 / cfg5 (PLK_JIT_DUMP: source and code
# object, for code size and ISA), and instruction-cache counters of the cfg2 and cfg5 traversals.
#   tools/gpu_r3h.sh <tag>
set -o pipefail
T=${1:-r3h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
for c in gtr_g4_dna_1M_64 lg08_g4_protein_200k_256 nh_gtr_g4_dna_2M_512; do
  mkdir -p gpurun_out/$T/dump_$c
  PLK_JIT_CACHE=0 PLK_JIT_DUMP=$R/gpurun_out/$T/dump_$c timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 2 --warmup 1 \
    > gpurun_out/$T/dump_$c.json 2> gpurun_out/$T/dump_$c.err || { tail -5 gpurun_out/$T/dump_$c.err; exit 1; }
  ls -la gpurun_out/$T/dump_$c
done
export TMPDIR=/tmp
for c in gtr_g4_dna_1M_64 nh_gtr_g4_dna_2M_512; do
  ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH \
      --output-format csv -d $R/gpurun_out/$T/ic_$c -o run -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 2 --warmup 1 \
      > $R/gpurun_out/$T/ic_$c.json 2> $R/gpurun_out/$T/ic_$c.err ) || { echo "icache pass $c failed"; tail -5 gpurun_out/$T/ic_$c.err; exit 1; }
done
echo done
