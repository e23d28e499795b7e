#!/bin/bash
# dump the generated 4-state kernels (cfg2, cfg5) and count their instruction mix
set -o pipefail
O=gpurun_out/r2e; mkdir -p $O/dump2 $O/dump5
PLK_JIT_DUMP=$O/dump2 timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/cfg2.json 2> $O/cfg2.err || { tail -5 $O/cfg2.err; exit 1; }
PLK_JIT_DUMP=$O/dump5 timeout -k 10 200 python bench.py --config nh_gtr_g4_dna_2M_512 --steps 3 --warmup 1 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.err || { tail -5 $O/cfg5.err; exit 1; }
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in "cfg2 gtr_g4_dna_1M_64" "cfg5 nh_gtr_g4_dna_2M_512"; do
  set -- $c
  ( cd /tmp && timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU --output-format csv -d $R/$O/mix_$1 -o run -- python3 $R/bench.py --config $2 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/$O/mix_$1.err ) || { tail -5 $O/mix_$1.err; echo "mix $1 failed"; }
done
echo done
