#!/bin/bash
set -o pipefail
O=gpurun_out/r5fdbg
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
for v in JIT_FUSEDBG=5 JIT_FUSEDBG=4 JIT_FUSE=1; do
  t=$(echo $v | tr '=,' '__')
  PLK_TUNE=$v timeout -k 10 300 python bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong > $O/c5_$t.json 2> $O/c5_$t.err || exit $?
  PLK_TUNE=$v timeout -k 10 300 python bench.py --scaling strong --no-cpu-baseline --steps 10 > $O/c5s_$t.json 2> $O/c5s_$t.err || exit $?
  echo $v; grep 'fuse dbg' $O/c5_$t.err $O/c5s_$t.err
  python -c "
import json;r=json.load(open('$O/c5_$t.json'));s=json.load(open('$O/c5s_$t.json'))
print(r['ms_per_step'], r['roofline']['traversal_ms'], s['ms_per_step'], s['roofline']['traversal_ms'])"
done
