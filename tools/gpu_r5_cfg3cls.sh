#!/bin/bash
# cfg3 (LG08, 256 taxa, 200k patterns) with 1 / 2 / 4 rate classes: the register footprint of
# one and two classes per wave on the same tree (efficiency per class count), code objects dumped
# for their VGPR / spill counts.
set -o pipefail
O=gpurun_out/${1:-r5c3}
mkdir -p $O/dump
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
for c in 4 2 1 4; do
  PLK_JIT_DUMP=$PWD/$O/dump timeout -k 10 300 python bench.py --config lg08_g4_protein_200k_256 --classes $c --no-cpu-baseline --no-strong > $O/cfg3_c${c}.json 2> $O/cfg3_c${c}.err || exit $?
  python -c "import json; r=json.load(open('$O/cfg3_c${c}.json')); print('classes $c', round(r['ms_per_step'],4), round(r['roofline']['traversal_ms'],4), round(r['roofline']['frac'],3))"
done
ls $O/dump | head
