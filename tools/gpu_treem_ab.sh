#!/bin/bash
# treeM A/B: staged (PLK_TREEM_DIRECT=0) vs direct tables; parity tests in the new default.
#   tools/gpu_treem_ab.sh <tag>
set -o pipefail
O=gpurun_out/${1:-tm}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dr.py -x -q --timeout 120 --timeout-method thread -k "s20 or treeM or fused20 or random or scaling or pmat64 or any_state or dr_equals or nonhomog" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # run <tag> <config> [VAR=value ...]
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '%.3e' % d['value'], d['kernel_ms_per_step']['partials'], round(d['roofline']['frac'],3), d['lnl'])"
}
run cfg3_staged lg08_g4_protein_200k_256 PLK_TREEM_DIRECT=0 || exit 1
run cfg3_direct lg08_g4_protein_200k_256 PLK_TREEM_DIRECT=1 || exit 1
run cfg4_staged yn98_codon_50k_128 PLK_TREEM_DIRECT=0 || exit 1
run cfg4_direct yn98_codon_50k_128 PLK_TREEM_DIRECT=1 || exit 1
timeout -k 10 200 python tools/bench_dr.py --config gtr_g4_dna_1M_64 --path-branches 16 > $O/dr_cfg2.json 2> $O/dr_cfg2.err || { tail -5 $O/dr_cfg2.err; exit 1; }
cat $O/dr_cfg2.json
