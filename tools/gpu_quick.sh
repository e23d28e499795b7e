#!/bin/bash
# Quick GPU iteration: gpu parity tests (not slow), then lnl benches of all configs.
#   tools/gpu_quick.sh <tag> [VAR=value ...]
set -o pipefail
TAG=${1:-quick}; shift
O=gpurun_out/$TAG
mkdir -p $O
for kv in "$@"; do export "$kv"; done
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # run <tag> <config> [extra bench args]
  local tag=$1 cfg=$2; shift 2
  timeout -k 10 240 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('$tag', '%.3e' % d['value'], 'part %.3e' % d['partials_only_updates_per_s'], {k: round(v,3) for k,v in d['kernel_ms_per_step'].items()}, d['partials_launches_per_step'], r['bound'], round(r['frac'],3), r['other_ceiling']['bound'], round(r['other_ceiling']['frac'],3))"
}
run cfg2 gtr_g4_dna_1M_64 || exit 1
run cfg3 lg08_g4_protein_200k_256 || exit 1
run cfg4 yn98_codon_50k_128 || exit 1
run cfg5 nh_gtr_g4_dna_2M_512 || exit 1
run cfg2m gtr_g4_dna_1M_64 --mode materialize || exit 1
