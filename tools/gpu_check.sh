#!/bin/bash
# GPU session: full gpu test suite, smoke, default bench (with CPU baseline), config benches.
#   tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
run() {  # run <tag> <config> [VAR=value ...]
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '%.3e' % d['value'], '%.3e' % d['partials_only_updates_per_s'], d['kernel_ms_per_step'], d['partials_launches_per_step'], d['roofline']['bound'], round(d['roofline']['frac'],3))"
}
run cfg3 lg08_g4_protein_200k_256 || exit 1
run cfg4 yn98_codon_50k_128 || exit 1
run cfg5 nh_gtr_g4_dna_2M_512 || exit 1
