#!/bin/bash
# GPU session: parity tests, then config benches under kernel-selection variants.
set -o pipefail
O=gpurun_out/r1g
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # run <tag> <config> [VAR=value ...]
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '%.3e' % d['value'], '%.3e' % d['partials_only_updates_per_s'], d['kernel_ms_per_step'], d['partials_launches_per_step'])"
}
run cfg3_m2 lg08_g4_protein_200k_256 PLK_TREEM_DM=2 || exit 1
run cfg3_m3 lg08_g4_protein_200k_256 PLK_TREEM_DM=3 || exit 1
run cfg4_m2 yn98_codon_50k_128 PLK_TREEM_DM=2 || exit 1
run cfg4_m3 yn98_codon_50k_128 PLK_TREEM_DM=3 || exit 1
bash tools/gpu_counters.sh cnt_cfg3_m2 lg08_g4_protein_200k_256 PLK_TREEM_DM=2 || exit 1
