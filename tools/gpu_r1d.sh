#!/bin/bash
set -o pipefail
O=gpurun_out/r1d
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for dm in 2 3 4; do
  PLK_TREES_DM=$dm timeout -k 10 240 python bench.py --config lg08_g4_protein_200k_256 --steps 10 --warmup 2 --no-cpu-baseline > $O/cfg3_dm$dm.json 2> $O/cfg3_dm$dm.err || { tail -5 $O/cfg3_dm$dm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg3_dm$dm.json')); print('cfg3 dm$dm', d['value'], d['partials_only_updates_per_s'], d['kernel_ms_per_step'], d['partials_launches_per_step'])"
done
timeout -k 10 300 python bench.py --config nh_gtr_g4_dna_2M_512 --steps 10 --warmup 2 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.err || { tail -5 $O/cfg5.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg5.json')); print('cfg5', d['value'], d['partials_only_updates_per_s'], d['kernel_ms_per_step'], d['partials_launches_per_step'])"
