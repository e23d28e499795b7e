#!/bin/bash
set -o pipefail
O=gpurun_out/r1c
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m "gpu and not slow" -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_prof.sh cfg2_lnl gtr_g4_dna_1M_64 lnl 20 || exit 1
bash tools/gpu_prof.sh cfg2_mat gtr_g4_dna_1M_64 materialize 20 || exit 1
bash tools/gpu_prof.sh cfg3_lnl lg08_g4_protein_200k_256 lnl 10 || exit 1
bash tools/gpu_prof.sh cfg4_lnl yn98_codon_50k_128 lnl 10 || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && cat $O/bench_default.json
