#!/bin/bash
# GPU session: parity tests, then benchmarks of each cfg2 mode and the protein/codon configs.
set -o pipefail
O=gpurun_out/r1b
mkdir -p $O
timeout -k 10 600 python -m pytest tests -m "gpu and not slow" -x -q > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cw in 1 2 4; do
  PLK_TREE4_CW=$cw timeout -k 10 180 python bench.py --steps 20 --warmup 3 --mode lnl --no-cpu-baseline > $O/bench_lnl_cw$cw.json 2> $O/bench_lnl_cw$cw.err || exit 1
  cat $O/bench_lnl_cw$cw.json
done
timeout -k 10 180 python bench.py --steps 20 --warmup 3 --mode materialize --no-cpu-baseline > $O/bench_mat.json 2> $O/bench_mat.err && cat $O/bench_mat.json || exit 1
timeout -k 10 180 python bench.py --steps 20 --warmup 3 --mode levelwise --no-cpu-baseline > $O/bench_lev.json 2> $O/bench_lev.err && cat $O/bench_lev.json || exit 1
timeout -k 10 240 python bench.py --config lg08_g4_protein_200k_256 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_lg08.json 2> $O/bench_lg08.err && cat $O/bench_lg08.json || exit 1
timeout -k 10 240 python bench.py --config yn98_codon_50k_128 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_yn98.json 2> $O/bench_yn98.err && cat $O/bench_yn98.json || exit 1
