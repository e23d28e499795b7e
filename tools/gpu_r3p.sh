#!/bin/bash
# Round-3 session P: the whole -m gpu suite after the batched staging in the P(t) and cherry-
# table kernels, cfg3 / cfg4 lines with kernel traces, the default line, and the N > 1 bench
# path rehearsed on one GPU (stdout must be exactly one JSON line).
set -o pipefail
T=${1:-r3p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/$T/all.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/$T/all.log; exit 1; }
tail -1 gpurun_out/$T/all.log
export TMPDIR=/tmp
for c in lg08_g4_protein_200k_256 yn98_codon_50k_128; do
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/k_$c -o run -- \
    python3 $R/bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2 > $R/gpurun_out/$T/k_$c.json 2> $R/gpurun_out/$T/k_$c.err ) || { echo "trace $c failed"; exit 1; }
  cut -d, -f1-4 gpurun_out/$T/k_$c/run_kernel_stats.csv | head -6
done
bash tools/ab_bench.sh $T/ab yn98_codon_50k_128 "cfg4:" || exit 1
bash tools/ab_bench.sh $T/ab lg08_g4_protein_200k_256 "cfg3:" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || { tail -5 gpurun_out/$T/bench_default.err; exit 1; }
bash tools/gpu_r3n.sh $T/n || exit 1
wc -l gpurun_out/$T/n/*.json
