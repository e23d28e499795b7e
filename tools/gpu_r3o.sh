#!/bin/bash
# Round-3 session O: P(t) kernels with batched LDS staging (tests, cfg3 / cfg4 lines and kernel
# traces), then the N > 1 bench path rehearsed on one GPU (tools/gpu_r3n.sh).
set -o pipefail
T=${1:-r3o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  -k "pmat or expm or golden or test_bench_mode_vs_oracle" > gpurun_out/$T/focus.log 2>&1 || { echo "focus failed"; tail -30 gpurun_out/$T/focus.log; exit 1; }
tail -1 gpurun_out/$T/focus.log
export TMPDIR=/tmp
for c in lg08_g4_protein_200k_256 yn98_codon_50k_128; do
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T/k_$c -o run -- \
    python3 $R/bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2 > $R/gpurun_out/$T/k_$c.json 2> $R/gpurun_out/$T/k_$c.err ) || { echo "trace $c failed"; exit 1; }
  grep -i "pmat" gpurun_out/$T/k_$c/run_kernel_stats.csv | cut -d, -f1-4
done
bash tools/ab_bench.sh $T/cfg4 yn98_codon_50k_128 "a:" || exit 1
bash tools/gpu_r3n.sh r3n
