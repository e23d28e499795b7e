#!/bin/bash
# Round-5 closing GPU step: whole -m gpu suite, default bench line, the same command under rocprofv3 --kernel-trace --stats
set -o pipefail
mkdir -p gpurun_out/r5z
# a fresh JIT cache: what the suite compiles is what the repository's .jit_cache should hold
export PLK_JIT_CACHE=$(pwd)/gpurun_out/jit_r5
rm -rf $PLK_JIT_CACHE; mkdir -p $PLK_JIT_CACHE
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=30 -m gpu tests > gpurun_out/r5z/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r5z/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { tail -40 gpurun_out/r5z/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -u bench.py > gpurun_out/r5z/bench_default.json 2> gpurun_out/r5z/bench_default.err || { tail -5 gpurun_out/r5z/bench_default.err; exit 1; }
head -c 400 gpurun_out/r5z/bench_default.json; echo
R=$(pwd); export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5z/prof -o run -- \
  python3 $R/bench.py > $R/gpurun_out/r5z/bench_default_under_rocprof.json 2> $R/gpurun_out/r5z/rocprof.err ) || { tail -5 gpurun_out/r5z/rocprof.err; exit 1; }
cp $(find gpurun_out/r5z/prof -name "*kernel_stats.csv" | head -1) gpurun_out/r5z/default_kernel_stats.csv
rm -rf gpurun_out/r5z/prof
head -5 gpurun_out/r5z/default_kernel_stats.csv
# the round-4 test order that once returned a -inf shard (profiles/r05/ab_runs.md), once
timeout -k 10 600 bash tools/gpu_r4_share3.sh > gpurun_out/r5z/share3.log 2>&1; rc=$?; tail -3 gpurun_out/r5z/share3.log; exit $rc
