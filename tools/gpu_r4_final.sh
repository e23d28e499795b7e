#!/bin/bash
# Round-4 closing GPU step: whole -m gpu suite, default bench line, the same command under rocprofv3 --kernel-trace --stats
set -o pipefail
mkdir -p gpurun_out/r4z
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=30 -m gpu tests > gpurun_out/r4z/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/r4z/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { tail -40 gpurun_out/r4z/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -u bench.py > gpurun_out/r4z/bench_default.json 2> gpurun_out/r4z/bench_default.err || { tail -5 gpurun_out/r4z/bench_default.err; exit 1; }
head -c 400 gpurun_out/r4z/bench_default.json; echo
R=$(pwd); export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4z/prof -o run -- \
  python3 $R/bench.py > $R/gpurun_out/r4z/bench_default_under_rocprof.json 2> $R/gpurun_out/r4z/rocprof.err ) || { tail -5 gpurun_out/r4z/rocprof.err; exit 1; }
cp $(find gpurun_out/r4z/prof -name "*kernel_stats.csv" | head -1) gpurun_out/r4z/default_kernel_stats.csv
rm -rf gpurun_out/r4z/prof
head -5 gpurun_out/r4z/default_kernel_stats.csv
