#!/bin/bash
# Round-5 closing run: whole -m gpu suite (the repository's JIT cache; new entries reported),
# default line and the same command under the kernel trace, per-configuration lines
set -o pipefail
O=gpurun_out/r5c
mkdir -p $O
n0=$(ls .jit_cache | wc -l)
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=20 -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { tail -40 $O/pytest_gpu.log; exit $rc; }
echo "jit cache entries: $n0 -> $(ls .jit_cache | wc -l)"
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
head -c 700 $O/bench_default.json; echo
R=$(pwd); export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
  python3 $R/bench.py > $R/$O/bench_default_under_rocprof.json 2> $R/$O/rocprof.err ) || { tail -5 $O/rocprof.err; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/default_kernel_stats.csv
rm -rf $O/prof
grep -E "jit_tree4|pmat4|wave_sums" $O/default_kernel_stats.csv | cut -c1-160
timeout -k 10 900 bash tools/gpu_r5_lines.sh r5c/l cfg3 cfg4 cfg5 cfg5s > $O/lines.log 2>&1; rc=$?; grep "==" $O/lines.log; exit $rc
