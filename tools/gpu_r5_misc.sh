#!/bin/bash
# Round 5: the bulk-reuse L2 micro test, the full-size config tests (patterns spread over the
# range), and a kernel-trace timeline of the default cfg2 line (gaps between the kernels of
# consecutive evaluations).
set -o pipefail
O=gpurun_out/${1:-r5x}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
timeout -k 10 180 tools/micro/l2_stale > $O/l2_stale.txt 2>&1 || { echo "l2_stale rc=$?"; cat $O/l2_stale.txt; exit 1; }
cat $O/l2_stale.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_configs.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" $O/pytest_configs.log | tail -12; [ $rc -eq 0 ] || exit $rc
R=$PWD
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o run -- \
  python3 $R/bench.py --no-cpu-baseline --no-strong --steps 30 --warmup 5 > $R/$O/trace_bench.json 2> $R/$O/trace.err ) || { tail -5 $O/trace.err; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python tools/trace_summary.py $f 16 | tee $O/trace_summary.txt
