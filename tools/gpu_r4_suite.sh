#!/bin/bash
# Round-4 GPU step: focused selection (optional), then the whole -m gpu suite with test durations,
# then (optional) the default bench line.   tools/gpu_r4_suite.sh <tag> ["-k expr"] [bench]
set -o pipefail
TAG=${1:-r4}; K=$2; mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "$K" \
    > gpurun_out/${TAG}_focus.log 2>&1
  rc=$?; tail -30 gpurun_out/${TAG}_focus.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=60 -m gpu tests \
  > gpurun_out/${TAG}_all.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/${TAG}_all.log | tail -3; [ $rc -eq 0 ] || { tail -40 gpurun_out/${TAG}_all.log; exit $rc; }
if [ "$3" = "bench" ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?; cat gpurun_out/${TAG}_bench.json; tail -5 gpurun_out/${TAG}_bench.err; exit $rc
fi
