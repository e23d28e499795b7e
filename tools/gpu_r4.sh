#!/bin/bash
# Round-4 GPU step: a focused pytest selection, then (optionally) the default bench line.
#   tools/gpu_r4.sh <tag> "<-k expression>" [bench]
set -o pipefail
TAG=${1:-r4}; K=$2; mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "$K" \
    > gpurun_out/${TAG}_focus.log 2>&1
  rc=$?; tail -30 gpurun_out/${TAG}_focus.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$3" = "bench" ]; then
  timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?; cat gpurun_out/${TAG}_bench.json; tail -5 gpurun_out/${TAG}_bench.err; exit $rc
fi
