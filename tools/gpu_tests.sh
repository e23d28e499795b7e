#!/bin/bash
# GPU test run with a hard stop on trouble: an optional focused pytest selection (-k
# expression) first, then the whole -m gpu suite; a time-out, crash or abort ends the
# script before the next step.
#   tools/gpu_tests.sh <tag> [-k expression [quick]]   (quick: the selection only)
set -o pipefail
TAG=${1:-t}; shift
mkdir -p gpurun_out
if [ "$1" = "-k" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests -k "$2" > gpurun_out/${TAG}_focus.log 2>&1
  rc=$?
  tail -25 gpurun_out/${TAG}_focus.log
  [ $rc -eq 0 ] || exit $rc
  [ "$3" = "quick" ] && exit 0
fi
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_all.log 2>&1
rc=$?
tail -15 gpurun_out/${TAG}_all.log
exit $rc
