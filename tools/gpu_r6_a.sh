#!/bin/bash
# round 6: the new root-rule / exchange / polytomy tests, then the affected suites
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r6a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_root_rules.py tests/test_gpu_underflow.py \
  "tests/test_gpu_parity.py::test_subtree_patterns_wide_polytomy_rescale" \
  "tests/test_gpu_parity.py::test_subtree_patterns_polytomy" \
  "tests/test_gpu_parity.py::test_subtree_patterns_bitwise_vs_uncompressed" \
  tests/test_gpu_multi.py > gpurun_out/r6a/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/r6a/pytest.log
exit $rc
