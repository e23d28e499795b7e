#!/bin/bash
# round 6: table-row prefetch distance (PLK_TUNE JIT_RD) on cfg2 -- quads bitwise with JIT_RD=2/3,
# then an A/B sweep at the driver's window
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r6rd}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "quads_bitwise" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=${TAG:-r6rd} SWEEP=";JIT_RD=2;JIT_RD=3;;JIT_RD=2;JIT_RD=3" bash tools/gpu_r6_sweep.sh
