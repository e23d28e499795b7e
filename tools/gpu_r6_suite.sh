#!/bin/bash
# round 6: the whole -m gpu suite with a fresh JIT cache written under gpurun_out (copied back
# into .jit_cache afterwards, so the round-end run finds every generated kernel compiled)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r6suite}
mkdir -p $O/jit_cache
cp -r .jit_cache/. $O/jit_cache/ 2>/dev/null
export TMPDIR=/tmp PLK_JIT_CACHE=$GRAFT_REPO_ROOT/$O/jit_cache
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/ ${PYT_EXTRA} > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && grep -E "^FAILED|Error" $O/pytest_gpu.log | head
exit $rc
