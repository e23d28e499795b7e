#!/bin/bash
# Round 5: fused root fragment with rotated first-tier order -- the fused / dynamic / interpreter
# bitwise tests, then cfg5 A/B lines and the cycle split (JIT_FUSEDBG=5).
set -o pipefail
O=gpurun_out/${1:-r5f3}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fused_root or dynamic_superblocks or jit_tree4_bitwise or share_code" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_fused.log 2>&1
rc=$?; tail -3 $O/pytest_fused.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/pytest_fused.log | head -30; exit $rc; }
bash tools/gpu_r5_fuse_ab.sh ${1:-r5f3}/ab JIT_FUSE=0 JIT_FUSE=1 || exit $?
v=JIT_FUSEDBG=5
PLK_TUNE=$v timeout -k 10 300 python bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong > $O/c5_dbg.json 2> $O/c5_dbg.err || exit $?
PLK_TUNE=$v timeout -k 10 300 python bench.py --scaling strong --no-cpu-baseline --steps 10 > $O/c5s_dbg.json 2> $O/c5s_dbg.err || exit $?
grep 'fuse dbg' $O/c5_dbg.err $O/c5s_dbg.err
