#!/bin/bash
# round 6: direct codes in the classes-in-the-wave kernel (PLK_TUNE JIT_DC_CIW=1) -- bitwise test,
# then the cfg5 shard and cfg5 at 2 M A/B at the driver's window
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${TAG:-r6dcciw}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "direct_codes_classes_in_wave" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=${TAG:-r6dcciw}/s SWEEP="JIT_DC_CIW=0;JIT_DC_CIW=1;JIT_DC_CIW=0;JIT_DC_CIW=1" ARGS="--config nh_gtr_g4_dna_2M_512" bash tools/gpu_r6_sweep.sh
