#!/bin/bash
# Round 5: the communicator's global sum on the host -- the comm tests, then the N > 1 bench
# path at one RCCL rank (weak, three lines) against the library before the change (PLK_LIB).
set -o pipefail
O=gpurun_out/${1:-r5comm}
mkdir -p $O
export PLK_JIT_CACHE=$PWD/gpurun_out/jit_cache
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -k "comm" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/pytest.log | head -30; exit $rc; }
for i in 1 2 3; do
  for v in new old; do
    L=""; [ $v = old ] && L=$PWD/ab/libplk_head.so
    PLK_LIB=$L timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29520 + i)) \
      bench.py --gpus 1 --steps 20 --warmup 3 --force-dist --no-cpu-baseline --no-strong > $O/dist1_${v}_$i.json 2> $O/dist1_${v}_$i.err || { tail -5 $O/dist1_${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$O/dist1_${v}_$i.json'));print('$v $i', round(d['ms_per_step'],4), d['lnl'])"
  done
done
