#!/bin/bash
# in-handle RCCL exchange cost: 1-GPU bench vs 1-rank RCCL (--force-dist) vs 2 gloo ranks; comm tests
set -o pipefail
O=gpurun_out/r2u; mkdir -p $O
timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > $O/plain.json 2> $O/plain.err || { tail -5 $O/plain.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 40 --warmup 3 --force-dist --no-cpu-baseline > $O/nccl1.json 2> $O/nccl1.err || { tail -5 $O/nccl1.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 40 --warmup 3 --dist-backend gloo > $O/gloo2.json 2> $O/gloo2.err || { tail -5 $O/gloo2.err; exit 1; }
for f in plain nccl1 gloo2; do python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', '%.4e' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'kernel %.4f' % d['kernel_ms_per_step']['partials'])"; done
bash tools/gpu_tests.sh r2u -k "comm or multi" quick || exit 1
