#!/bin/bash
# Round-3 session N: the N > 1 bench path rehearsed on one GPU (torch.distributed.run, one
# rank, --force-dist: process group, in-handle RCCL communicator, the exchange check), weak
# and strong scaling; two gloo ranks sharing the GPU.
set -o pipefail
T=${1:-r3n}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 1 --steps 10 --warmup 2 --force-dist --no-cpu-baseline > gpurun_out/$T/dist1_weak.json 2> gpurun_out/$T/dist1_weak.err || { tail -20 gpurun_out/$T/dist1_weak.err; exit 1; }
tail -c 600 gpurun_out/$T/dist1_weak.json; echo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 1 --steps 10 --warmup 2 --force-dist --scaling strong --no-cpu-baseline > gpurun_out/$T/dist1_strong.json 2> gpurun_out/$T/dist1_strong.err || { tail -20 gpurun_out/$T/dist1_strong.err; exit 1; }
tail -c 600 gpurun_out/$T/dist1_strong.json; echo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --no-cpu-baseline > gpurun_out/$T/gloo2.json 2> gpurun_out/$T/gloo2.err || { tail -20 gpurun_out/$T/gloo2.err; exit 1; }
tail -c 600 gpurun_out/$T/gloo2.json; echo
