#!/bin/bash
# Round-2 check: multi-GPU boundary tests + full suite, cfg3 jit_treeM bench and A/B, the
# N>1 bench rehearsals on one GPU (gloo: 2 ranks on cuda:0; nccl: 1 rank with the in-handle
# RCCL communicator).
set -o pipefail
bash tools/gpu_tests.sh t4 -k "multi or comm or sharded" || exit 1
O=gpurun_out/r2a; mkdir -p $O
for spec in "base:" "dm2:PLK_JITM_DM=2" "dm4:PLK_JITM_DM=4" "l2:PLK_JITM_L=2" "minw1:PLK_JITM_MINW=1" "treeM:PLK_JITM=0"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python bench.py --config lg08_g4_protein_200k_256 --steps 10 --warmup 2 --no-cpu-baseline > $O/cfg3_$name.json 2> $O/cfg3_$name.err || { tail -5 $O/cfg3_$name.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg3_$name.json')); r=d['roofline']; print('$name', d['kernel_path'], '%.4e' % d['value'], 'trav_ms %.3f' % r['traversal_ms'], 'frac %.3f' % r['frac'], 'exec %.3f' % r['executed']['frac'])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo > $O/rehearse_gloo2.json 2> $O/rehearse_gloo2.err || { tail -5 $O/rehearse_gloo2.err; exit 1; }
cat $O/rehearse_gloo2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 10 --warmup 2 --force-dist --no-cpu-baseline > $O/rehearse_nccl1.json 2> $O/rehearse_nccl1.err || { tail -5 $O/rehearse_nccl1.err; exit 1; }
cat $O/rehearse_nccl1.json
