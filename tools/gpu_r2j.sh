#!/bin/bash
# memory-latency pass for cfg5 / cfg2 / cfg3
set -o pipefail
for c in "cfg5 nh_gtr_g4_dna_2M_512" "cfg2 gtr_g4_dna_1M_64" "cfg3 lg08_g4_protein_200k_256"; do
  set -- $c
  O=$GRAFT_REPO_ROOT/gpurun_out/stalls/$1; mkdir -p $O
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS \
    SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS --output-format csv -d $O/c -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config $2 --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2> $O/c.err ) || { tail -5 $O/c.err; exit 1; }
done
echo done
