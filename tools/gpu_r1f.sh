#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof/cfg3f_sqc
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --config lg08_g4_protein_200k_256 --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQ_WAIT_ANY SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD --output-format csv -d $O/a -o run -- python3 $B > /dev/null 2> $O/a.err || { tail -5 $O/a.err; exit 1; }
PLK_FUSED20=0 timeout -k 10 300 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQ_WAIT_ANY SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD --output-format csv -d $O/k2 -o run -- python3 $B > /dev/null 2> $O/k2.err || { tail -5 $O/k2.err; exit 1; }
echo done
