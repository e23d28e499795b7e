#!/bin/bash
set -o pipefail
O=gpurun_out/r1e
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQC[A-Z_0-9]*\|SQ_INST_LEVEL[A-Z_0-9]*\|SQ_IFETCH[A-Z_0-9]*\|SQ_WAIT[A-Z_0-9]*\|SQ_INSTS[A-Z_0-9]*\|SQ_ACTIVE[A-Z_0-9]*\|SQ_BUSY[A-Z_0-9]*\|SQ_LDS[A-Z_0-9]*" $O/counters.txt | sort -u > $O/sq_counters.txt || true
bash tools/gpu_prof.sh cfg3f_lnl lg08_g4_protein_200k_256 lnl 10 || exit 1
bash tools/gpu_prof.sh cfg5f_lnl nh_gtr_g4_dna_2M_512 lnl 10 || exit 1
