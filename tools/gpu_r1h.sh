#!/bin/bash
set -o pipefail
bash tools/gpu_counters.sh cnt_cfg3_m3 lg08_g4_protein_200k_256 PLK_TREEM_DM=3 || exit 1
bash tools/gpu_counters.sh cnt_cfg4_m3 yn98_codon_50k_128 PLK_TREEM_DM=3 || exit 1
bash tools/gpu_counters.sh cnt_cfg2_lnl gtr_g4_dna_1M_64 || exit 1
