#!/bin/bash
# Round-5 final profiles: kernel-trace stats + FETCH/WRITE/SQ passes per configuration,
# digested on the box (tools/traffic_from_pmc.py) into gpurun_out/r05final, raw traces removed
set -o pipefail
p() { tag=$1; cfg=$2; steps=$3
  bash tools/gpu_prof.sh $tag $cfg lnl $steps > /dev/null || exit 1
  python tools/traffic_from_pmc.py $tag $cfg lnl ../gpurun_out/r05final > /dev/null || exit 1
  rm -rf gpurun_out/prof/$tag; echo "$tag done"; }
p r5f_cfg2_lnl gtr_g4_dna_1M_64 20
p r5f_cfg5_lnl nh_gtr_g4_dna_2M_512 10
p r5f_cfg4_lnl yn98_codon_50k_128 10
p r5f_cfg3_lnl lg08_g4_protein_200k_256 5
