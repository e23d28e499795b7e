#!/bin/bash
# Round-5 bench lines per configuration (each step under its own time limit):
#   tools/gpu_r5_lines.sh <tag> [configs...]   configs: cfg2 cfg3 cfg4 cfg5 cfg5s
set -o pipefail
TAG=${1:-r5}; shift; mkdir -p gpurun_out
CFGS=${@:-cfg5 cfg3 cfg4}
for c in $CFGS; do
  case $c in
    cfg2) A="--config gtr_g4_dna_1M_64 --no-strong" ;;
    cfg3) A="--config lg08_g4_protein_200k_256 --cpu-runs 3" ;;
    cfg4) A="--config yn98_codon_50k_128 --cpu-runs 3" ;;
    cfg5) A="--config nh_gtr_g4_dna_2M_512 --cpu-runs 3" ;;
    cfg5s) A="--scaling strong --no-cpu-baseline --steps 20" ;;
  esac
  timeout -k 10 300 python -u bench.py $A > gpurun_out/${TAG}_${c}.json 2> gpurun_out/${TAG}_${c}.err
  rc=$?; echo "== $c rc=$rc"; head -c 600 gpurun_out/${TAG}_${c}.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_${c}.err; exit $rc; }
done
