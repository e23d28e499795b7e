#!/bin/bash
# Round-3 GPU session, in parts (each fits one gpurun call):
#   part 1: the whole -m gpu suite, the default bench line, the strong-scaling config-5 line
#           (2M patterns on one GPU), the mirror bench lines, cfg2 profile (stats + PMC)
#   part 2: cfg3 / cfg4 / cfg5 profiles (stats + PMC), the DR pass per config, stall passes
# Digest: tools/traffic_from_pmc.py, tools/stalls_digest.py; copy into profiles/r03/.
#   tools/gpu_round3.sh <prefix> <part>
set -o pipefail
P=${1:-r3}; PART=${2:-1}
mkdir -p gpurun_out
if [ "$PART" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${P}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${P}_pytest.log; exit 1; }
  tail -1 gpurun_out/${P}_pytest.log
  timeout -k 10 300 python bench.py > gpurun_out/${P}_bench_default.json 2> gpurun_out/${P}_bench_default.err || { tail -5 gpurun_out/${P}_bench_default.err; exit 1; }
  cat gpurun_out/${P}_bench_default.json
  timeout -k 10 300 python bench.py --scaling strong > gpurun_out/${P}_bench_strong_cfg5.json 2> gpurun_out/${P}_bench_strong_cfg5.err || { tail -5 gpurun_out/${P}_bench_strong_cfg5.err; exit 1; }
  timeout -k 10 150 bpp-phyl_amd/host/bin/bench_mirror cfg2 > gpurun_out/${P}_mirror_cfg2.json || exit 1
  timeout -k 10 150 bpp-phyl_amd/host/bin/bench_mirror cfg3 > gpurun_out/${P}_mirror_cfg3.json || exit 1
  timeout -k 10 200 python bench.py --patterns 609573 --no-cpu-baseline > gpurun_out/${P}_bench_609k.json 2>> gpurun_out/${P}_bench_default.err || exit 1
  bash tools/gpu_prof.sh ${P}_cfg2_lnl gtr_g4_dna_1M_64 lnl 20 || exit 1
  exit 0
fi
bash tools/gpu_prof.sh ${P}_cfg3_lnl lg08_g4_protein_200k_256 lnl 5 || exit 1
bash tools/gpu_prof.sh ${P}_cfg4_lnl yn98_codon_50k_128 lnl 10 || exit 1
bash tools/gpu_prof.sh ${P}_cfg5_lnl nh_gtr_g4_dna_2M_512 lnl 10 || exit 1
for c in gtr_g4_dna_1M_64 lg08_g4_protein_200k_256 yn98_codon_50k_128 nh_gtr_g4_dna_2M_512; do
  mkdir -p gpurun_out/prof/${P}_dr_$c
  ( export TMPDIR=/tmp; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof/${P}_dr_$c/trace -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/bench_dr.py --config $c --reps 3 --path-branches 8 > $GRAFT_REPO_ROOT/gpurun_out/prof/${P}_dr_$c/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof/${P}_dr_$c/trace.err ) || { echo "dr profile $c failed"; exit 1; }
  cat gpurun_out/prof/${P}_dr_$c/bench.json
done
bash tools/gpu_stalls.sh ${P}_cfg3 lg08_g4_protein_200k_256 || exit 1
bash tools/gpu_stalls.sh ${P}_cfg5 nh_gtr_g4_dna_2M_512 || exit 1
timeout -k 10 150 bpp-phyl_amd/host/bin/bench_mirror cfg2 > gpurun_out/${P}_mirror_cfg2.json || exit 1
timeout -k 10 200 python bench.py --patterns 609573 --no-cpu-baseline > gpurun_out/${P}_bench_609k.json 2> gpurun_out/${P}_bench_609k.err || exit 1
PLK_TUNE=PMAT_STAGED=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${P}_bench_pmatstaged.json 2> gpurun_out/${P}_bench_pmatstaged.err || exit 1
