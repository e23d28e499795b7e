#!/bin/bash
# Round profile set, in two parts (each fits one gpurun call):
#   part 1: the whole -m gpu suite, then cfg2 (lnl, materialize, subtree)
#   part 2: cfg3 / cfg4 / cfg5 lnl, the default bench line, the DR pass, stall passes
# For each config/mode: the bench line, rocprofv3 kernel-trace stats and PMC passes
# (tools/gpu_prof.sh); digest with tools/traffic_from_pmc.py and tools/stalls_digest.py.
#   tools/gpu_profile_round.sh <prefix> <part>
set -o pipefail
P=${1:-r}; PART=${2:-1}
mkdir -p gpurun_out
if [ "$PART" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${P}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${P}_pytest.log; exit 1; }
  tail -1 gpurun_out/${P}_pytest.log
  bash tools/gpu_prof.sh ${P}_cfg2_lnl gtr_g4_dna_1M_64 lnl 20 || exit 1
  bash tools/gpu_prof.sh ${P}_cfg2_mat gtr_g4_dna_1M_64 materialize 10 || exit 1
  bash tools/gpu_prof.sh ${P}_cfg2_sub gtr_g4_dna_1M_64 subtree 10 || exit 1
  exit 0
fi
bash tools/gpu_prof.sh ${P}_cfg3_lnl lg08_g4_protein_200k_256 lnl 5 || exit 1
bash tools/gpu_prof.sh ${P}_cfg4_lnl yn98_codon_50k_128 lnl 10 || exit 1
bash tools/gpu_prof.sh ${P}_cfg5_lnl nh_gtr_g4_dna_2M_512 lnl 10 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench_default.json 2> gpurun_out/${P}_bench_default.err || { tail -5 gpurun_out/${P}_bench_default.err; exit 1; }
cat gpurun_out/${P}_bench_default.json
# row f4: the double-recursive all-branch derivative pass (kernel-trace stats)
mkdir -p gpurun_out/prof/${P}_cfg2_dr
( export TMPDIR=/tmp; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof/${P}_cfg2_dr/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_dr.py --config gtr_g4_dna_1M_64 --path-branches 16 > $GRAFT_REPO_ROOT/gpurun_out/prof/${P}_cfg2_dr/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof/${P}_cfg2_dr/trace.err ) || { echo "dr profile failed"; exit 1; }
cat gpurun_out/prof/${P}_cfg2_dr/bench.json
bash tools/gpu_stalls.sh ${P}_cfg2 gtr_g4_dna_1M_64 || exit 1
bash tools/gpu_stalls.sh ${P}_cfg3 lg08_g4_protein_200k_256 || exit 1
bash tools/gpu_stalls.sh ${P}_cfg5 nh_gtr_g4_dna_2M_512 || exit 1
