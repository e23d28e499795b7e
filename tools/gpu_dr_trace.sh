set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/prof/drt; export TMPDIR=/tmp; cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof/drt/trace -o run -- python3 $R/tools/bench_dr.py --config gtr_g4_dna_1M_64 --path-branches 2 --reps 2 > $R/gpurun_out/prof/drt/bench.json 2> $R/gpurun_out/prof/drt/err || { tail -3 $R/gpurun_out/prof/drt/err; exit 1; }
