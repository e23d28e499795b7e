#!/bin/bash
# Timing anatomy: traversal launches with and without the per-launch table staging
# (PLK_DEBUG_NOSTAGE=1 gives wrong results; timing only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/nostage
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
run() { tag=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t$tag -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-strong --steps 10 "$@" > $O/b$tag.json 2> $O/b$tag.err || { tail -5 $O/b$tag.err; exit 1; }
  python3 $R/tools/trace_summary.py $O/t$tag/run_kernel_trace.csv 8 > $O/s$tag.txt && rm -rf $O/t$tag
  echo "== $tag"; cat $O/s$tag.txt | tail -4; }
for ns in 0 1; do
  if [ $ns = 1 ]; then export PLK_DEBUG_NOSTAGE=1; fi
  run c5_4k_$ns --config nh_gtr_g4_dna_2M_512 --patterns 4096
  run c5_250k_$ns --config nh_gtr_g4_dna_2M_512
  run c2_4k_$ns --patterns 4096
  run c2_1M_$ns
done
