#!/bin/bash
# cfg5 traversal launches vs pattern count (kernel trace per size)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sweep
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for p in 4096 16384 65536 131072 250000 500000 1000000; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t$p -o run -- \
    python3 $R/bench.py --config nh_gtr_g4_dna_2M_512 --patterns $p --no-cpu-baseline --no-strong --steps 10 > $O/b$p.json 2> $O/b$p.err || { tail -5 $O/b$p.err; exit 1; }
  python3 $R/tools/trace_summary.py $O/t$p/run_kernel_trace.csv 12 > $O/s$p.txt && rm -rf $O/t$p
  echo "done $p"
done
