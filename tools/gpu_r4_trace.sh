#!/bin/bash
# Per-dispatch kernel trace of cfg5 at 250k and 2M patterns (tier structure on stderr)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace
mkdir -p $O
export TMPDIR=/tmp PLK_DEBUG_PROG=1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t250 -o run -- \
  python3 $R/bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong --steps 10 > $O/b250.json 2> $O/b250.err || { tail -5 $O/b250.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t2M -o run -- \
  python3 $R/bench.py --config nh_gtr_g4_dna_2M_512 --scaling strong --no-cpu-baseline --steps 10 > $O/b2M.json 2> $O/b2M.err || { tail -5 $O/b2M.err; exit 1; }
grep "plk " $O/b250.err | head -40
