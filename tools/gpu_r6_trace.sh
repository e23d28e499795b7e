#!/bin/bash
# round 6: per-dispatch kernel trace of cfg2 evaluations (PATS pattern counts): the durations of
# pmat4 / plk_jit_tree4 / cls_blocks and the gaps between them (rocprofv3 kernel trace, csv)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=gpurun_out/${TAG:-r6trace}
mkdir -p $O
export TMPDIR=/tmp
for pat in ${PATS:-65536 1000000}; do
  mkdir -p $R/$O/t_$pat
  (cd /tmp && PLK_TUNE="${TUNE:-}" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/t_$pat -o tr -- \
    python3 $R/bench.py --no-cpu-baseline --no-strong --patterns $pat $ARGS > $R/$O/line_$pat.json 2> $R/$O/err_$pat.log) || { echo "FAIL $pat"; tail -5 $O/err_$pat.log; exit 1; }
  f=$(find $O/t_$pat -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_gaps.py $f > $O/gaps_$pat.txt && cat $O/gaps_$pat.txt
done
