#!/bin/bash
# cfg5 (250 k shard): FETCH_SIZE and WRITE_SIZE per tier launch (separate passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5tierpmc
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/$ctr -o run -- \
    python3 $R/bench.py --config nh_gtr_g4_dna_2M_512 --no-cpu-baseline --no-strong --steps 2 --warmup 1 > /dev/null 2> $O/$ctr.err || { tail -5 $O/$ctr.err; exit 1; }
  f=$(find $O/$ctr -name "*counter_collection.csv" | head -1)
  python3 - $f $ctr <<'PY'
import csv, sys, collections
agg = collections.OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    if 'plk_jit_tree4' not in r['Kernel_Name']: continue
    agg.setdefault(r['Dispatch_Id'], 0.0)
    agg[r['Dispatch_Id']] += float(r['Counter_Value'])
v = list(agg.values())[-4:]
print(sys.argv[2], 'last 4 jit launches (KB):', [round(x) for x in v], ' MB:', [round(x / 1024, 1) for x in v])
PY
  rm -rf $O/$ctr
done
