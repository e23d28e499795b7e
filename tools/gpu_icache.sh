#!/bin/bash
# Instruction-fetch counters of the cfg5 traversal (tier-0 vs tier-1 dispatches)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/icache
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -o -E "\b(SQC|SQ_IFETCH|SQ_WAIT_INST|SQ_INST_CYCLES)[A-Z_]*\b" $O/avail.txt | sort -u > $O/names.txt || true
cat $O/names.txt | tr '\n' ' '; echo
C1=""
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH; do grep -qx $c $O/names.txt && C1="$C1 $c"; done
echo "counters:$C1"
[ -n "$C1" ] || exit 0
for p in 4096 250000; do
  timeout -s KILL 90 rocprofv3 --pmc $C1 SQ_WAVES SQ_WAIT_INST_ANY --output-format csv -d $O/p$p -o run -- \
    python3 $R/bench.py --config nh_gtr_g4_dna_2M_512 --patterns $p --no-cpu-baseline --no-strong --steps 2 --warmup 1 > /dev/null 2> $O/p$p.err || { tail -5 $O/p$p.err; exit 1; }
  python3 - $O/p$p/run_counter_collection.csv <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    agg[(r["Dispatch_Id"], r["Kernel_Name"][:30], r.get("Grid_Size", ""))][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in list(agg.items())[-8:]:
    print(k, {c: round(x) for c, x in v.items()})
PY
done
