#!/bin/bash
# The default command (python bench.py) under the kernel trace: per-launch durations split by
# workload (cfg2's 250 launches, then the strong sub-record's config-5 tiers), digested on the box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5deftrace
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/bench.py > $O/bench_default_under_trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
t=$(find $O/t -name "*kernel_trace.csv" | head -1)
cp $(find $O/t -name "*kernel_stats.csv" | head -1) $O/default_kernel_stats.csv
python3 - $t $O/bench_default_under_trace.json $O/default_trace_digest.json <<'PY'
import csv, json, sys, statistics as st
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
d = json.load(open(sys.argv[2]))
def dur(r): return (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000.0
jit = [r for r in rows if 'plk_jit_tree4' in r['Kernel_Name']]
warm, steps = d['warmup'], d['steps']
n2 = warm + steps + 1           # cfg2: the setup's evaluation, warmup and timed steps (one launch each)
c2 = [dur(r) for r in jit[:n2]]
c5 = [dur(r) for r in jit[n2:]]
out = {"command": "python bench.py (default line, under rocprofv3 --kernel-trace --stats)",
       "cfg2_jit_tree4_launches": len(c2), "cfg2_jit_tree4_mean_us": st.mean(c2), "cfg2_jit_tree4_median_us": st.median(c2),
       "cfg2_timed_launches_mean_us": st.mean(c2[-steps:]),
       "bench_traversal_us_hip_events": d['roofline']['traversal_ms'] * 1e3, "bench_ms_per_step_under_trace": d['ms_per_step'],
       "cfg5_2M_launches": len(c5), "cfg5_2M_tier0_median_us": st.median(c5[0::2]) if c5 else None,
       "cfg5_2M_tier1_median_us": st.median(c5[1::2]) if c5 else None}
for k in ("pmat4_kernel", "wave_sums_to_blocks"):
    v = [dur(r) for r in rows if k in r['Kernel_Name']]
    out[k + "_mean_us_all"] = st.mean(v) if v else None
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
PY
rm -rf $O/t
