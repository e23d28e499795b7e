"""Gaps and durations of the kernels of each evaluation in a rocprofv3 kernel-trace CSV
(tools/gpu_r6_trace.sh): per evaluation, from the P(t) kernel's start to the last kernel's end,
each kernel's duration and the idle time before it.  Medians over the evaluations."""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "plk" in r["Kernel_Name"] or "pmat" in r["Kernel_Name"] or "wave_sums" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    for k in ("pmat4", "plk_jit_tree4", "cls_blocks", "wave_sums_to_blocks", "unit_codes"):
        if k in n:
            return k
    return n[:30]


evals, cur = [], []
for r in rows:
    k = short(r["Kernel_Name"])
    if k == "pmat4" and cur:
        evals.append(cur)
        cur = []
    cur.append((k, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
if cur:
    evals.append(cur)
evals = [e for e in evals if e[0][0] == "pmat4"][2:]  # (skip the first evaluations)
keys = {}
for e in evals:
    prev_end = e[0][1]
    for i, (k, s, t) in enumerate(e):
        keys.setdefault(k, {"dur": [], "gap": []})
        keys[k]["dur"].append((t - s) / 1e3)
        keys[k]["gap"].append((s - prev_end) / 1e3)
        prev_end = t
span = [(e[-1][2] - e[0][1]) / 1e3 for e in evals]
print("evaluations %d, span (P(t) start -> last end) median %.1f us" % (len(evals), st.median(span)))
for k, v in keys.items():
    print("  %-22s dur median %.1f us   idle before it median %.1f us" % (k, st.median(v["dur"]), st.median(v["gap"])))
