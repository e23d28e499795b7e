"""Per-dispatch summary of a rocprofv3 kernel trace: the last N plk_* dispatches with start
offsets, durations and gaps (tools/gpu_r4_sweep.sh)."""
import csv
import sys

path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows = [r for r in csv.DictReader(open(path)) if "plk" in r["Kernel_Name"] or r["Kernel_Name"].startswith("__amd")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-n:]
t0, prev = int(tail[0]["Start_Timestamp"]), None
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"{r['Kernel_Name'][:34]:34s} start {(s - t0) / 1000:9.1f} dur {(e - s) / 1000:8.1f} gap {gap:6.1f} "
          f"grid {r.get('Grid_Size_X', '')}x{r.get('Grid_Size_Y', '')}")
    prev = e
