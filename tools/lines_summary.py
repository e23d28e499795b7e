"""One row per bench line: ms per step, value, roofline frac, CPU baseline, strong sub-record.
    python tools/lines_summary.py gpurun_out/r4e_cfg2.json ..."""
import json
import sys

for p in sys.argv[1:]:
    try:
        d = json.load(open(p))
    except Exception as e:  # noqa: BLE001
        print(p, "missing", e)
        continue
    cb = d.get("cpu_baseline") or {}
    s = d.get("strong") or {}
    print(p.split("/")[-1], round(d["ms_per_step"], 4), "%.3g" % d["value"], round(d["roofline"]["frac"], 3),
          "%.3g" % cb.get("value", 0), s.get("ms_per_step"), d.get("host_us_per_eval"))
