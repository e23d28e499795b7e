#!/usr/bin/env python3
"""Per-wave view of the tools/gpu_counters.sh passes (last traversal's partials launches)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import traffic_from_pmc as T  # noqa: E402


def main():
    tag = sys.argv[1]
    src = os.path.join(T.ROOT, "gpurun_out", "prof", tag)
    bench = json.load(open(os.path.join(src, "bench.json")))
    n = int(round(bench["partials_launches_per_step"]))
    tot = {}
    names = set()
    for g in ("g1", "g2", "g3"):
        d = os.path.join(src, g)
        if not os.path.isdir(d):
            continue
        for name, c in T.last_traversal(T.per_dispatch(T.rows(d)), n):
            names.add(name.split("(")[0])
            for k, v in c.items():
                tot[k] = tot.get(k, 0.0) + v
    waves = tot.get("SQ_WAVES", 1.0) / 2  # two passes carry SQ_WAVES
    out = {"tag": tag, "kernels": sorted(names), "launches": n,
           "partials_ms": bench["kernel_ms_per_step"]["partials"],
           "per_wave": {k: v / waves for k, v in sorted(tot.items()) if k.startswith("SQ_") and k != "SQ_WAVES"},
           "totals": {k: v for k, v in sorted(tot.items()) if not k.startswith("SQ_")}}
    pw = out["per_wave"]
    if "SQ_WAVE_CYCLES" in pw:
        wc = pw["SQ_WAVE_CYCLES"]
        out["fractions_of_wave_cycles"] = {k: pw[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                   "SQ_ACTIVE_INST_VALU") if k in pw}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
