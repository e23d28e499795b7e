"""Digest tools/gpu_stalls.sh output: per-dispatch averages of the SQ counters of the
traversal kernel, per wave, with the ratios used in DESIGN.md.

    python tools/stalls_digest.py gpurun_out/stalls/<tag> [kernel-substring] [--json out.json]
"""
import collections
import csv
import json
import os
import sys

KERNELS = ("plk_jit_tree4", "plk_jit_treeM", "treeM_kernel", "tree4_kernel")


def load(path, want):
    agg = collections.defaultdict(float)
    disp = set()
    name = None
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if want and want not in k:
            continue
        if not want and not any(x in k for x in KERNELS):
            continue
        name = k.split("(")[0][:60]
        disp.add(r["Dispatch_Id"])
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
    n = max(len(disp), 1)
    return name, n, {k: v / n for k, v in agg.items()}


def main():
    d = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    out = {}
    name = None
    for p in ("a", "b", "c"):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if os.path.exists(f):
            name, n, c = load(f, want)
            out.update(c)
    w = out.get("SQ_WAVES", 1.0)
    per_wave = {k: v / w for k, v in out.items() if k.startswith("SQ_") and k != "SQ_WAVES"}
    res = {"kernel": name, "per_dispatch": out, "per_wave": per_wave}
    wc = out.get("SQ_WAVE_CYCLES")
    if wc:
        # SQ_WAVE_CYCLES and the SQ_ACTIVE_* / SQ_WAIT_* counters share one unit on gfx950
        # (per-wave cycles summed over waves), so their ratios are fractions of wave lifetime
        res["frac_of_wave_cycles"] = {k: out[k] / wc for k in out
                                      if k.startswith(("SQ_ACTIVE", "SQ_WAIT", "SQ_BUSY"))}
    lat = {}
    for lvl, n in (("SQ_INST_LEVEL_SMEM", ["SQ_INSTS_SMEM"]), ("SQ_INST_LEVEL_LDS", ["SQ_INSTS_LDS"]),
                   ("SQ_INST_LEVEL_VMEM", ["SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"])):
        cnt = sum(out.get(k, 0.0) for k in n)
        if lvl in out and cnt:
            lat[lvl[len("SQ_INST_LEVEL_"):]] = out[lvl] / cnt
    if lat:
        res["avg_latency"] = lat
    print(json.dumps(res, indent=1))
    if "--json" in sys.argv:
        json.dump(res, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
