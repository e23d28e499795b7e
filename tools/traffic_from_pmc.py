#!/usr/bin/env python3
"""Digest a tools/gpu_prof.sh run: HBM bytes per partials traversal from the separate
FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md HBM section: KB units, and on gfx950
FETCH_SIZE tallies half the bytes of a wide streaming read, so bytes = (2*FETCH + WRITE)*1024),
the SQ instruction mix of the same launches, and the kernel-trace stats.  Copies the
summaries into profiles/<round>/ and records traffic in profiles/<round>/traffic.json under
"<config>/<mode>" (bench.py reads profiles/r02/traffic.json, then the round-1 file).

  python tools/traffic_from_pmc.py <tag> <config> <mode> <round>
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PARTIALS = ("tree4_kernel", "treeS_kernel", "treeM_kernel", "partials_", "plk_jit_tree4", "plk_jit_treeM",
            "cherry_table_kernel", "cls_blocks_kernel")  # partials_links_ included


def rows(d):
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = []
    for f in fs:
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def per_dispatch(rs):
    """dispatch id -> (kernel name, {counter: summed value})"""
    acc = OrderedDict()
    for r in sorted(rs, key=lambda r: int(r["Dispatch_Id"])):
        k = int(r["Dispatch_Id"])
        if k not in acc:
            acc[k] = (r["Kernel_Name"], {})
        c = acc[k][1]
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return acc


def last_traversal(acc, n_launch):
    ks = [k for k, (name, _) in acc.items() if any(p in name for p in PARTIALS)]
    return [acc[k] for k in ks[-n_launch:]]


def main():
    tag, config, mode, rnd = sys.argv[1:5]
    src = os.path.join(ROOT, "gpurun_out", "prof", tag)
    bench = json.load(open(os.path.join(src, "bench.json")))
    # the traversal's launches plus the table builds that feed it (cherry_table_kernel)
    n_launch = int(round(bench["partials_launches_per_step"] + bench.get("table_launches_per_step", 0)))
    # one class per workgroup: the classes' root reduction (cls_blocks_kernel) is part of the
    # traversal (inside its HIP events), one launch after it
    if any("cls_blocks_kernel" in n for n, _ in per_dispatch(rows(os.path.join(src, "fetch"))).values()):
        n_launch += 1
    P = bench["config"]["patterns_per_gpu"]
    fetch = last_traversal(per_dispatch(rows(os.path.join(src, "fetch"))), n_launch)
    write = last_traversal(per_dispatch(rows(os.path.join(src, "write"))), n_launch)
    sq = last_traversal(per_dispatch(rows(os.path.join(src, "sq"))), n_launch)
    f_kb = sum(c["FETCH_SIZE"] for _, c in fetch)
    w_kb = sum(c["WRITE_SIZE"] for _, c in write)
    hbm = (2 * f_kb + w_kb) * 1024
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    summary = {
        "config": config, "mode": mode, "patterns": P, "partials_launches_per_traversal": n_launch,
        "kernels": sorted({n for n, _ in fetch}),
        "fetch_size_kb": f_kb, "write_size_kb": w_kb, "hbm_bytes_per_traversal": hbm,
        "hbm_bytes_per_pattern": hbm / P,
        "sq": {k: sum(c.get(k, 0.0) for _, c in sq) for k in (sq[0][1] if sq else {})},
    }
    sqs = summary["sq"]
    if sqs.get("SQ_WAVES"):
        w = sqs["SQ_WAVES"]
        summary["sq_per_wave"] = {k: v / w for k, v in sqs.items() if k != "SQ_WAVES"}
    tp = os.path.join(ROOT, "profiles", rnd, "traffic.json")
    tr = json.load(open(tp)) if os.path.exists(tp) else {}
    tr[f"{config}/{mode}"] = {
        "patterns": P, "hbm_bytes_per_traversal": hbm, "fetch_size_kb": f_kb, "write_size_kb": w_kb,
        "source": (f"profiles/{rnd}/{tag}_pmc.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                   f"last traversal's {n_launch} partials launches; bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 "
                   f"(gfx950: FETCH_SIZE counts half of a wide streaming read, MI355X_MICROARCH.md HBM)"),
    }
    json.dump(tr, open(tp, "w"), indent=1)
    json.dump(summary, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench.json"))
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
