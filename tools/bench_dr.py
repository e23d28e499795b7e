"""Row f4 measurement: derivatives of EVERY branch, double-recursive pass
(plk_all_branch_derivatives) against one path pass per branch (plk_branch_derivatives,
what RHomogeneousTreeLikelihood does per BrLen parameter).

    python tools/bench_dr.py --config gtr_g4_dna_1M_64 [--patterns N] [--reps K]

One JSON line: branch x pattern derivative updates/s for both, the DR kernels' HIP-event
duration and their algorithmic HBM rate.  Two engine paths (`dr_path`):
  * fused (4 states: dr_pre_s4_kernel; 20 / 64 states: dr_pre_m_kernel on matrix cores;
    with or without rescaling): per father f, U_f read (8 C S,
    not at the root), every son's L (8 C S internal, 1 B tip), the U of internal sons
    written (8 C S), the weight (8 B);
  * levelwise (otherwise, or PLK_TUNE=DR_PRE=0): every upper vector U_v written once (8 C S)
    and read by the reduction (8 C S); the preorder update of U_v reads U_father (8 C S,
    not at the root's sons) and every sibling (8 C S internal, 1 B tip); the reduction
    reads L_v (8 C S internal, 1 B tip) and the weight (8 B) -- `reduction_kernel_ms` and
    `reduction_roofline` then time the reduction launch alone.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bpp-phyl_amd"))
import plk  # noqa: E402
import workload  # noqa: E402


def dr_bytes(wl):
    et = wl.et
    CS8 = 8 * wl.C * wl.S
    kids = {p: list(ch) for p, ch in et.ops}
    parent = {c: p for p, ch in et.ops for c in ch}
    up = red = 0
    for v, f in parent.items():
        up += CS8 + (CS8 if f != et.root else 0)
        up += sum(CS8 if s >= et.n_tips else 1 for s in kids[f] if s != v)
        red += CS8 + (CS8 if v >= et.n_tips else 1) + 8
    return up, red


def dr_fused_bytes(wl):
    et = wl.et
    CS8 = 8 * wl.C * wl.S
    b = 0
    for f, ch in et.ops:
        b += (CS8 if f != et.root else 0) + 8
        b += sum(2 * CS8 if s >= et.n_tips else 1 for s in ch)
    return b


def dr_fused_flops(wl):
    """Contractions of the fused preorder: per father and class, P_f^T U_f (not at the
    root) and, per son, P L, dP L and d2P L -- 2 S^2 flops each."""
    et = wl.et
    n = 0
    for f, ch in et.ops:
        n += (1 if f != et.root else 0) + 3 * len(ch)
    return n * wl.C * 2 * wl.S * wl.S


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="gtr_g4_dna_1M_64")
    ap.add_argument("--patterns", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--path-branches", type=int, default=0, help="time the path method on this many branches (0: all)")
    args = ap.parse_args()
    wl = workload.make_workload(args.config)
    P = args.patterns or wl.n_patterns
    wl.n_patterns = P
    ev = workload.Evaluator(wl, 0, 0, P, extra_flags=plk.PLK_FLAG_DOUBLE_RECURSIVE)
    eng, et = ev.eng, wl.et
    eng.update_pmatrices(ev.branches, et.brlen[ev.branches], ev.model_idx, deriv_mask=7)
    eng.update_partials(ev.ops)
    lnl, _, _ = eng.root_loglik(et.root)
    nb = len(ev.branches)
    d1, d2 = eng.all_branch_derivatives()  # warm-up
    eng.reset_timing()
    eng.set_timing(plk.PLK_TIME_PARTIALS)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        d1, d2 = eng.all_branch_derivatives()
    t_dr = (time.perf_counter() - t0) / args.reps
    tm = eng.get_timing()
    eng.set_timing(False)
    red_ms = tm["partials_ms"] / args.reps
    sel = ev.branches if not args.path_branches else ev.branches[:: max(1, nb // args.path_branches)]
    eng.branch_derivatives(int(sel[0]))  # warm-up
    t0 = time.perf_counter()
    worst = 0.0
    for b in sel:
        p1, p2 = eng.branch_derivatives(int(b))
        worst = max(worst, abs(p1 - d1[b]) / max(1.0, abs(p1)), abs(p2 - d2[b]) / max(1.0, abs(p2)))
    t_path = (time.perf_counter() - t0) / len(sel) * nb
    up, red = dr_bytes(wl)
    # the library's choice (plk.hip dr_derivatives): fused for 4 / 20 states, levelwise for 64
    # unless PLK_TUNE DR_PRE=1; DR_PRE=0 always levelwise
    tune = os.environ.get("PLK_TUNE", "")
    fused = wl.C in (1, 2, 4) and "DR_PRE=0" not in tune and (wl.S in (4, 20) or (wl.S == 64 and "DR_PRE=1" in tune))
    fb = dr_fused_bytes(wl)
    rec = {
        "metric": "branch x site-pattern derivative updates/s (d1 and d2 of every branch)",
        "config": args.config, "patterns": P, "branches": nb, "states": wl.S, "classes": wl.C, "lnl": lnl,
        "dr_ms": t_dr * 1e3, "dr_updates_per_s": nb * P / t_dr,
        "path_ms_all_branches": t_path * 1e3, "path_updates_per_s": nb * P / t_path,
        "speedup_dr_vs_path": t_path / t_dr,
        "path_branches_timed": int(len(sel)),
        "max_rel_diff_dr_vs_path": worst,
        "dr_path": "fused" if fused else "levelwise",
    }
    if fused:
        rec["fused_kernels_ms"] = red_ms
        fl = dr_fused_flops(wl)
        rec["fused_flop_roofline"] = {"bound": "mfma" if wl.S > 4 else "valu", "achieved": fl * P / (red_ms * 1e-3) / 1e12,
                                      "peak": 78.6, "unit": "TFLOP/s",
                                      "frac": fl * P / (red_ms * 1e-3) / 1e12 / 78.6,
                                      "algorithmic_flops_per_pattern": fl,
                                      "basis": "per father and class: 2 S^2 per contraction (P_f^T U_f below the root, "
                                               "P_j L_j, dP_i L_i, d2P_i L_i of every son)"}
        rec["fused_roofline"] = {"bound": "hbm", "achieved": fb * P / (red_ms * 1e-3) / 1e9, "peak": 8000.0,
                                 "unit": "GB/s", "frac": fb * P / (red_ms * 1e-3) / 1e9 / 8000.0,
                                 "algorithmic_bytes_per_pattern": fb}
        rec["levelwise_bytes_per_pattern"] = up + red
    else:
        rec["reduction_kernel_ms"] = red_ms
        rec["reduction_roofline"] = {"bound": "hbm", "achieved": red * P / (red_ms * 1e-3) / 1e9, "peak": 8000.0,
                                     "unit": "GB/s", "frac": red * P / (red_ms * 1e-3) / 1e9 / 8000.0,
                                     "algorithmic_bytes_per_pattern": red}
        rec["dr_pass_algorithmic_GBps"] = (up + red) * P / t_dr / 1e9
        rec["preorder_bytes_per_pattern"] = up
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
