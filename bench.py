#!/usr/bin/env python3
"""bench.py -- site-pattern x node partial updates/s of the MI355X pruning engine.

Contract (driver): python bench.py --gpus N --steps K --warmup W
  N = 1: single process on cuda:0.  N > 1: launched by torch.distributed.run, one
  rank per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the environment).

Workload: BASELINE.json config 2 -- GTR+Gamma4, 4 states, 1M synthetic site patterns,
64-taxon balanced tree (unrooted by the API like the reference, so I = 62 internal
nodes).  Weak scaling: every rank evaluates its own 1M-pattern slice of one global
synthetic alignment (patterns are independent), so per-GPU work is fixed as N grows.

One step = one likelihood evaluation as RHomogeneousTreeLikelihood::fireParameterChanged
does it: all branch transition matrices (K4), the full postorder traversal (partials
kernel, one launch per tree level), the root reduction (K5) whose fixed-order
4096-pattern block sums are all-gathered over RCCL and summed in global order (the
only cross-GPU exchange).  value = (P x I x K x N) / max-over-ranks wall time of the
K timed steps, inputs already resident in HBM.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bpp-phyl_amd"))

import phylo  # noqa: E402
import plk  # noqa: E402
import shard  # noqa: E402
import workload  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="gtr_g4_dna_1M_64", choices=sorted(workload.CONFIGS))
    ap.add_argument("--patterns", type=int, default=None, help="override patterns per rank")
    ap.add_argument("--cpu-sample", type=int, default=None, help="patterns in the CPU-baseline sample")
    ap.add_argument("--cpu-reps", type=int, default=10, help="traversals per CPU-baseline variant (~10-15 s of CPU work for cfg2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-events", action="store_true", help="A/B: time the steps without per-kernel HIP events")
    ap.add_argument("--event-every", type=int, default=4,
                    help="HIP events bracket the partials launches of every K-th timed step (an event pair costs "
                         "~6 us of stream time per step on the box; 1 = every step)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path on ONE GPU (every rank on cuda:0, collectives on the host); "
                         "never a measurement")
    ap.add_argument("--mode", default="lnl", choices=["lnl", "materialize", "levelwise", "subtree"],
                    help="lnl: fused traversal, interior partials kept in registers (recomputed on demand); "
                         "materialize: fused traversal writing every partial; levelwise: one launch per level; "
                         "subtree: per-subtree pattern compression (reference usePatterns=true) -- value is then "
                         "an EFFECTIVE rate (SURVEY 8d), reported beside the computed updates")
    return ap.parse_args()


def cpu_baseline(wl, n_sample: int, reps: int, eng_sites=None):
    """The oracle (faithful C++11 -O2 -g restatement of computeSubtreeLikelihood with the
    reference's nested-vector layout, usePatterns=true -- the reference default) timed on
    one host core over a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/bench infrastructure only

    try:
        os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
    except Exception:
        pass
    et = wl.et
    states = wl.simulate(0, n_sample).astype(np.int32)
    C, S = wl.C, wl.S
    pm = np.zeros((et.n_nodes, C, S, S))
    for n in range(et.n_nodes):
        if n != et.root:
            m = wl.models[0] if wl.model_of_node is None else wl.models[wl.model_of_node[n]]
            for c in range(C):
                pm[n, c] = m.pij(et.brlen[n] * wl.rates[c])
    ss, sons, lr = et.son_arrays()
    res, sites = {}, None
    for up in (True, False):
        _, site, t_trav, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, wl.alphabet.init_table, pm, wl.probs,
                                                wl.root_freqs, use_patterns=up, scaling=wl.scaling, n_rep=reps,
                                                want_sites=up)
        res[up] = n_sample * et.n_internal / t_trav
        if up:
            sites = site
    parity = None
    if eng_sites is not None:
        # SURVEY 8(d)'s third figure, on the sample: the GPU's per-pattern lnL vs the oracle's
        e = np.asarray(eng_sites[:n_sample], dtype=np.float64)
        lo, le = float(np.add.accumulate(sites)[-1]), float(np.add.accumulate(e)[-1])
        parity = {"patterns": n_sample, "rel_err_lnl": abs(le - lo) / abs(lo),
                  "max_rel_err_site": float(np.max(np.abs(e - sites) / np.abs(sites)))}
    return {
        "value": res[True],
        "unit": "site-pattern x node partial updates/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"{n_sample} patterns of the same workload ({et.n_tips} taxa, I={et.n_internal}), "
                   f"oracle/oracle.cpp computeSubtreeLikelihood restatement, g++ -O2 -g, usePatterns=true "
                   f"(reference default), median-free mean of {reps} traversals on 1 pinned core of "
                   f"{platform.processor() or platform.machine()}"),
        "value_use_patterns_false": res[False],
        "parity_vs_oracle": parity,
    }


FP64_PEAK_TFS = 78.6   # MI355X fp64 peak, vector and matrix alike (AMD spec sheet; the guide lists no fp64 row)
RIDGE = FP64_PEAK_TFS * 1e12 / (HBM_PEAK_GBS * 1e9)  # flop/B


def measured_traffic(config, mode, P, launches_per_step):
    """HBM bytes per partials launch from the committed PMC passes (profiles/traffic.json,
    keyed config/mode), rescaled to this run's pattern count."""
    prof = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        tr = json.load(open(prof)).get(f"{config}/{mode}")
    except Exception:
        return None, None
    if not tr:
        return None, None
    per_traversal = tr["hbm_bytes_per_traversal"] * P / tr["patterns"]
    return per_traversal / launches_per_step, tr["source"]


def roofline(wl, mode, P, steps, part_s, launches, bytes_pattern, flops_pattern, traffic):
    """Roofline of the partials kernel.  achieved = algorithmic bytes (or flops) per launch
    (SURVEY 8(d) per-pattern figures x patterns) / mean launch duration (HIP events).
    The binding ceiling follows the bytes the design actually moves: the fused traversal
    (mode lnl, 4 states) keeps interior partials in registers, so it moves ~N+8 B/pattern
    and is fp64-compute bound; the materialising paths stream every partial through HBM
    (intensity <= 7.6 flop/B < the 9.8 flop/B ridge) and are HBM bound."""
    if part_s <= 0:
        return None
    per_launch_s = part_s / launches
    pat_per_launch = P * steps / launches
    gbs = bytes_pattern * pat_per_launch / per_launch_s / 1e9
    tfs = flops_pattern * pat_per_launch / per_launch_s / 1e12
    fused = mode == "lnl" and wl.S == 4 and wl.C in (1, 2, 4)  # tree4_supported() in plk.hip
    if traffic:
        intensity = flops_pattern * pat_per_launch / traffic
        compute_bound = intensity > RIDGE
    else:
        compute_bound = fused
    hbm = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
           "traffic": traffic,
           "basis": (f"algorithmic {bytes_pattern} B/pattern/traversal = 16*C*S*I + N + 8 "
                     f"({bytes_pattern / wl.et.n_internal:.1f} B/update) x {pat_per_launch:.0f} patterns per launch "
                     f"/ mean HIP-event launch duration")}
    if mode == "materialize" and wl.S == 4 and wl.C in (1, 2, 4):
        # the fused traversal writing every partial: children come from registers, so the
        # bytes are the writes (8*C*S per internal node) plus codes, weight and site lnL
        mb = 8 * wl.C * wl.S * wl.et.n_internal + wl.et.n_tips + 16
        g2 = mb * pat_per_launch / per_launch_s / 1e9
        hbm.update(achieved=g2, frac=g2 / HBM_PEAK_GBS,
                   basis=(f"fused traversal writing every partial: {mb} B/pattern = 8*C*S*I writes + N tip codes "
                          f"+ 8 weight + 8 site lnL x {pat_per_launch:.0f} patterns per launch / mean HIP-event "
                          f"launch duration"))
    if fused:
        # the fused traversal's own bytes: tip codes (1 B per tip), weight in, site lnL out
        fb = wl.et.n_tips + 16
        g2 = fb * pat_per_launch / per_launch_s / 1e9
        hbm.update(achieved=g2, frac=g2 / HBM_PEAK_GBS,
                   basis=(f"fused traversal: {fb} B/pattern = N tip codes + 8 weight + 8 site lnL "
                          f"x {pat_per_launch:.0f} patterns per launch / mean HIP-event launch duration"))
    mf = {"bound": "mfma", "achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": tfs / FP64_PEAK_TFS,
          "traffic": traffic,
          "basis": (f"algorithmic {flops_pattern} flop/pattern/traversal = 2*C*S^2 per internal child + (k-1)*C*S "
                    f"per combine ({flops_pattern / wl.et.n_internal:.1f} flop/update) x {pat_per_launch:.0f} "
                    f"patterns per launch / mean HIP-event launch duration; peak = fp64 (vector = matrix) spec")}
    main, alt = (mf, hbm) if compute_bound else (hbm, mf)
    main = dict(main)
    main["other_ceiling"] = {k: alt[k] for k in ("bound", "achieved", "peak", "unit", "frac")}
    main["launch_ms"] = per_launch_s * 1e3
    return main


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    rehearse = world > 1 and args.dist_backend == "gloo"
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        if rehearse:
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    device = local if world > 1 and not rehearse else 0
    coll_dev = "cpu" if rehearse else "cuda"

    wl = workload.make_workload(args.config)
    P = args.patterns or wl.n_patterns
    wl.n_patterns = P
    start, end = rank * P, (rank + 1) * P
    t_setup = time.time()
    extra = {"lnl": plk.PLK_FLAG_LNL_ONLY, "materialize": 0, "levelwise": plk.PLK_FLAG_LEVELWISE,
             "subtree": plk.PLK_FLAG_SUBTREE_PATTERNS}[args.mode]
    ev = workload.Evaluator(wl, device, start, end, extra_flags=extra)
    t_setup = time.time() - t_setup
    units_step = P * wl.et.n_internal

    def one_step():
        lnl, _, blocks = ev.step()
        if dist is None:
            return lnl  # plk_evaluate already summed the block sums in the fixed global order
        # the one cross-GPU exchange: RCCL all-gather of fixed-order block sums
        return shard.allgather_lnl(blocks, dist, device=coll_dev)

    for _ in range(args.warmup):
        lnl = one_step()
    ev.eng.reset_timing()
    # HIP events around the partials launches only (each timed launch adds an event pair),
    # on every K-th timed step: the kernel's mean launch duration is sampled inside the
    # timed region without charging every step the events' own stream time
    k_ev = max(1, args.event_every)
    mask = 0 if args.no_events else plk.PLK_TIME_PARTIALS
    ev_steps = 0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i % k_ev == 0:
            ev.eng.set_timing(mask)
            ev_steps += 1
        elif k_ev > 1 and i % k_ev == 1:
            ev.eng.set_timing(0)
        lnl = one_step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tm = ev.eng.get_timing()
    ev.eng.set_timing(False)
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    if rank == 0:
        ms_step = elapsed * 1e3 / args.steps
        value = units_step * world * args.steps / elapsed
        bytes_pattern = wl.algorithmic_bytes_per_pattern()
        flops_pattern = wl.algorithmic_flops_per_pattern()
        part_s = tm["partials_ms"] * 1e-3
        launches = max(tm["launches"], 1)
        traffic, traffic_src = measured_traffic(args.config, args.mode, P, launches / ev_steps)
        roof = roofline(wl, args.mode, P, ev_steps, part_s, launches, bytes_pattern, flops_pattern, traffic)
        if roof:
            roof["event_sample"] = f"HIP events on {ev_steps} of {args.steps} timed steps (every {k_ev})"
        if traffic_src and roof:
            roof["traffic_source"] = traffic_src
        computed = None
        if args.mode == "subtree":
            # per-subtree compression computes fewer node updates than it is credited with;
            # the roofline is then priced on the updates actually computed
            computed = ev.eng.compressed_work()
            if roof:
                f = computed / units_step
                roof["achieved"] *= f
                roof["frac"] *= f
                roof["basis"] += f"; scaled to the {computed} node updates actually computed per traversal"
                roof.pop("other_ceiling", None)
        rec = {
            "metric": ("site-pattern x node partial updates/s" if args.mode != "subtree" else
                       "site-pattern x node partial updates/s (EFFECTIVE: per-subtree pattern compression)"),
            "value": value,
            "unit": "updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded counter-based simulation under the model, 1 pattern = 1 column)",
            "config": {
                "workload": (f"{args.config}: {wl.models[0].name}{'+G%d' % wl.C if wl.C > 1 else ''} "
                             f"{wl.alphabet.name}, {P} patterns per GPU, {wl.et.n_tips}-taxon balanced tree "
                             f"({'rooted' if wl.model_of_node is not None else 'unrooted'}, I={wl.et.n_internal})"),
                "patterns_per_gpu": P,
                "taxa": wl.et.n_tips,
                "internal_nodes": wl.et.n_internal,
                "states": wl.S,
                "classes": wl.C,
                "mode": args.mode,
                "parallelism": f"pattern-shard x{world}",
            },
            "lnl": lnl,
            "partials_only_updates_per_s": units_step * ev_steps / part_s if part_s > 0 else None,
            "kernel_ms_per_step": {"partials": tm["partials_ms"] / ev_steps, "pmatrix": tm["pmat_ms"] / ev_steps,
                                   "root": tm["root_ms"] / ev_steps},
            "partials_launches_per_step": launches / ev_steps,
            "roofline": roof,
            "setup_s": t_setup,
        }
        if computed is not None:
            rec["computed_updates_per_step"] = computed
            rec["computed_updates_per_s"] = computed * world * args.steps / elapsed
        if world == 1 and not args.no_cpu_baseline:
            ns = args.cpu_sample or workload.CONFIGS[args.config]["cpu_sample"]
            _, eng_sites, _ = ev.eng.root_loglik(wl.et.root, want_sites=True)
            rec["cpu_baseline"] = cpu_baseline(wl, min(ns, P), args.cpu_reps, eng_sites)
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
