#!/usr/bin/env python3
"""bench.py -- site-pattern x node partial updates/s of the MI355X pruning engine.

Contract (driver): python bench.py --gpus N --steps K --warmup W
  N = 1: single process on cuda:0.  N > 1: launched by torch.distributed.run, one
  rank per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the environment).

Workload: BASELINE.json config 2 -- GTR+Gamma4, 4 states, 1M synthetic site patterns,
64-taxon balanced tree (unrooted by the API like the reference, so I = 62 internal
nodes).  Weak scaling (default): every rank evaluates its own 1M-pattern slice of one
global synthetic alignment (patterns are independent), so per-GPU work is fixed as N
grows.  --scaling strong: BASELINE config 5 as stated ("2M patterns ... site-sharded across
8 x MI355X") -- the job's 2M patterns split into contiguous 4096-aligned ranges over the N
ranks (N = 1: all 2M on one GPU), value counting the job's P x I per step.

One step = one likelihood evaluation as RHomogeneousTreeLikelihood::fireParameterChanged
does it (plk_evaluate): all branch transition matrices (K4), the full postorder
traversal -- by default (--mode lnl) the fused, tree-specialised kernel that keeps
interior partials in registers and reads cherries from code-pair tables -- and the root
reduction, whose fixed-order 4096-pattern block sums are all-gathered across ranks and
summed in global order (the only cross-GPU exchange).  value = (P x I x K) /
max-over-ranks wall time of the K timed steps (P = the job's patterns: N x 1M weak,
2M strong), inputs already resident in HBM; this is
the reference-equivalent rate (the reference computes every one of those node
updates).  computed_updates_* report the updates actually computed per pattern
(cherry-table nodes are lookups, SURVEY 8(d) "effective"), and roofline.executed the
fp64 work the kernels really issue (plk_traversal_work, counted from the program).
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
# the tree-specialised kernels compile at setup (not timed); the repository's code-object
# cache (`.jit_cache`, filled by the test suite) spares the compile when it holds them
os.environ.setdefault("PLK_JIT_CACHE", os.path.join(ROOT, ".jit_cache"))
sys.path.insert(0, os.path.join(ROOT, "bpp-phyl_amd"))

import phylo  # noqa: E402
import plk  # noqa: E402
import shard  # noqa: E402
import workload  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of the job: one rank each under torch.distributed.run (WORLD_SIZE must match), "
                         "else one process over devices 0..N-1 (plk_create_multi)")
    ap.add_argument("--devices", default=None,
                    help="one-process multi-device mode: comma-separated device list of --gpus entries "
                         "(e.g. 0,0 rehearses two shards on one GPU; the line is then marked a rehearsal)")
    ap.add_argument("--sim-cpu", default=None, choices=["numpy", "torch"],
                    help="simulate the alignment on the host (default: on the GPU, the same states bitwise)")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the config-5 strong-scaling sub-record of the default line")
    ap.add_argument("--strong-steps", type=int, default=40, help="timed steps of the strong sub-record (~0.1 s)")
    ap.add_argument("--strong-patterns", type=int, default=None,
                    help="tests only: patterns of the strong sub-record (default config 5's 2M)")
    # the driver's window.  Its 25 evaluations (~4 ms of GPU work) run at a shader clock of
    # ~2.0-2.08 GHz; under sustained load the clock settles at ~2.37 GHz after ~150 evaluations,
    # and the traversal's cycle count is the same in both (profiles/r06/clock/) -- a longer
    # window only measures the clock, so the default is the graded one
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=None, choices=sorted(workload.CONFIGS),
                    help="default: gtr_g4_dna_1M_64 (config 2); with --scaling strong nh_gtr_g4_dna_2M_512 (config 5)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: every rank evaluates its own --patterns slice (per-GPU work fixed as N grows); "
                         "strong: --patterns (default: the config's global count, 2M for config 5) in total, split "
                         "into contiguous 4096-aligned ranges over the ranks")
    ap.add_argument("--patterns", type=int, default=None,
                    help="override patterns per rank (weak) or in total (strong)")
    ap.add_argument("--classes", type=int, default=None,
                    help="A/B experiments only: the config's model with this many Gamma classes")
    ap.add_argument("--cpu-sample", type=int, default=None, help="patterns in the CPU-baseline sample")
    ap.add_argument("--cpu-runs", type=int, default=5, help="timed CPU-baseline traversals per variant (median, after 1 warm-up)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-events", action="store_true", help="A/B: time the steps without per-kernel HIP events")
    ap.add_argument("--event-every", type=int, default=4,
                    help="HIP events bracket the partials launches of every K-th timed step (an event pair costs "
                         "~6 us of stream time per step on the box; 1 = every step)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path on ONE GPU (every rank on cuda:0, collectives on the host); "
                         "never a measurement")
    ap.add_argument("--force-dist", action="store_true",
                    help="under torch.distributed.run with ONE rank: still take the N>1 path (process group, "
                         "in-handle RCCL communicator, exchange check) -- a single-GPU rehearsal of it")
    ap.add_argument("--clock-json", default=None,
                    help="diagnostic: generate the traversal kernel with per-workgroup clock stamps "
                         "(PLK_DEBUG_CLOCK=1) and write every evaluation's shader clock (MHz), span and host "
                         "step time to this JSON file (the main measurement only)")
    ap.add_argument("--mode", default="lnl", choices=["lnl", "materialize", "levelwise", "subtree"],
                    help="lnl: fused traversal, interior partials kept in registers (recomputed on demand); "
                         "materialize: fused traversal writing every partial; levelwise: one launch per level; "
                         "subtree: per-subtree pattern compression (reference usePatterns=true) -- value is then "
                         "an EFFECTIVE rate (SURVEY 8d), reported beside the computed updates")
    args = ap.parse_args()
    if args.clock_json and os.environ.get("PLK_DEBUG_CLOCK") != "2":  # (2: stamps end at the prologue)
        os.environ["PLK_DEBUG_CLOCK"] = "1"
    if args.config is None:
        args.config = "nh_gtr_g4_dna_2M_512" if args.scaling == "strong" else "gtr_g4_dna_1M_64"
    return args


def host_cpu() -> dict:
    """CPU model and core counts of this host (state them)."""
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except Exception:
        usable = os.cpu_count()
    return {"model": model, "nproc": os.cpu_count(), "usable_cores": usable}


def cpu_baseline(wl, n_sample: int, runs: int, eng_sites=None):
    """The oracle (faithful C++11 -O2 -g restatement of computeSubtreeLikelihood with the
    reference's nested-vector layout) timed on ONE pinned host core over a bounded sample
    of the same workload: median of `runs` traversals after 1 warm-up, for
    usePatterns = true (the reference default, per-subtree pattern compression) and
    false.  The reference itself cannot be built here."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test/bench infrastructure only

    cpu = host_cpu()
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
        times = []
        for r in range(runs + 1):   # the first run is the warm-up
            _, site, t_trav, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, wl.alphabet.init_table, pm,
                                                    wl.probs, wl.root_freqs, use_patterns=up, scaling=wl.scaling,
                                                    n_rep=1, want_sites=up and r == 0)
            if r == 0:
                if up:
                    sites = site
                continue
            times.append(t_trav)
        res[up] = n_sample * et.n_internal / float(np.median(times))
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
        "sample": (f"{n_sample} patterns of the same workload ({et.n_tips} taxa, I={et.n_internal}); "
                   f"oracle/oracle.cpp computeSubtreeLikelihood restatement, g++ -O2 -g, usePatterns=true "
                   f"(reference default); median of {runs} traversals after 1 warm-up on 1 pinned core"),
        "host_cpu": cpu,
        "value_use_patterns_false": res[False],
        "parity_vs_oracle": parity,
    }


FP64_PEAK_TFS = 78.6   # MI355X fp64 peak, vector and matrix alike (AMD spec sheet; the guide lists no fp64 row)
RIDGE = FP64_PEAK_TFS * 1e12 / (HBM_PEAK_GBS * 1e9)  # flop/B
TRAFFIC_FILES = ("profiles/r06/final/traffic.json", "profiles/r05/close/traffic.json", "profiles/r05/final/traffic.json", "profiles/r04/final/traffic.json", "profiles/r03/final/traffic.json", "profiles/r03/traffic.json", "profiles/r02/traffic.json", "profiles/traffic.json")


def measured_traffic(config, mode, P):
    """HBM bytes per traversal (traversal + table launches) from the committed PMC passes
    (keyed config/mode), rescaled to this run's pattern count."""
    for rel in TRAFFIC_FILES:
        try:
            tr = json.load(open(os.path.join(ROOT, rel))).get(f"{config}/{mode}")
        except Exception:
            tr = None
        if tr:
            return tr["hbm_bytes_per_traversal"] * P / tr["patterns"], tr["source"]
    return None, None


def roofline(wl, mode, P, ev_steps, tm, work, traffic):
    """Roofline of one traversal: the traversal launches plus the table builds that feed
    them (cherry_table_kernel), timed with HIP events on the handle's stream.

    achieved: SURVEY 8(d)'s algorithmic work per traversal (flops for the fused lnL-only
    traversal, which keeps interior partials in registers and is fp64 bound; bytes for
    the materialising paths, which stream every partial through HBM) / traversal time.
    executed: the fp64 flops the kernels actually issue, counted from the program that
    ran (plk_traversal_work) -- lower than algorithmic where cherries are table lookups,
    higher where MFMA tiles carry padding rows (20 states in 32-row tiles).
    hbm: the bytes the kernels really move (PMC FETCH/WRITE, profiles/) / traversal time.
    algorithmic_bytes_equiv: SURVEY 8(d)'s materialised-partials byte basis as a rate --
    an equivalence, not a hardware rate, for the fused traversal (it never moves them)."""
    part_ms, tab_ms = tm["partials_ms"], tm.get("tables_ms", 0.0)
    if part_ms <= 0:
        return None
    t_s = (part_ms + tab_ms) * 1e-3 / ev_steps
    launches = tm["launches"] / ev_steps
    bytes_pattern = wl.algorithmic_bytes_per_pattern()
    flops_pattern = wl.algorithmic_flops_per_pattern()
    alg_flops = flops_pattern * P
    alg_bytes = bytes_pattern * P
    fused = mode == "lnl"
    if mode == "materialize" and wl.S == 4 and wl.C in (1, 2, 4):
        # the fused traversal writing every partial: children come from registers, so the
        # bytes are the writes (8*C*S per internal node) plus codes, weight and site lnL
        alg_bytes = (8 * wl.C * wl.S * wl.et.n_internal + wl.et.n_tips + 16) * P
    subtree = mode == "subtree"
    if subtree and traffic:
        # per-subtree compression: the work is the distinct patterns per node, which depends
        # on the data, so the bytes the compressed traversal moves (PMC) are the basis
        alg_bytes = traffic
    if traffic:
        compute_bound = alg_flops / traffic > RIDGE and not subtree
    else:
        compute_bound = fused
    ex = None
    if work:
        issued = work["issued_flops"] + work["table_flops"]
        ex = {"useful_flops_per_traversal": work["useful_flops"], "issued_flops_per_traversal": work["issued_flops"],
              "table_flops_per_traversal": work["table_flops"],
              "achieved": issued / t_s / 1e12, "unit": "TFLOP/s", "frac": issued / t_s / 1e12 / FP64_PEAK_TFS,
              "useful_frac": (work["useful_flops"] + work["table_flops"]) / t_s / 1e12 / FP64_PEAK_TFS,
              "counted_from_program": bool(work["exact"])}
    hbm = None
    if traffic:
        g = traffic / t_s / 1e9
        hbm = {"achieved": g, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": g / HBM_PEAK_GBS,
               "bytes_per_traversal": traffic}
    if compute_bound:
        # 4 states: the fused traversal issues v_fma_f64 on the VALU (north_star keeps MFMA for
        # the dense 20 / 61-state contractions); 20 / 64 states: v_mfma_f64 on the matrix cores.
        # MI355X's fp64 peak is the same 78.6 TF/s for both pipes.
        unit_name = "valu" if wl.S == 4 else "mfma"
        main = {"bound": unit_name, "achieved": alg_flops / t_s / 1e12, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                "basis": (f"algorithmic {flops_pattern} flop/pattern/traversal = 2*C*S^2 per internal child + "
                          f"(k-1)*C*S per combine ({flops_pattern / wl.et.n_internal:.1f} flop/update) x {P} "
                          f"patterns / traversal time ({launches:.0f} traversal launch(es) + table builds, HIP "
                          f"events); peak = fp64 spec ({'VALU v_fma_f64' if wl.S == 4 else 'MFMA v_mfma_f64'}; "
                          f"vector = matrix on MI355X)")}
    else:
        main = {"bound": "hbm", "achieved": alg_bytes / t_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "basis": (f"algorithmic {alg_bytes / P:.0f} B/pattern/traversal x {P} patterns / traversal time "
                          f"({launches:.0f} launch(es), HIP events)")}
        if subtree and traffic:
            main["basis"] = (f"bytes the compressed traversal moves ({alg_bytes / P:.0f} B/pattern, PMC "
                             f"FETCH/WRITE) / traversal time ({launches:.0f} launch(es), HIP events); the "
                             f"uncompressed basis ({bytes_pattern} B/pattern) would exceed the HBM peak -- "
                             f"compression skips that work, see value (effective)")
    main["frac"] = main["achieved"] / main["peak"]
    main["traffic"] = traffic
    main["traversal_ms"] = t_s * 1e3
    main["launch_ms"] = part_ms / tm["launches"]
    main["table_ms_per_traversal"] = tab_ms / ev_steps
    main["executed"] = ex
    main["hbm"] = hbm
    if compute_bound:
        main["algorithmic_bytes_equiv"] = {
            "GB/s": bytes_pattern * P / t_s / 1e9,
            "note": (f"SURVEY 8(d) byte basis {bytes_pattern} B/pattern (every partial written and read once) "
                     f"as a rate; the fused traversal does not move these bytes (see hbm), so this is an "
                     f"equivalence, not a fraction of the HBM peak")}
    return main


def _json_stdout():
    """The one JSON line goes to the process's real stdout; everything else written to fd 1
    (RCCL's version banner, gloo's connection messages, library prints) is sent to stderr, so
    that stdout under torch.distributed.run carries exactly rank 0's line."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


class LaunchError(SystemExit):
    """Bad --gpus / --devices / launcher combination: exit non-zero before any GPU call."""

    def __init__(self, msg: str):
        print(f"bench.py: {msg}", file=sys.stderr, flush=True)
        super().__init__(2)


def launch_layout(args):
    """How the N GPUs are driven.  Under torch.distributed.run (WORLD_SIZE set): one rank
    per GPU, WORLD_SIZE must equal --gpus.  Without a launcher and --gpus N > 1: ONE process
    over devices 0..N-1 (or --devices) through one plk_create_multi handle, which shards the
    patterns in contiguous 4096-aligned ranges, launches every device before the first wait
    and sums the block sums in global order (bitwise one device).  Never silently fewer GPUs."""
    world_env = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env:
        if args.devices:
            raise LaunchError("--devices is the one-process multi-device mode; not under torch.distributed.run")
        if world != args.gpus:
            raise LaunchError(f"WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU")
        return {"kind": "ranks", "world": world, "devices": None}
    devices = None
    if args.devices:
        devices = [int(x) for x in args.devices.split(",") if x.strip() != ""]
        if len(devices) != args.gpus:
            raise LaunchError(f"--devices lists {len(devices)} device(s) for --gpus {args.gpus}")
    elif args.gpus > 1:
        n = plk.device_count()
        if args.gpus > n:
            raise LaunchError(f"--gpus {args.gpus} but only {n} GPU(s) visible")
        devices = list(range(args.gpus))
    if args.gpus < 1:
        raise LaunchError("--gpus must be >= 1")
    return {"kind": "multi" if devices and len(devices) > 1 else "single", "world": 1, "devices": devices}


def single_device(lay) -> int:
    """The device of a one-GPU, one-process run: --gpus 1 --devices K runs on device K (never
    silently device 0)."""
    return lay["devices"][0] if lay["kind"] == "single" and lay["devices"] else 0


def measure(args, lay, ctx, config, scaling, patterns=None, classes=None, mode="lnl", steps=None, warmup=None):
    """Set up one workload over the launch layout and time `steps` evaluations bracketed by
    a barrier + device synchronisation on both sides (max over ranks).  Returns the record
    pieces; `value` = the job's P x I per step x steps / time."""
    import torch

    dist, rank, world = ctx["dist"], ctx["rank"], lay["world"]
    rehearse = ctx["rehearse"]
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    wl = workload.make_workload(config, n_classes=classes)
    cfg = workload.CONFIGS[config]
    P_arg = patterns or (cfg.get("global_patterns", wl.n_patterns) if scaling == "strong" else wl.n_patterns)
    n_gpu = args.gpus
    if lay["kind"] == "ranks":
        start, end, P_job = shard.bench_range(scaling, rank, world, P_arg)
        device = ctx["device"]
        P_timed = end - start          # the patterns of the handle whose kernels are timed
    else:
        P_job = P_arg * n_gpu if scaling == "weak" else P_arg
        start, end = 0, P_job
        device = lay["devices"] if lay["kind"] == "multi" else single_device(lay)
        P_timed = shard.shard_range(0, n_gpu, P_job)[1] if lay["kind"] == "multi" else P_job
    wl.n_patterns = end - start
    t_setup = time.time()
    extra = {"lnl": plk.PLK_FLAG_LNL_ONLY, "materialize": 0, "levelwise": plk.PLK_FLAG_LEVELWISE,
             "subtree": plk.PLK_FLAG_SUBTREE_PATTERNS}[mode]
    sim_dev = ("cpu" if args.sim_cpu == "torch" else None) if args.sim_cpu else \
        (f"cuda:{ctx['device']}" if torch.cuda.is_available() else None)
    ev = workload.Evaluator(wl, device, start, end, extra_flags=extra, sim_device=sim_dev)
    # the simulation's blocks go back to the device: with torch's cache holding them, every
    # libplk launch / wait call was measured 2-10 us slower (cfg2 step 0.171 vs 0.159 ms)
    torch.cuda.empty_cache()
    xchg = None
    if dist is not None and rehearse:
        # one GPU, every rank on cuda:0: RCCL cannot put two ranks on one device, so the
        # rehearsal exchanges the block sums through torch.distributed (gloo)
        xchg = shard.BlockExchange(dist, ev.n_blocks, device=ctx["coll_dev"])
    elif dist is not None:
        # the RCCL communicator inside the handle (plk_comm_init): plk_evaluate all-gathers
        # every rank's block sums on the engine's stream and returns the global lnL
        cid = torch.zeros(128, dtype=torch.uint8, device="cuda")
        if rank == 0:
            cid.copy_(torch.frombuffer(bytearray(plk.comm_get_id()), dtype=torch.uint8))
        dist.broadcast(cid, 0)
        ev.eng.comm_init(world, rank, bytes(cid.cpu().numpy()))
    t_setup = time.time() - t_setup

    def one_step():
        lnl, _, blocks = ev.step()
        if xchg is None:
            return lnl  # global: plk_evaluate summed every rank's / device's block sums in global order
        return xchg.lnl(blocks)

    if dist is not None and not rehearse:
        # check the in-handle exchange once against torch.distributed's all-gather of the
        # same per-rank block sums (bitwise), before anything is timed
        lnl0, _, blocks0 = ev.step()
        ref = shard.BlockExchange(dist, ev.n_blocks, device=ctx["coll_dev"]).lnl(blocks0)
        if ref != lnl0:
            raise RuntimeError(f"rank {rank}: in-handle RCCL lnL {lnl0!r} != torch all-gather {ref!r}")
    lnl = None
    clk = args.clock_json and steps == args.steps   # (the main measurement, not the strong sub-record)
    step_ms = []
    for _ in range(warmup):
        tw = time.perf_counter()
        lnl = one_step()
        step_ms.append((time.perf_counter() - tw) * 1e3)
    ev.eng.reset_timing()
    # HIP events around the traversal launches and their table builds only (each timed
    # launch adds an event pair), on every K-th timed step: the kernels' mean durations are
    # sampled inside the timed region without charging every step the events' stream time
    k_ev = max(1, args.event_every)
    mask = 0 if args.no_events else (plk.PLK_TIME_PARTIALS | plk.PLK_TIME_TABLES)
    ev_steps = 0
    if dist is not None:
        dist.barrier()
    ev.eng.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        if i % k_ev == 0:
            ev.eng.set_timing(mask)
            ev_steps += 1
        elif k_ev > 1 and i % k_ev == 1:
            ev.eng.set_timing(0)
        if clk:
            tw = time.perf_counter()
            lnl = one_step()
            step_ms.append((time.perf_counter() - tw) * 1e3)
        else:
            lnl = one_step()
    if dist is not None:
        dist.barrier()
    ev.eng.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tm = ev.eng.get_timing()
    ev.eng.set_timing(False)
    if clk and rank == 0:
        rec = ev.eng.clock_records()
        n_pre = len(rec) - warmup - steps     # the exchange check's evaluation, if any
        with open(args.clock_json, "w") as f:
            json.dump({"config": config, "warmup": warmup, "steps": steps, "elapsed_ms": elapsed * 1e3,
                       "fields": ["shader_MHz_all_workgroups", "slowest_wg_MHz", "fastest_wg_MHz",
                                  "traversal_span_us", "workgroups", "host_step_ms", "phase"],
                       "evaluations": [list(map(float, r)) + [step_ms[i - n_pre] if i >= n_pre else None,
                                                               "check" if i < n_pre else
                                                               "warmup" if i < n_pre + warmup else "timed"]
                                       for i, r in enumerate(rec)]}, f, indent=1)
    if os.environ.get("PLK_DEBUG_HOST"):
        ev.eng.reset_timing()
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device=ctx["coll_dev"])
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    units_step = P_job * wl.et.n_internal   # the whole job's node updates per step
    fan = ev.eng.fanout() if lay["kind"] == "multi" else None
    return {"wl": wl, "ev": ev, "P": P_timed, "P_job": P_job, "lnl": lnl, "elapsed": elapsed, "tm": tm, "fanout": fan,
            "ev_steps": ev_steps, "k_ev": k_ev, "steps": steps, "units_step": units_step, "t_setup": t_setup,
            "value": units_step * steps / elapsed, "ms_step": elapsed * 1e3 / steps}


def parallelism(lay, args) -> str:
    if lay["kind"] == "ranks":
        return f"pattern-shard x{lay['world']}"
    if lay["kind"] == "multi":
        return f"multi-device x{args.gpus}"
    return "pattern-shard x1"


def main():
    args = parse()
    lay = launch_layout(args)
    out = _json_stdout()
    world = lay["world"]
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    use_dist = lay["kind"] == "ranks" and (world > 1 or args.force_dist)
    rehearse = use_dist and args.dist_backend == "gloo"
    if use_dist:
        import torch.distributed as dist  # noqa: F811
        if rehearse:
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(single_device(lay))
    device = local if use_dist and not rehearse else single_device(lay)
    ctx = {"dist": dist, "rank": rank, "rehearse": rehearse, "device": device,
           "coll_dev": "cpu" if rehearse else "cuda"}

    m = measure(args, lay, ctx, args.config, args.scaling, patterns=args.patterns, classes=args.classes,
                mode=args.mode)
    wl, ev, P, P_job, tm, ev_steps, k_ev = m["wl"], m["ev"], m["P"], m["P_job"], m["tm"], m["ev_steps"], m["k_ev"]
    rec = None
    if rank == 0:
        work = ev.eng.traversal_work()
        traffic, traffic_src = measured_traffic(args.config, args.mode, P)
        roof = roofline(wl, args.mode, P, ev_steps, tm, work, traffic) if not args.no_events else None
        if roof:
            roof["event_sample"] = f"HIP events on {ev_steps} of {args.steps} timed steps (every {k_ev})"
            if traffic_src:
                roof["traffic_source"] = traffic_src
            if lay["kind"] == "multi":
                roof["timed_shard"] = f"device {lay['devices'][0]} (shard 0 of {args.gpus}, {P} patterns)"
        computed = work["node_updates"]
        rec = {
            "metric": "site-pattern x node partial updates/s",
            "value": m["value"],
            "unit": "updates/s",
            "n_gpus": args.gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": m["ms_step"],
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded counter-based simulation under the model, 1 pattern = 1 column)",
            "config": {
                "workload": (f"{args.config}: {wl.models[0].name}{'+G%d' % wl.C if wl.C > 1 else ''} "
                             f"{wl.alphabet.name}, {P_job} patterns in total ({P} on GPU 0), "
                             f"{wl.et.n_tips}-taxon balanced tree "
                             f"({'rooted' if wl.model_of_node is not None else 'unrooted'}, I={wl.et.n_internal})"),
                "patterns_per_gpu": P,
                "patterns_total": P_job,
                "taxa": wl.et.n_tips,
                "internal_nodes": wl.et.n_internal,
                "states": wl.S,
                "classes": wl.C,
                "mode": args.mode,
                "parallelism": parallelism(lay, args),
            },
            "lnl": m["lnl"],
            "kernel_path": ev.eng.kernel_path(),
            # node updates the kernels compute per pattern (cherry-table nodes and
            # per-subtree compression are lookups / skipped) -- value above is the
            # reference-equivalent ("effective") rate
            "computed_updates_per_step": computed * P_job / P,
            "computed_updates_per_s": computed * P_job / P * args.steps / m["elapsed"],
            "table_nodes": work["table_nodes"],
            "partials_only_updates_per_s": (P * wl.et.n_internal * ev_steps / (tm["partials_ms"] * 1e-3)
                                            if tm["partials_ms"] > 0 else None),
            "kernel_ms_per_step": {"partials": tm["partials_ms"] / max(ev_steps, 1),
                                   "tables": tm["tables_ms"] / max(ev_steps, 1),
                                   "pmatrix": tm["pmat_ms"] / max(ev_steps, 1),
                                   "root": tm["root_ms"] / max(ev_steps, 1)},
            "partials_launches_per_step": tm["launches"] / max(ev_steps, 1),
            # host side of plk_evaluate per evaluation (us): P(t) launch call, traversal launch
            # call, block-sum launch call, completion wait, host sum, caller between evaluations
            "host_us_per_eval": ({k: round(v / tm["evaluations"], 2) for k, v in
                                  zip(("pmat_call", "traversal_call", "blocks_call", "wait", "sum", "caller"),
                                      tm["host_us"])} if tm.get("evaluations") else None),
            "table_launches_per_step": tm["table_launches"] / max(ev_steps, 1),
            "roofline": roof,
            "setup_s": m["t_setup"],
        }
        if m["fanout"]:
            # host fan-out of the multi-device handle over the timed steps (plk_get_fanout): per shard
            # the mean offsets from posting an evaluation to its worker starting, its traversal
            # launch call returning and its completion wait returning
            rec["fanout"] = m["fanout"]
        if args.devices:
            rec["config"]["devices"] = args.devices
            if len(set(lay["devices"])) < len(lay["devices"]):
                rec["rehearsal"] = (f"devices {args.devices}: several shards share a GPU -- the multi-device "
                                    f"path exercised, not an {args.gpus}-GPU measurement")
        if args.mode == "subtree":
            rec["metric"] += " (EFFECTIVE: per-subtree pattern compression)"
        if world == 1 and lay["kind"] == "single" and not args.no_cpu_baseline:
            ns = args.cpu_sample or workload.CONFIGS[args.config]["cpu_sample"]
            _, eng_sites, _ = ev.eng.root_loglik(wl.et.root, want_sites=True)
            rec["cpu_baseline"] = cpu_baseline(wl, min(ns, P), args.cpu_runs, eng_sites)
    ev.eng.close()
    del m, ev
    if not args.no_strong and args.scaling == "weak" and args.config == "gtr_g4_dna_1M_64":
        # the strong-scaling curve BASELINE config 5 names, from the same sweep: config 5's 2M
        # patterns split over the same N GPUs, timed the same way (the N = 1 line is all 2M on
        # one GPU), so the driver's N = 1, 2, 4, 8 lines carry both curves
        s = measure(args, lay, ctx, "nh_gtr_g4_dna_2M_512", "strong", patterns=args.strong_patterns,
                    steps=args.strong_steps, warmup=5)
        if rank == 0:
            trav = (s["tm"]["partials_ms"] + s["tm"]["tables_ms"]) / max(s["ev_steps"], 1)
            flops = s["wl"].algorithmic_flops_per_pattern() * s["P"]
            rec["strong"] = {
                "config": "nh_gtr_g4_dna_2M_512 (BASELINE config 5): NH-GTR+G4 DNA, 512-taxon rooted tree, "
                          f"I={s['wl'].et.n_internal}, {s['P_job']} patterns split over {args.gpus} GPU(s)",
                "scaling": "strong",
                "n_gpus": args.gpus,
                "value": s["value"],
                "unit": "updates/s",
                "ms_per_step": s["ms_step"],
                "steps": s["steps"],
                "patterns_total": s["P_job"],
                "patterns_per_gpu": s["P"],
                "kernel_path": s["ev"].eng.kernel_path(),
                "traversal_ms": trav,
                "traversal_frac_fp64": (flops / (trav * 1e-3) / 1e12 / FP64_PEAK_TFS) if trav > 0 else None,
                "lnl": s["lnl"],
                "setup_s": s["t_setup"],
            }
            if s["fanout"]:
                rec["strong"]["fanout"] = s["fanout"]
        s["ev"].eng.close()
    if rank == 0:
        print(json.dumps(rec), file=out, flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
