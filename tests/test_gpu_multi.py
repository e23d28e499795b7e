"""Multi-GPU at the C-ABI boundary, on the one-GPU test box.

  - plk_create_multi: one process, several devices.  Listing device 0 twice gives two
    shards on one GPU, which exercises everything the handle does for several GPUs --
    block-aligned pattern ranges, sliced tip codes / weights / per-pattern outputs,
    launches on every shard before the first wait, the global fixed-order block sum --
    except the devices being different.  Results must equal one handle BITWISE (lnL,
    block sums, per-pattern lnL, partials) for every kernel path.
  - plk_comm_init: the RCCL communicator inside a handle (one process per GPU).  With one
    rank the all-gather + device-side fixed-order sum must return the single-handle lnL
    bitwise; multi-rank runs happen in bench.py --gpus N on a multi-GPU node.
  - the Bio++ mirror sharded through BPP_AMD_DEVICES reproduces the reference goldens.
"""
import os
import subprocess

import numpy as np
import pytest

import phylo
import plk
import workload
from conftest import run_make

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(eng, wl, states):
    eng.set_code_table(wl.alphabet.init_table)
    for i in range(wl.et.n_tips):
        eng.set_tip_codes(i, phylo.states_to_codes(states[i]))
    eng.set_category_rates(wl.rates, wl.probs)
    eng.set_root_frequencies(wl.root_freqs)
    for k, m in enumerate(wl.models):
        eng.set_eigen(k, m.V, m.Vinv, m.lam)
    return eng


@pytest.mark.parametrize("config,n,flags,devs", [
    ("gtr_g4_dna_1M_64", 3 * 4096 + 100, plk.PLK_FLAG_LNL_ONLY, [0, 0]),
    ("gtr_g4_dna_1M_64", 5 * 4096, 0, [0, 0, 0]),
    ("lg08_g4_protein_200k_256", 2 * 4096 + 7, plk.PLK_FLAG_LNL_ONLY, [0, 0]),
    ("yn98_codon_50k_128", 4096 + 50, plk.PLK_FLAG_LNL_ONLY, [0, 0]),
    ("nh_gtr_g4_dna_2M_512", 3 * 4096, plk.PLK_FLAG_LNL_ONLY, [0, 0, 0]),
    ("gtr_g4_dna_1M_64", 2 * 4096, plk.PLK_FLAG_LEVELWISE, [0, 0])])
def test_multi_device_handle_bitwise(config, n, flags, devs):
    wl = workload.make_workload(config, n_patterns=n)
    et = wl.et
    states = wl.simulate(0, n)
    base = (plk.PLK_FLAG_SCALING if wl.scaling else 0) | (plk.PLK_FLAG_NONNEG_GUARD if wl.guard else 0) | flags
    one = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, len(wl.models), base), wl, states)
    multi = _setup(plk.Engine(devs, wl.S, wl.C, n, et.n_tips, et.n_internal, len(wl.models), base), wl, states)
    assert multi.shard_count() == min(len(devs), (n + 4095) // 4096)
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    mi = None if wl.model_of_node is None else wl.model_of_node[br].astype(np.int32)
    ops = phylo.split_ops(et.ops)
    w = np.random.default_rng(3).integers(1, 5, size=n).astype(np.float64)
    one.set_pattern_weights(w)
    multi.set_pattern_weights(w)
    for scale in (1.0, 0.8):
        t = et.brlen[br] * scale
        l1, b1 = one.evaluate(br, t, ops, et.root, mi)
        lm, bm = multi.evaluate(br, t, ops, et.root, mi)
        assert l1 == lm and np.array_equal(b1, bm)
    r1 = one.root_loglik(et.root, want_sites=True, want_blocks=True)
    rm = multi.root_loglik(et.root, want_sites=True, want_blocks=True)
    assert r1[0] == rm[0] and np.array_equal(r1[1], rm[1]) and np.array_equal(r1[2], rm[2])
    node = et.ops[len(et.ops) // 2][0]
    assert np.array_equal(one.get_partials(node), multi.get_partials(node))
    assert multi.kernel_path() == one.kernel_path()
    w1, wm = one.traversal_work(), multi.traversal_work()
    assert wm["patterns"] == n and wm["node_updates"] == w1["node_updates"]


def test_shard_request_staging_after_allocation_churn():
    """The round-4 -inf shard (profiles/r05/ab_runs.md): a fresh shard handle's
    P(t) request, staged in host-written device memory, read back as other data after many
    device buffers had been freed and the caches thrashed (tools/micro/l2_stale.hip
    reproduces it).  The staging is pinned host memory now; here the same conditions -- 48
    handles with their buffers created and destroyed, a 1.6 GB write -- come before fresh
    two- and three-shard handles whose 1 022-branch requests take the staging path, and
    their lnL and block sums must equal one handle's bitwise, evaluation after evaluation."""
    n = 3 * 4096 + 9
    wl = workload.make_workload("nh_gtr_g4_dna_2M_512", n_patterns=n)
    et = wl.et
    states = wl.simulate(0, n)
    base = plk.PLK_FLAG_SCALING | plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    mi = wl.model_of_node[br].astype(np.int32)
    ops = phylo.split_ops(et.ops)
    for k in range(48):  # freed device buffers of many sizes, with kernels' data in them
        m = 4096 * (1 + k % 5)
        e = _setup(plk.Engine(0, wl.S, wl.C, m, et.n_tips, et.n_internal, len(wl.models), base), wl,
                   wl.simulate(k, k + m))
        e.evaluate(br, et.brlen[br] * (1.0 + 0.01 * k), ops, et.root, mi)
        e.close()
    # a cache thrash: a materialising 64-taxon traversal writes 62 partials x 200k x 128 B
    wl2 = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=200_000)
    big = _setup(plk.Engine(0, 4, 4, 200_000, wl2.et.n_tips, wl2.et.n_internal, 1, plk.PLK_FLAG_NONNEG_GUARD), wl2,
                 wl2.simulate(0, 200_000))
    br2 = np.array([v for v in range(wl2.et.n_nodes) if v != wl2.et.root], dtype=np.int32)
    big.evaluate(br2, wl2.et.brlen[br2], phylo.split_ops(wl2.et.ops), wl2.et.root)
    big.close()
    one = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, len(wl.models), base), wl, states)
    for devs in ([0, 0], [0, 0, 0]):
        multi = _setup(plk.Engine(devs, wl.S, wl.C, n, et.n_tips, et.n_internal, len(wl.models), base), wl, states)
        for scale in (1.0, 0.7, 1.3):
            t = et.brlen[br] * scale
            l1, b1 = one.evaluate(br, t, ops, et.root, mi)
            lm, bm = multi.evaluate(br, t, ops, et.root, mi)
            assert np.isfinite(lm) and l1 == lm and np.array_equal(b1, bm)
        multi.close()


def test_multi_device_branch_derivatives():
    wl = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=2 * 4096 + 11)
    et, n = wl.et, wl.n_patterns
    states = wl.simulate(0, n)
    one = _setup(plk.Engine(0, 4, 4, n, et.n_tips, et.n_internal, 1), wl, states)
    multi = _setup(plk.Engine([0, 0], 4, 4, n, et.n_tips, et.n_internal, 1), wl, states)
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    for e in (one, multi):
        e.update_pmatrices(br, et.brlen[br], deriv_mask=7)
        e.update_partials(phylo.split_ops(et.ops))
        e.root_loglik(et.root)
    for b in (0, et.n_tips, br[-1]):
        a1, a2 = one.branch_derivatives(int(b))
        m1, m2 = multi.branch_derivatives(int(b))
        assert abs(a1 - m1) <= 1e-12 * abs(a1) and abs(a2 - m2) <= 1e-12 * abs(a2)


@pytest.mark.parametrize("config,flags", [("gtr_g4_dna_1M_64", plk.PLK_FLAG_LNL_ONLY),
                                          ("lg08_g4_protein_200k_256", plk.PLK_FLAG_LNL_ONLY),
                                          ("gtr_g4_dna_1M_64", plk.PLK_FLAG_LEVELWISE)])
def test_comm_single_rank_bitwise(config, flags):
    """plk_comm_init with one rank: the RCCL all-gather and the device-side fixed-order sum
    return the handle's own host-side sum bitwise, evaluation after evaluation."""
    n = 3 * 4096 + 21
    wl = workload.make_workload(config, n_patterns=n)
    et = wl.et
    states = wl.simulate(0, n)
    base = (plk.PLK_FLAG_SCALING if wl.scaling else 0) | plk.PLK_FLAG_NONNEG_GUARD | flags
    ref = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    eng = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    eng.comm_init(1, 0, plk.comm_get_id())
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    ops = phylo.split_ops(et.ops)
    for scale in (1.0, 1.2, 0.9):
        t = et.brlen[br] * scale
        l0, b0 = ref.evaluate(br, t, ops, et.root)
        l1, b1 = eng.evaluate(br, t, ops, et.root)
        assert l0 == l1 and np.array_equal(b0, b1)
    s0 = ref.root_loglik(et.root, want_sites=True)
    s1 = eng.root_loglik(et.root, want_sites=True)
    assert s0[0] == s1[0] and np.array_equal(s0[1], s1[1])
    if wl.S == 4:
        # derivatives are global under a communicator (all-gathered, summed in rank order):
        # at one rank they are the handle's own values bitwise
        for e in (ref, eng):
            e.update_pmatrices(br, et.brlen[br], deriv_mask=7)
            e.update_partials(ops)
            e.root_loglik(et.root)
        for b in (0, int(br[-1])):
            assert ref.branch_derivatives(b) == eng.branch_derivatives(b)


def test_comm_init_failure_leaves_single_rank_path(monkeypatch):
    """A failure after ncclCommInitRank (forced exchange-setup failure) releases the
    communicator and its buffers: later evaluations take the single-rank path and give the
    handle's own lnL, and plk_comm_init can be retried."""
    n = 2 * 4096 + 5
    wl = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=n)
    et = wl.et
    states = wl.simulate(0, n)
    base = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY
    ref = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    eng = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    monkeypatch.setenv("PLK_TEST_COMM_FAIL", "1")
    with pytest.raises(plk.PlkError):
        eng.comm_init(1, 0, plk.comm_get_id())
    monkeypatch.delenv("PLK_TEST_COMM_FAIL")
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    ops = phylo.split_ops(et.ops)
    l0, b0 = ref.evaluate(br, et.brlen[br], ops, et.root)
    l1, b1 = eng.evaluate(br, et.brlen[br], ops, et.root)
    assert l0 == l1 and np.array_equal(b0, b1)
    eng.comm_init(1, 0, plk.comm_get_id())
    l2, b2 = eng.evaluate(br, et.brlen[br], ops, et.root)
    assert l2 == l0 and np.array_equal(b2, b0)


@pytest.mark.skipif(plk.device_count() < 2, reason="distinct-device handles need two GPUs (the test box has one)")
@pytest.mark.parametrize("config,flags", [("gtr_g4_dna_1M_64", plk.PLK_FLAG_LNL_ONLY),
                                          ("lg08_g4_protein_200k_256", plk.PLK_FLAG_LNL_ONLY),
                                          ("gtr_g4_dna_1M_64", 0)])
def test_multi_device_distinct_gpus(config, flags):
    """plk_create_multi over two different GPUs: per-device JIT module, hipSetDevice
    discipline and per-device mapped staging -- lnL, block sums and branch derivatives equal
    one handle (bitwise / 1e-12)."""
    n = 3 * 4096 + 77
    wl = workload.make_workload(config, n_patterns=n)
    et = wl.et
    states = wl.simulate(0, n)
    base = (plk.PLK_FLAG_SCALING if wl.scaling else 0) | plk.PLK_FLAG_NONNEG_GUARD | flags
    one = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    multi = _setup(plk.Engine([0, 1], wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    ops = phylo.split_ops(et.ops)
    for scale in (1.0, 0.7):
        t = et.brlen[br] * scale
        l1, b1 = one.evaluate(br, t, ops, et.root)
        lm, bm = multi.evaluate(br, t, ops, et.root)
        assert l1 == lm and np.array_equal(b1, bm)
    for e in (one, multi):
        e.update_pmatrices(br, et.brlen[br] * 0.7, deriv_mask=7)
        e.update_partials(ops)
        e.root_loglik(et.root)
    for b in (0, et.n_tips, br[-1]):
        a1, a2 = one.branch_derivatives(int(b))
        m1, m2 = multi.branch_derivatives(int(b))
        assert abs(a1 - m1) <= 1e-12 * abs(a1) and abs(a2 - m2) <= 1e-12 * abs(a2)


def test_cpp_drop_in_sharded_goldens():
    """The Bio++ mirror's drop-in program with the patterns sharded over two handles on the
    GPU (BPP_AMD_DEVICES=0,0): the reference goldens, optimisers included."""
    host = os.path.join(ROOT, "bpp-phyl_amd", "host")
    run_make("-s", "-j8", "-C", host)
    env = dict(os.environ, BPP_AMD_DEVICES="0,0")
    r = subprocess.run([os.path.join(host, "bin", "test_likelihood_gpu")], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout


def _bench_line(*extra):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--patterns", "50000", "--strong-patterns", "40000", "--strong-steps", "2",
                        "--no-cpu-baseline", *extra], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus2_one_process_rehearsal():
    """bench.py --gpus 2 without a launcher: one process, one plk_create_multi handle over the
    devices (here --devices 0,0, two shards on the one GPU of this box): the line says
    n_gpus 2, multi-device x2, marks the rehearsal, and its config-5 strong sub-record gives the
    1-GPU lnL bitwise (the same 40 000 patterns split over two shards)."""
    one = _bench_line("--gpus", "1")
    two = _bench_line("--gpus", "2", "--devices", "0,0")
    assert one["n_gpus"] == 1 and one["config"]["parallelism"] == "pattern-shard x1" and "rehearsal" not in one
    assert two["n_gpus"] == 2 and two["config"]["parallelism"] == "multi-device x2" and "rehearsal" in two
    assert two["config"]["patterns_total"] == 100000 and two["config"]["patterns_per_gpu"] == 53248
    assert one["strong"]["n_gpus"] == 1 and two["strong"]["n_gpus"] == 2
    assert one["strong"]["patterns_total"] == two["strong"]["patterns_total"] == 40000
    assert one["strong"]["lnl"] == two["strong"]["lnl"]
    assert one["kernel_path"] == two["kernel_path"] == "jit_tree4"


def test_multi_device_fanout_eight_shards():
    """Eight shards of one plk_create_multi handle (all on the one GPU of this box): every
    shard runs on its own host worker; lnL and block sums equal one handle bitwise evaluation
    after evaluation, derivatives agree, and plk_get_fanout reports every shard's offsets."""
    n = 8 * 4096 + 123
    wl = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=n)
    et = wl.et
    states = wl.simulate(0, n)
    base = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY
    one = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    multi = _setup(plk.Engine([0] * 8, wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    assert multi.shard_count() == 8
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    ops = phylo.split_ops(et.ops)
    multi.reset_timing()
    for k in range(12):
        t = et.brlen[br] * (1.0 + 0.05 * k)
        l1, b1 = one.evaluate(br, t, ops, et.root)
        lm, bm = multi.evaluate(br, t, ops, et.root)
        assert l1 == lm and np.array_equal(b1, bm)
    f = multi.fanout()
    assert f["evaluations"] == 12 and len(f["traversal_launched_us"]) == 8
    assert all(0.0 <= a <= b <= c for a, b, c in zip(f["start_us"], f["traversal_launched_us"], f["waited_us"]))
    assert 0.0 <= f["launch_spread_mean_us"] <= f["launch_spread_max_us"]
    assert one.fanout()["evaluations"] == 0
    r1 = one.root_loglik(et.root, want_sites=True, want_blocks=True)
    rm = multi.root_loglik(et.root, want_sites=True, want_blocks=True)
    assert r1[0] == rm[0] and np.array_equal(r1[1], rm[1]) and np.array_equal(r1[2], rm[2])
    for e in (one, multi):
        e.update_pmatrices(br, et.brlen[br], deriv_mask=7)
        e.update_partials(ops)
        e.root_loglik(et.root)
    for b in (0, et.n_tips, int(br[-1])):
        a1, a2 = one.branch_derivatives(b)
        m1, m2 = multi.branch_derivatives(b)
        assert abs(a1 - m1) <= 1e-12 * abs(a1) and abs(a2 - m2) <= 1e-12 * abs(a2)


def _random_sharded_problem(seed):
    """A random unbalanced tree (polytomies, rooted or unrooted), 1-3 GTR / LG08 / YN98 models,
    1-4 classes, rescaling or not, a traversal mode, 1-3 blocks of 4096 patterns and a few."""
    from test_gpu_parity import MODES, _random_topology
    rng = np.random.default_rng(5000 + seed)
    S = 20 if seed % 4 == 3 else 64 if seed % 8 == 5 else 4
    C = 1 if S == 64 else int(rng.choice([1, 2, 4]))
    n = int(rng.choice([4096 + 1, 2 * 4096 + 333, 3 * 4096 + 17]))
    devs = [0, 0] if rng.random() < 0.5 else [0, 0, 0]
    scaling = bool(rng.random() < 0.4)
    lo, hi = (0.3, 1.2) if scaling else (0.01, 0.3)
    et = phylo.engine_tree(_random_topology(int(rng.integers(4, 24 if S == 64 else 60)), rng, lo, hi),
                           unroot=bool(rng.random() < 0.5))
    n_models = int(rng.integers(1, 4))
    if S == 4:
        models = [phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5)) for _ in range(n_models)]
        alph = phylo.DNA
    elif S == 20:
        models, alph = [phylo.lg08()] * n_models, phylo.PROTEIN
    else:
        models = [phylo.yn98(float(rng.uniform(1.0, 4.0)), float(rng.uniform(0.1, 1.0))) for _ in range(n_models)]
        alph = phylo.CODON
    mon = rng.integers(0, n_models, et.n_nodes).astype(np.int32) if n_models > 1 else None
    rates, probs = phylo.gamma_rates(C, float(rng.uniform(0.3, 2.0))) if C > 1 else (np.ones(1), np.ones(1))
    wl = workload.Workload("m", et, models, mon, rates, probs, models[0].pi, alph, n, scaling, True, seed)
    states = wl.simulate(0, n)
    mode = ["lnl_only", "materialize", "levelwise", "subtree"][seed % 4 if n_models == 1 else seed % 3]
    flags = plk.PLK_FLAG_NONNEG_GUARD | (plk.PLK_FLAG_SUBTREE_PATTERNS if mode == "subtree" else MODES[mode]) | \
        (plk.PLK_FLAG_SCALING if scaling else 0)
    return rng, S, C, n, devs, et, n_models, mon, wl, states, mode, flags


@pytest.mark.parametrize("seed", range(16))
def test_multi_device_random_topologies_incremental(seed):
    """Random unbalanced trees (polytomies, rooted or unrooted, 1-3 models, 4 / 20 / 64
    states) on two- and three-shard handles, every traversal mode: the sharded handle equals
    one handle bitwise (lnL, block sums, per-pattern lnL) after a full traversal and after
    incremental ones (the changed branches' P(t) and the ancestors' ops only), and the
    incremental result equals a full re-traversal bitwise."""
    rng, S, C, n, devs, et, n_models, mon, wl, states, mode, flags = _random_sharded_problem(seed)
    mk = lambda d: _setup(plk.Engine(d, S, C, n, et.n_tips, et.n_internal, n_models, flags), wl, states)  # noqa: E731
    one, multi = mk(0), mk(devs)
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    mi = None if mon is None else mon[br]
    ops = phylo.split_ops(et.ops)
    parents = {c: p for p, ch in et.ops for c in ch}
    bl = et.brlen.copy()

    def both(fn):
        r = [fn(e) for e in (one, multi)]
        for e in (one, multi):
            r.append(e.root_loglik(et.root, want_sites=True, want_blocks=True))
        (l1, b1), (lm, bm), s1, sm = r
        assert np.isfinite(l1) and l1 == lm and np.array_equal(b1, bm)
        assert s1[0] == l1 and sm[0] == lm and np.array_equal(s1[1], sm[1]) and np.array_equal(s1[2], sm[2])
        return l1

    both(lambda e: e.evaluate(br, bl[br], ops, et.root, mi))
    for _ in range(2):
        ch = rng.choice(br, size=min(2, len(br)), replace=False).astype(np.int32)
        bl[ch] *= rng.uniform(0.5, 1.5, size=len(ch))
        if mode == "lnl_only":  # nothing is stored: every call is a full traversal
            inc = both(lambda e: e.evaluate(br, bl[br], ops, et.root, mi))
        else:
            anc = set()
            for b in ch:
                v = int(b)
                while v in parents:
                    v = parents[v]
                    anc.add(v)
            sub = phylo.split_ops([(p, c) for p, c in et.ops if p in anc])
            inc = both(lambda e: e.evaluate(ch, bl[ch], sub, et.root, None if mon is None else mon[ch]))
        fresh = mk(0)
        full, _ = fresh.evaluate(br, bl[br], ops, et.root, mi)
        fresh.close()
        assert inc == full


@pytest.mark.parametrize("seed", range(8))
def test_comm_random_topologies(seed):
    """plk_comm_init at one rank on random trees (the sharded fuzz's problems): lnL, block
    sums and per-pattern lnL equal the handle without a communicator bitwise, after a full
    and an incremental evaluation, and -- where partials are stored -- so do the branch
    derivatives (all-gathered and summed in rank order)."""
    rng, S, C, n, devs, et, n_models, mon, wl, states, mode, flags = _random_sharded_problem(100 + seed)
    ref = _setup(plk.Engine(0, S, C, n, et.n_tips, et.n_internal, n_models, flags), wl, states)
    eng = _setup(plk.Engine(0, S, C, n, et.n_tips, et.n_internal, n_models, flags), wl, states)
    eng.comm_init(1, 0, plk.comm_get_id())
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    mi = None if mon is None else mon[br]
    ops = phylo.split_ops(et.ops)
    for scale in (1.0, 1.1):
        r = [e.evaluate(br, et.brlen[br] * scale, ops, et.root, mi) for e in (ref, eng)]
        assert np.isfinite(r[0][0]) and r[0][0] == r[1][0] and np.array_equal(r[0][1], r[1][1])
    s0, s1 = (e.root_loglik(et.root, want_sites=True) for e in (ref, eng))
    assert s0[0] == s1[0] and np.array_equal(s0[1], s1[1])
    if mode != "lnl_only" and mode != "subtree":
        for e in (ref, eng):
            e.update_pmatrices(br, et.brlen[br], mi, deriv_mask=7)
            e.update_partials(ops)
            e.root_loglik(et.root)
        for b in rng.choice(br, size=min(3, len(br)), replace=False):
            assert ref.branch_derivatives(int(b)) == eng.branch_derivatives(int(b))
