"""Row f4: double-recursive derivatives of every branch (plk_all_branch_derivatives,
PLK_FLAG_DOUBLE_RECURSIVE) -- the reference's DRHomogeneousTreeLikelihood
(Likelihood/DRHomogeneousTreeLikelihood.cpp:287-423, 543-651).

Checked against
  - the single-traversal path derivatives of the same engine (plk_branch_derivatives,
    themselves checked against central differences of the oracle in test_gpu_parity.py):
    relative 1e-10 on d1 and d2 (the reference's own R-vs-DR check is 1e-6 absolute,
    test/test_likelihood.cpp:122-135);
  - central differences of the CPU oracle for a few branches.
"""
import numpy as np
import pytest

import phylo
import plk
import workload

from test_gpu_parity import MODES, _caterpillar, _random_problem, engine_for, oracle_for, run_engine

pytestmark = pytest.mark.gpu

DR = plk.PLK_FLAG_DOUBLE_RECURSIVE


def _close(a, b, rel):
    return abs(a - b) <= rel * max(1.0, abs(a), abs(b))


def _dr_vs_path(eng, et, rel=1e-10):
    d1, d2 = eng.all_branch_derivatives()
    assert d1[et.root] == 0.0 and d2[et.root] == 0.0
    for b in range(et.n_nodes):
        if b == et.root:
            continue
        p1, p2 = eng.branch_derivatives(b)
        assert _close(d1[b], p1, rel), (b, d1[b], p1)
        assert _close(d2[b], p2, rel), (b, d2[b], p2)
    return d1, d2


@pytest.mark.parametrize("S,C,mode,scaling,n_taxa,n_pat", [
    (4, 4, "materialize", False, 16, 3000), (4, 1, "lnl_only", False, 9, 700), (4, 2, "levelwise", True, 12, 777),
    (4, 8, "materialize", False, 10, 300), (20, 4, "lnl_only", False, 10, 500), (20, 2, "levelwise", True, 12, 400),
    (64, 1, "lnl_only", False, 8, 300), (64, 2, "materialize", False, 6, 130), (4, 4, "lnl_only", False, 3, 1)])
def test_dr_equals_path_derivatives(S, C, mode, scaling, n_taxa, n_pat):
    et, m, alph, rates, probs, states = _random_problem(S, C, n_taxa, n_pat, seed=70 + S + C + n_taxa)
    flags = plk.PLK_FLAG_NONNEG_GUARD | MODES[mode] | DR | (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, S, C, n_pat, states, alph.init_table, rates, probs, m.pi, [m], flags=flags)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    _dr_vs_path(eng, et)


def test_dr_vs_oracle_finite_differences():
    et, m, alph, rates, probs, states = _random_problem(4, 4, 14, 900, seed=81)
    eng = engine_for(et, 4, 4, 900, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | DR)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    d1, d2 = eng.all_branch_derivatives()
    for b in (0, 3, et.n_tips, et.ops[0][0], br[-1]):
        def lnl_at(t):
            bl = et.brlen.copy()
            bl[b] = t
            e2 = phylo.EngineTree(et.n_tips, et.n_internal, et.root, et.tip_names, et.ops, bl, {}, [], [])
            return oracle_for(e2, states, alph.init_table, rates, probs, m.pi, [m])[0]

        t = et.brlen[b]
        fd1 = (lnl_at(t + 1e-5) - lnl_at(t - 1e-5)) / 2e-5
        fd2 = (lnl_at(t + 1e-4) - 2 * lnl_at(t) + lnl_at(t - 1e-4)) / 1e-8
        assert abs(d1[b] - fd1) <= 1e-6 * max(1.0, abs(fd1)), (b, d1[b], fd1)
        assert abs(d2[b] - fd2) <= 2e-4 * max(1.0, abs(fd2)), (b, d2[b], fd2)


def test_dr_polytomy_and_deep_caterpillar():
    # polytomies: U_v of a son of a 5-way node has 4 siblings + the father's U (ACCUMULATE chunks)
    t = phylo.Tree.from_newick("((a:0.1,b:0.2,c:0.05,d:0.3,e:0.12):0.1,(f:0.2,g:0.1):0.05,h:0.3,i:0.2);")
    et = phylo.engine_tree(t)
    m = phylo.gtr(1.2, 0.4, 0.6, 0.8, 0.5, 0.3, 0.2, 0.25, 0.25)
    rates, probs = phylo.gamma_rates(4, 0.5)
    wl = workload.Workload("p", et, [m], None, rates, probs, m.pi, phylo.DNA, 1000, False, True, 9)
    states = wl.simulate(0, 1000).astype(np.int32)
    eng = engine_for(et, 4, 4, 1000, states, phylo.DNA.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | DR)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    _dr_vs_path(eng, et)
    # a 300-taxon caterpillar drives the upper vectors through rescaling
    tree = _caterpillar(300, lo=0.1, hi=0.4)
    et = phylo.engine_tree(tree)
    wl = workload.Workload("c", et, [m], None, rates, probs, m.pi, phylo.DNA, 600, False, True, 5)
    states = wl.simulate(0, 600).astype(np.int32)
    eng = engine_for(et, 4, 4, 600, states, phylo.DNA.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_SCALING | DR)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    lnl, _, _ = run_engine(eng, et)
    assert lnl < -745 * 4
    d1, d2 = _dr_vs_path(eng, et, rel=1e-9)
    assert np.all(np.isfinite(d1)) and np.all(np.isfinite(d2))


def test_dr_nonhomogeneous_rooted():
    """NH trees stay rooted (2-son root); per-branch models."""
    wl = workload.make_workload("nh_gtr_g4_dna_2M_512", n_patterns=1500)
    et = wl.et
    states = wl.simulate(0, 1500).astype(np.int32)
    eng = engine_for(et, 4, 4, 1500, states, phylo.DNA.init_table, wl.rates, wl.probs, wl.root_freqs, wl.models,
                     model_of_node=wl.model_of_node, flags=plk.PLK_FLAG_SCALING | DR)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], np.asarray(wl.model_of_node)[br].astype(np.int32), deriv_mask=7)
    run_engine(eng, et)
    d1, d2 = eng.all_branch_derivatives()
    for b in (0, 1, et.n_tips, et.n_nodes - 2, int(br[len(br) // 2])):
        p1, p2 = eng.branch_derivatives(b)
        assert _close(d1[b], p1, 1e-9) and _close(d2[b], p2, 1e-9), (b, d1[b], p1, d2[b], p2)


def test_dr_after_incremental_traversal():
    """An incremental call lists only the ancestors of a changed branch; the engine keeps
    the tree of earlier calls, so every branch is still served."""
    et, m, alph, rates, probs, states = _random_problem(4, 4, 16, 800, seed=91)
    eng = engine_for(et, 4, 4, 800, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | DR)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    b = 2
    bl = et.brlen.copy()
    bl[b] *= 1.7
    eng.update_pmatrices(np.array([b], dtype=np.int32), bl[[b]], deriv_mask=7)
    parents = {c: p for p, ch in et.ops for c in ch}
    anc = set()
    n = b
    while n in parents:
        n = parents[n]
        anc.add(n)
    eng.update_partials(phylo.split_ops([(p, ch) for p, ch in et.ops if p in anc]))
    d1, _ = eng.all_branch_derivatives()
    # fresh engine on the changed lengths, full traversal
    et2 = phylo.EngineTree(et.n_tips, et.n_internal, et.root, et.tip_names, et.ops, bl, {}, [], [])
    eng2 = engine_for(et2, 4, 4, 800, states, alph.init_table, rates, probs, m.pi, [m],
                      flags=plk.PLK_FLAG_NONNEG_GUARD | DR)
    eng2.update_pmatrices(br, bl[br], deriv_mask=7)
    run_engine(eng2, et2)
    e1, _ = eng2.all_branch_derivatives()
    assert np.allclose(d1, e1, rtol=1e-12, atol=0)


def test_dr_errors():
    et, m, alph, rates, probs, states = _random_problem(4, 4, 6, 100, seed=3)
    eng = engine_for(et, 4, 4, 100, states, alph.init_table, rates, probs, m.pi, [m])
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    with pytest.raises(plk.PlkError) as ei:
        eng.all_branch_derivatives()  # no PLK_FLAG_DOUBLE_RECURSIVE
    assert ei.value.code == -5
    eng = engine_for(et, 4, 4, 100, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | DR)
    run_engine(eng, et)
    with pytest.raises(plk.PlkError) as ei:
        eng.all_branch_derivatives()  # dP / d2P missing
    assert ei.value.code == -5
    with pytest.raises(plk.PlkError) as ei:
        plk.Engine(0, 4, 4, 100, 6, 4, 1, DR | plk.PLK_FLAG_SUBTREE_PATTERNS)
    assert ei.value.code == -4


@pytest.mark.parametrize("S,C", [(4, 4), (20, 2)])
def test_path_derivatives_after_incremental_traversal(S, C):
    """plk_branch_derivatives on a branch outside the last (incremental) op list: the engine
    answers from the merged tree, equal to a fresh engine's full traversal."""
    et, m, alph, rates, probs, states = _random_problem(S, C, 16, 500, seed=93 + S)
    eng = engine_for(et, S, C, 500, states, alph.init_table, rates, probs, m.pi, [m])
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    b = 0
    bl = et.brlen.copy()
    bl[b] *= 1.5
    eng.update_pmatrices(np.array([b], dtype=np.int32), bl[[b]], deriv_mask=7)
    parents = {c: p for p, ch in et.ops for c in ch}
    anc, n = set(), b
    while n in parents:
        n = parents[n]
        anc.add(n)
    eng.update_partials(phylo.split_ops([(p, ch) for p, ch in et.ops if p in anc]))
    far = [v for v in range(et.n_nodes) if v != et.root and parents.get(v) not in anc]
    assert far
    et2 = phylo.EngineTree(et.n_tips, et.n_internal, et.root, et.tip_names, et.ops, bl, {}, [], [])
    eng2 = engine_for(et2, S, C, 500, states, alph.init_table, rates, probs, m.pi, [m])
    eng2.update_pmatrices(br, bl[br], deriv_mask=7)
    run_engine(eng2, et2)
    for v in far[:4] + [b]:
        a1, a2 = eng.branch_derivatives(v)
        e1, e2 = eng2.branch_derivatives(v)
        assert _close(a1, e1, 1e-12) and _close(a2, e2, 1e-12), (v, a1, e1, a2, e2)


@pytest.mark.parametrize("S,C,n_taxa,n_pat", [(4, 4, 12, 400), (20, 2, 8, 150), (4, 1, 5, 64)])
def test_dr_vs_oracle_restatement(S, C, n_taxa, n_pat):
    """Engine DR pass against the oracle's DRHomogeneousTreeLikelihood restatement
    (oracle.dr_derivatives, itself pinned by central differences in test_oracle_golden.py)
    on the same alignment; P, dP, d2P on the oracle side from scipy-free expm of Q
    (oracle.reversible_pij): relative 1e-10 per branch."""
    import oracle
    et, m, alph, rates, probs, states = _random_problem(S, C, n_taxa, n_pat, seed=100 + S + C)
    eng = engine_for(et, S, C, n_pat, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | DR)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    d1, d2 = eng.all_branch_derivatives()
    P = np.zeros((et.n_nodes, C, S, S))
    dP, d2P = np.zeros_like(P), np.zeros_like(P)
    for n in range(et.n_nodes):
        if n == et.root:
            continue
        for c in range(C):
            p = oracle.reversible_pij(m.Q, m.pi, et.brlen[n] * rates[c])
            P[n, c], dP[n, c], d2P[n, c] = p, rates[c] * m.Q @ p, rates[c] ** 2 * m.Q @ m.Q @ p
    ss, sons, lr = et.son_arrays()
    o1, o2 = oracle.dr_derivatives(ss, sons, lr, et.root, states, alph.init_table, P, dP, d2P, probs, m.pi)
    for b in br:
        assert _close(d1[b], o1[b], 1e-10), (b, d1[b], o1[b])
        assert _close(d2[b], o2[b], 1e-10), (b, d2[b], o2[b])


@pytest.mark.parametrize("C,n_taxa,n_pat,amb", [(4, 64, 5000, True), (1, 9, 700, False), (2, 33, 1300, True),
                                                 (4, 3, 1, False)])
def test_dr_fused_preorder_vs_path(C, n_taxa, n_pat, amb):
    """4 states without rescaling: the fused preorder (dr_pre_s4_kernel: father-side vectors
    in registers, branch terms reduced where they are formed) against the path derivatives
    of every branch."""
    et, m, alph, rates, probs, states = _random_problem(4, C, n_taxa, n_pat, seed=90 + C + n_taxa, amb=amb)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng = engine_for(et, 4, C, n_pat, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY | DR)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    _dr_vs_path(eng, et)


@pytest.mark.parametrize("S,C,tree_kind,n_pat,scaling", [
    (20, 4, "balanced40", 500, True), (20, 2, "balanced24", 333, False), (20, 1, "caterpillar120long", 300, True),
    (64, 1, "balanced24", 300, False), (64, 2, "balanced16", 130, True), (64, 1, "caterpillar150long", 200, True),
    (4, 4, "caterpillar300long", 600, True), (4, 2, "balanced64", 2000, True)])
def test_dr_any_state_count_vs_path(S, C, tree_kind, n_pat, scaling):
    """All-branch derivatives beyond unscaled DNA: the fused preorder for 20 states on fp64
    matrix cores (dr_pre_m20_kernel) and for 4 states with rescaling (dr_pre_s4_kernel<C,
    true>; stored upper vectors rescaled jointly over states and classes), the levelwise
    preorder + MFMA reduction for 64 states, against the path derivatives at 1e-10 (1e-9
    through deep rescaling).  "long" caterpillars drive partials and upper vectors below
    2^-256."""
    rng = np.random.default_rng(S * 7 + C + n_pat)
    if tree_kind.startswith("balanced"):
        tree = phylo.balanced_tree(int(tree_kind[8:]), seed=S + C, lo=0.05, hi=0.4)
    else:
        tree = _caterpillar(int(tree_kind[11:-4]), seed=3, lo=0.1, hi=0.5)
    et = phylo.engine_tree(tree)
    if S == 4:
        m, alph = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5)), phylo.DNA
    elif S == 20:
        m, alph = phylo.lg08(), phylo.PROTEIN
    else:
        m, alph = phylo.yn98(2.0, 0.3), phylo.CODON
    rates, probs = phylo.gamma_rates(C, 0.6) if C > 1 else (np.ones(1), np.ones(1))
    wl = workload.Workload("d", et, [m], None, rates, probs, m.pi, alph, n_pat, scaling, True, 4)
    states = wl.simulate(0, n_pat).astype(np.int32)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    flags = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY | DR | (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, S, C, n_pat, states, alph.init_table, rates, probs, m.pi, [m], flags=flags)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    _, site, _ = run_engine(eng, et)
    if tree_kind.endswith("long"):
        assert site.min() < -256 * np.log(2)
    _dr_vs_path(eng, et, rel=1e-9 if tree_kind.endswith("long") else 1e-10)


@pytest.mark.parametrize("seed", range(24))
def test_dr_random_topologies(seed):
    """Random unbalanced trees with polytomies (test_gpu_parity._random_topology), one or two
    rate models over the branches, 4 / 20 / 64 states, every traversal mode, with and without
    rescaling: every branch's double-recursive derivatives against the single-traversal path
    derivatives (1e-10), and two branches' first derivatives against central differences of
    the oracle's lnL."""
    from test_gpu_parity import _random_topology
    rng = np.random.default_rng(2000 + seed)
    S = 20 if seed % 4 == 3 else 64 if seed % 8 == 5 else 4
    C = 1 if S == 64 else int(rng.choice([1, 2, 4]))
    n_taxa = int(rng.integers(3, 25 if S != 4 else 90))
    n = int(rng.choice([1, 300, 1500]))
    scaling = bool(rng.random() < 0.35)
    lo, hi = (0.3, 1.0) if scaling else (0.02, 0.3)
    et = phylo.engine_tree(_random_topology(n_taxa, rng, lo, hi), unroot=bool(rng.random() < 0.5))
    n_models = int(rng.integers(1, 3))
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
    wl = workload.Workload("d", et, models, mon, rates, probs, models[0].pi, alph, n, scaling, True, seed)
    states = wl.simulate(0, n).astype(np.int32)
    mode = ["lnl_only", "materialize", "levelwise"][seed % 3]
    flags = plk.PLK_FLAG_NONNEG_GUARD | MODES[mode] | DR | (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, S, C, n, states, alph.init_table, rates, probs, models[0].pi, models, model_of_node=mon,
                     flags=flags)
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], None if mon is None else mon[br], deriv_mask=7)
    lnl0 = abs(run_engine(eng, et)[0])
    d1, _ = _dr_vs_path(eng, et)
    for b in rng.choice(br, size=min(2, len(br)), replace=False):
        b = int(b)
        h = 1e-5 * max(1.0, et.brlen[b])

        def lnl_at(t):
            bl = et.brlen.copy()
            bl[b] = t
            e2 = phylo.EngineTree(et.n_tips, et.n_internal, et.root, et.tip_names, et.ops, bl, {}, [], [])
            return oracle_for(e2, states, alph.init_table, rates, probs, models[0].pi, models, model_of_node=mon,
                              scaling=scaling)[0]

        fd1 = (lnl_at(et.brlen[b] + h) - lnl_at(et.brlen[b] - h)) / (2 * h)
        # central-difference error: truncation O(h^2) plus the lnL round-off amplified by 1/h
        assert abs(d1[b] - fd1) <= 1e-5 * max(1.0, abs(fd1)) + 64 * 2.2e-16 * lnl0 / h, (b, d1[b], fd1)
