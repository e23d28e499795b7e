"""CPU tests: pin the oracle (oracle/oracle.cpp) against the reference's goldens and
the committed fixtures (tests/golden/).  No GPU needed."""
import json
import os

import numpy as np
import pytest

import oracle
import phylo

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _ref():
    with open(os.path.join(GOLD, "reference.json")) as f:
        return json.load(f)


def _oracle_case(case, rates=None, use_patterns=True):
    et = phylo.engine_tree(phylo.Tree.from_newick(case["newick"]), unroot=case["unroot"])
    states = np.stack([phylo.DNA.encode(case["sequences"][n]) for n in et.tip_names])
    m = case["model"]
    if case["rates"]["name"] == "Gamma":
        r, p = oracle.gamma_rates(case["rates"]["n"], case["rates"]["alpha"]) if rates is None else rates
    else:
        r, p = np.ones(1), np.ones(1)
    C = len(r)
    pm = np.zeros((et.n_nodes, C, 4, 4))
    for n in range(et.n_nodes):
        if n != et.root:
            for c in range(C):
                pm[n, c] = oracle.t92_pij(m["kappa"], m["theta"], et.brlen[n] * r[c])
    ss, sons, lr = et.son_arrays()
    lnl, sites, _, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, phylo.DNA.init_table, pm, p,
                                          oracle.t92_freqs(m["theta"]), use_patterns=use_patterns, want_sites=True)
    return lnl, sites


def test_gamma_rates_alpha1():
    # mean-of-category discretisation, alpha = beta = 1
    r, p = oracle.gamma_rates(4, 1.0)
    assert np.allclose(r, [0.13695378, 0.47675186, 1.0, 2.38629436], atol=1e-8)
    assert np.allclose(p, 0.25)
    assert abs(np.dot(r, p) - 1.0) < 1e-9


@pytest.mark.parametrize("alpha", [0.2, 0.5, 1.0, 2.0, 7.5])
def test_gamma_rates_vs_exact(alpha):
    r, _ = oracle.gamma_rates(4, alpha)
    r2, _ = phylo.gamma_rates(4, alpha)
    # bpp-core's AS91/AS32 accuracy vs scipy's exact quantiles
    assert np.allclose(r, r2, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("use_patterns", [True, False])
def test_likelihood_golden(use_patterns):
    """test/test_likelihood.cpp:108: initial -lnL = 85.030942031997312824."""
    case = _ref()["test_likelihood"]
    lnl, _ = _oracle_case(case, use_patterns=use_patterns)
    assert abs(-lnl - 85.030942031997312824) < 1e-9


def test_likelihood_clock_golden():
    """test/test_likelihood_clock.cpp:115: initial -lnL = 94.3957 (printed to 4 decimals)."""
    case = _ref()["test_likelihood_clock"]
    lnl, _ = _oracle_case(case)
    assert abs(-lnl - 94.3957) < 5e-5


def test_example1_config1():
    """BASELINE config 1 (example1.ph / example1.mp.dnd, gaps -> N): restatement-derived value."""
    case = _ref()["example1"]
    lnl, _ = _oracle_case(case)
    assert abs(-lnl - 43.259398988513) < 1e-9


def test_gap_raises_bad_int():
    case = dict(_ref()["test_likelihood"])
    seqs = dict(case["sequences"])
    seqs["A"] = "-" + seqs["A"][1:]
    case["sequences"] = seqs
    with pytest.raises(ValueError):
        _oracle_case(case)


def test_t92_closed_form_vs_expm():
    f = np.load(os.path.join(GOLD, "pmatrix.npz"))
    for t, P in zip(f["T92_t"], f["T92_P"]):
        assert np.allclose(oracle.t92_pij(3.0, 0.5, t), P, atol=1e-14)
    for t, P in zip(f["T92_k2_t03_t"], f["T92_k2_t03_P"]):
        assert np.allclose(oracle.t92_pij(2.0, 0.3, t), P, atol=1e-14)


@pytest.mark.parametrize("name", ["GTR", "LG08", "T92", "YN98"])
def test_reversible_pij_vs_expm(name):
    f = np.load(os.path.join(GOLD, "pmatrix.npz"))
    Q, pi = f[f"{name}_Q"], f[f"{name}_pi"]
    for t, P in zip(f[f"{name}_t"], f[f"{name}_P"]):
        assert np.allclose(oracle.reversible_pij(Q, pi, t), P, atol=1e-13)


def test_gtr_generator_matches_host():
    ex, pi = oracle.gtr_model(1.2, 0.4, 0.6, 0.8, 0.5, 0.45, 0.30 / 0.55, 0.25 / 0.45)
    Q = oracle.reversible_generator(ex, pi)
    m = phylo.gtr(a=1.2, b=0.4, c=0.6, d=0.8, e=0.5, piA=0.30, piC=0.20, piG=0.25, piT=0.25)
    assert np.allclose(pi, m.pi, atol=1e-15)
    assert np.allclose(Q, m.Q, atol=1e-14)
    # normalisation -sum pi_i Q_ii = 1 (Model/AbstractSubstitutionModel.cpp:645-690)
    assert abs(-np.dot(np.diag(Q), pi) - 1.0) < 1e-14


def _fixture_case(name):
    f = np.load(os.path.join(GOLD, "pruning.npz"))
    g = {k[len(name) + 1:]: f[k] for k in f.files if k.startswith(name + "_")}
    return g


def _oracle_fixture(g, alph, use_patterns=True, scaling=False):
    n_nodes = len(g["leaf_row"])
    C = len(g["rates"])
    S = g["pi"].shape[0]
    pm = np.zeros((n_nodes, C, S, S))
    root = int(g["root"])
    for n in range(n_nodes):
        if n != root:
            for c in range(C):
                pm[n, c] = oracle.reversible_pij(g["Q"], g["pi"], g["brlen"][n] * g["rates"][c])
    return oracle.tree_loglik(g["son_start"], g["sons"], g["leaf_row"], root, g["states"], alph.init_table, pm,
                              g["probs"], g["pi"], use_patterns=use_patterns, scaling=scaling, want_sites=True)


@pytest.mark.parametrize("name,alph", [("T92", phylo.DNA), ("GTR", phylo.DNA), ("GTRamb", phylo.DNA),
                                        ("LG08", phylo.PROTEIN), ("YN98", phylo.CODON)])
@pytest.mark.parametrize("use_patterns", [True, False])
def test_oracle_vs_numpy_pruning(name, alph, use_patterns):
    g = _fixture_case(name)
    lnl, sites, _, _ = _oracle_fixture(g, alph, use_patterns=use_patterns)
    assert np.allclose(sites, g["site_lnl"], rtol=1e-12, atol=0)
    assert abs(lnl - float(g["lnl"])) <= 1e-12 * abs(lnl)


def test_oracle_scaling_is_exact_when_not_triggered():
    g = _fixture_case("GTR")
    a = _oracle_fixture(g, phylo.DNA, scaling=False)
    b = _oracle_fixture(g, phylo.DNA, scaling=True)
    assert a[0] == b[0]


def test_oracle_scaling_rescues_underflow():
    # 512-taxon caterpillar-free balanced tree, long branches: unscaled underflows
    tree = phylo.balanced_tree(512, seed=3, lo=0.3, hi=0.6)
    et = phylo.engine_tree(tree)
    m = phylo.gtr(a=1.2, b=0.4, c=0.6, d=0.8, e=0.5, piA=0.3, piC=0.2, piG=0.25, piT=0.25)
    rates, probs = phylo.gamma_rates(4, 0.5)
    import workload
    wl = workload.Workload("t", et, [m], None, rates, probs, m.pi, phylo.DNA, 64, True, True)
    states = wl.simulate(0, 64)
    pm = np.zeros((et.n_nodes, 4, 4, 4))
    for n in range(et.n_nodes):
        if n != et.root:
            for c in range(4):
                pm[n, c] = m.pij(et.brlen[n] * rates[c])
    ss, sons, lr = et.son_arrays()
    l0, s0, _, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, phylo.DNA.init_table, pm, probs, m.pi,
                                      scaling=False, want_sites=True)
    l1, s1, _, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, phylo.DNA.init_table, pm, probs, m.pi,
                                      scaling=True, want_sites=True)
    assert np.isfinite(l1)
    assert np.all(np.isfinite(s1))
    ok = np.isfinite(s0) & (s0 > -700)   # sites the unscaled arithmetic still resolves
    assert np.allclose(s0[ok], s1[ok], rtol=1e-12)
    assert (~np.isfinite(s0)).any() or (s0 < -700).any()


def _dr_problem(seed, n_taxa=9, n_sites=60, C=3):
    rng = np.random.default_rng(seed)
    tree = phylo.balanced_tree(n_taxa, seed=seed, lo=0.02, hi=0.4)
    et = phylo.engine_tree(tree)
    m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5))
    rates, probs = phylo.gamma_rates(C, 0.7)
    states = rng.integers(0, 4, size=(et.n_tips, n_sites)).astype(np.int32)
    return et, m, rates, probs, states


def _pmats(et, m, rates, brlen):
    C = len(rates)
    P = np.zeros((et.n_nodes, C, 4, 4))
    dP, d2P = np.zeros_like(P), np.zeros_like(P)
    for n in range(et.n_nodes):
        if n == et.root:
            continue
        for c in range(C):
            p = oracle.reversible_pij(m.Q, m.pi, brlen[n] * rates[c])
            P[n, c] = p
            dP[n, c] = rates[c] * m.Q @ p
            d2P[n, c] = rates[c] ** 2 * m.Q @ m.Q @ p
    return P, dP, d2P


@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_dr_derivatives_vs_central_differences(seed):
    """Pins the oracle's DRHomogeneousTreeLikelihood restatement (orc_dr_derivatives) with
    central differences of its own pruning (orc_tree_loglik), every branch."""
    et, m, rates, probs, states = _dr_problem(seed)
    ss, sons, lr = et.son_arrays()
    P, dP, d2P = _pmats(et, m, rates, et.brlen)
    d1, d2 = oracle.dr_derivatives(ss, sons, lr, et.root, states, phylo.DNA.init_table, P, dP, d2P, probs, m.pi)
    assert d1[et.root] == 0.0
    for v in range(et.n_nodes):
        if v == et.root:
            continue

        def lnl_at(t):
            bl = et.brlen.copy()
            bl[v] = t
            pm, _, _ = _pmats(et, m, rates, bl)
            return oracle.tree_loglik(ss, sons, lr, et.root, states, phylo.DNA.init_table, pm, probs, m.pi,
                                      use_patterns=False)[0]

        t = et.brlen[v]
        fd1 = (lnl_at(t + 1e-5) - lnl_at(t - 1e-5)) / 2e-5
        fd2 = (lnl_at(t + 1e-4) - 2 * lnl_at(t) + lnl_at(t - 1e-4)) / 1e-8
        assert abs(d1[v] - fd1) <= 1e-6 * max(1.0, abs(fd1)), (v, d1[v], fd1)
        assert abs(d2[v] - fd2) <= 1e-4 * max(1.0, abs(fd2)), (v, d2[v], fd2)


# ---------------------------------------------------------------- the two root rules (row a10)

def test_root_rules_agree_without_nonpositive_terms():
    """On positive root partials the NH rule (no guards, clamp) and the homogeneous rule
    (terms <= 0 dropped) are the same sum: the golden holds under both."""
    case = _ref()["test_likelihood"]
    et = phylo.engine_tree(phylo.Tree.from_newick(case["newick"]), unroot=case["unroot"])
    states = np.stack([phylo.DNA.encode(case["sequences"][n]) for n in et.tip_names])
    m = case["model"]
    r, p = oracle.gamma_rates(case["rates"]["n"], case["rates"]["alpha"])
    pm = np.zeros((et.n_nodes, len(r), 4, 4))
    for n in range(et.n_nodes):
        if n != et.root:
            pm[n] = np.stack([oracle.t92_pij(m["kappa"], m["theta"], et.brlen[n] * rc) for rc in r])
    pi = oracle.t92_freqs(m["theta"])
    import negroot
    lh, sh = negroot.oracle_sites(et, states, phylo.DNA.init_table, pm, p, pi, False, False)
    ln, sn = negroot.oracle_sites(et, states, phylo.DNA.init_table, pm, p, pi, False, True)
    assert lh == ln and np.array_equal(sh, sn)
    assert abs(-ln - 85.030942031997312824) < 1e-9


@pytest.mark.parametrize("S,C", [(4, 4), (20, 2), (64, 1)])
@pytest.mark.parametrize("kind", ["mixed", "clamp"])
def test_root_rules_oracle_vs_numpy(S, C, kind):
    """The oracle's two root rules (orc_tree_loglik_rule) against a numpy restatement of
    L/RHomogeneousTreeLikelihood.cpp:192-216 and L/RNonHomogeneousTreeLikelihood.cpp:198-221
    on inputs with root terms <= 0: per site (-inf at the same sites, no NaN), and the two
    rules differ where the census says they must."""
    import negroot
    et, m, init, states, rates, probs, pi, pm = negroot.problem(S, C, 16 if S < 64 else 8, 400, seed=S + C)
    delta, pm2, census = negroot.choose(et, states, init, pm, pi, probs, kind)
    assert census["neg_terms"] > 0
    Lr, lf = negroot.root_partials_signed(et, states, init, pm2)
    l_h, l_nh = negroot.rule_sums(Lr, pi, probs)
    with np.errstate(divide="ignore"):
        want_h = np.log(l_h) + lf
        want_nh = np.log(np.maximum(l_nh, 0.0)) + lf
    lh, sh = negroot.oracle_sites(et, states, init, pm2, probs, pi, False, False)
    ln, sn = negroot.oracle_sites(et, states, init, pm2, probs, pi, False, True)
    # sums in a different order: cancellation in the NH sum near 0 costs digits there
    negroot.same_sites(sh, want_h, rel=1e-11)
    negroot.same_sites(sn, want_nh, rel=1e-8)
    fin = np.isfinite(sn)
    assert np.any(sh[fin] != sn[fin])                    # the guards fired
    if kind == "clamp":
        assert census["clamp_sites"] > 0 and np.isneginf(ln)
        assert np.any(np.isneginf(sn) & np.isfinite(sh))  # the clamp fired (log 0, not NaN)
    else:
        assert np.isfinite(ln) and np.isfinite(lh) and ln < lh
