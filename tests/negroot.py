"""Problems whose root terms go <= 0: the inputs of the root-rule parity tests
(tests/test_oracle_golden.py on the CPU, tests/test_gpu_root_rules.py on the MI355X).

The reference's root reductions differ only when a term is <= 0:
  - RHomogeneousTreeLikelihood drops every term <= 0, per state (getLikelihoodForASiteForA
    RateClass, L/RHomogeneousTreeLikelihood.cpp:205-216) and per class
    (getLogLikelihoodForASite :192-201);
  - RNonHomogeneousTreeLikelihood adds every term and clamps the site sum l < 0 -> 0 before
    the log (L/RNonHomogeneousTreeLikelihood.cpp:198-221, clamp at :206).
The reference comments both as corrections for "slightly negative likelihoods" from rounding
in P(t).  Here the transition matrices of the root's first son (and of one tip, so negative
values also run through the cherry tables, the interior nodes and the rescale decisions)
get a negative rank-one shift of one row, strong enough that some root terms are negative:
  - "mixed": some terms < 0, every NH site sum > 0 -> both rules finite and different;
  - "clamp": some NH site sums < 0 -> -inf under the NH rule (log(0), not NaN), finite under
    the homogeneous rule at some of those sites.
The sign analysis below is a numpy pruning of the same inputs with a positive per-site
normalisation at every node (signs and ratios are those of the unnormalised arrays).
"""
from __future__ import annotations

import numpy as np

import oracle
import phylo


def root_partials_signed(et, states, init, pm):
    """Root partials [n_sites][C][S] divided by a positive factor per site (flat patterns),
    and the log of that factor."""
    ss, sons, lr = et.son_arrays()
    n = states.shape[1]
    C, S = pm.shape[1], pm.shape[2]
    L, lf = {}, {}
    order = [p for p, _ in et.ops]            # postorder of the internal nodes
    for t in range(et.n_tips):
        L[t] = np.broadcast_to(init[states[lr[t]]][:, None, :], (n, C, S))
        lf[t] = np.zeros(n)
    for p in order:
        acc, f = np.ones((n, C, S)), np.zeros(n)
        for k in sons[ss[p]:ss[p + 1]]:
            acc = acc * np.einsum("cxy,icy->icx", pm[k], L[int(k)])
            f = f + lf[int(k)]
        m = np.abs(acc).reshape(n, -1).max(axis=1)
        m[m == 0] = 1.0
        L[p], lf[p] = acc / m[:, None, None], f + np.log(m)
    return L[et.root], lf[et.root]


def rule_sums(Lr, pi, probs):
    """(homogeneous l, NH l before the clamp) per site, up to the per-site factor."""
    t = Lr * pi[None, None, :]
    lc_h = np.where(t > 0, t, 0.0).sum(axis=2) * probs[None, :]
    l_h = np.where(lc_h > 0, lc_h, 0.0).sum(axis=1)
    l_nh = (t.sum(axis=2) * probs[None, :]).sum(axis=1)
    return l_h, l_nh


def perturb(pm, et, delta):
    """P(t) with row 0 of the root's first son's matrices and row 1 of tip 0's shifted by -delta."""
    ss, sons, _ = et.son_arrays()
    b = int(sons[ss[et.root]])
    out = pm.copy()
    out[b, :, 0, :] -= delta
    out[0, :, 1, :] -= 0.5 * delta
    return out


def choose(et, states, init, pm, pi, probs, kind):
    """The first delta of a fixed ladder that gives a `kind` problem, and its sign census."""
    for delta in np.geomspace(1e-4, 0.95, 60):
        pm2 = perturb(pm, et, delta)
        Lr, _ = root_partials_signed(et, states, init, pm2)
        l_h, l_nh = rule_sums(Lr, pi, probs)
        n_neg_terms = int((Lr * pi <= 0).sum())
        if kind == "mixed" and n_neg_terms > 0 and l_nh.min() > 0 and np.any(l_nh < l_h * (1 - 1e-9)):
            return delta, pm2, dict(neg_terms=n_neg_terms, clamp_sites=0)
        if kind == "clamp" and np.any((l_nh < 0) & (l_h > 0)):
            return delta, pm2, dict(neg_terms=n_neg_terms, clamp_sites=int((l_nh < 0).sum()))
    raise AssertionError(f"no delta gives a {kind} problem")


def problem(S, C, n_taxa, n_sites, seed, tiny=False):
    """A seeded balanced-tree problem: engine tree, model, code table, states, rates, probs, pi
    and the oracle's transition matrices [n_nodes][C][S][S].  tiny: one code's vector is
    1e-80 on 30 % of the cells, so partials fall below 2^-256 and the rescaling fires."""
    rng = np.random.default_rng(seed)
    et = phylo.engine_tree(phylo.balanced_tree(n_taxa, seed=seed, lo=0.05, hi=0.4))
    if S == 4:
        m, alph = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5)), phylo.DNA
    elif S == 20:
        m, alph = phylo.lg08(), phylo.PROTEIN
    else:
        E = rng.uniform(0.1, 2.0, (S, S))
        E = E + E.T
        pi = rng.dirichlet(np.ones(S) * 5)
        Q = phylo.reversible_generator(E, pi)
        V, Vinv, lam = phylo.reversible_eigen(Q, pi)
        m, alph = phylo.Model("rand", S, Q, pi, V, Vinv, lam), phylo.Alphabet("R", S, {}, np.eye(S))
    rates, probs = phylo.gamma_rates(C, 0.5) if C > 1 else (np.ones(1), np.ones(1))
    states = rng.choice(S, size=(et.n_tips, n_sites), p=m.pi).astype(np.int32)
    init = np.array(alph.init_table, dtype=np.float64, copy=True)
    if tiny:
        code = alph.n_codes - 1 if alph.n_codes > S else S - 1
        init[code] = 1e-80
        states[rng.random(states.shape) < 0.3] = code
    pm = np.zeros((et.n_nodes, C, S, S))
    for n in range(et.n_nodes):
        if n != et.root:
            for c in range(C):
                pm[n, c] = oracle.reversible_pij(m.Q, m.pi, et.brlen[n] * rates[c])
    return et, m, init, states, rates, probs, m.pi, pm


def oracle_sites(et, states, init, pm, probs, pi, scaling, nh_root):
    ss, sons, lr = et.son_arrays()
    lnl, site, _, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, init, pm, probs, pi, use_patterns=False,
                                         scaling=scaling, want_sites=True, nh_root=nh_root)
    return lnl, site


def same_sites(a, b, rel=1e-12):
    """Per-site equality with -inf at the same sites, no NaN, finite sites at rel."""
    a, b = np.asarray(a), np.asarray(b)
    assert not np.isnan(a).any() and not np.isnan(b).any()
    fa, fb = np.isfinite(a), np.isfinite(b)
    assert np.array_equal(fa, fb), (np.flatnonzero(fa != fb)[:8], a[fa != fb][:8], b[fa != fb][:8])
    assert np.array_equal(a[~fa], b[~fb])
    assert np.allclose(a[fa], b[fb], rtol=rel, atol=0)
