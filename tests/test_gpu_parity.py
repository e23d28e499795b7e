"""GPU parity tests (run on the MI355X box): libplk through its C-ABI vs the CPU oracle
and the committed golden fixtures.

Tolerances (north_star: |dlnL|/|lnL| < 1e-10):
  - total lnL: relative 1e-12 against the oracle on identical inputs,
  - per-pattern lnL: relative 1e-12,
  - transition matrices vs scipy expm fixtures: absolute 1e-13,
  - sharded vs whole evaluation: bitwise equal (fixed-order block sums).
"""
import json
import os

import numpy as np
import pytest

import oracle
import phylo
import plk
import workload
from conftest import clear_tune, set_tune

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
REL = 1e-12


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if plk.device_count() < 1:
        pytest.fail("no GPU visible: gpu-marked tests must run on the MI355X box")


def engine_for(et, S, C, n_patterns, states, init_table, rates, probs, pi, models, model_of_node=None,
               flags=plk.PLK_FLAG_NONNEG_GUARD):
    eng = plk.Engine(0, S, C, n_patterns, et.n_tips, et.n_internal, len(models), flags)
    eng.set_code_table(init_table)
    for i in range(et.n_tips):
        eng.set_tip_codes(i, states[i].astype(np.uint8))
    eng.set_category_rates(rates, probs)
    eng.set_root_frequencies(pi)
    for k, m in enumerate(models):
        eng.set_eigen(k, m.V, m.Vinv, m.lam)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    mi = None if model_of_node is None else np.asarray(model_of_node)[br].astype(np.int32)
    eng.update_pmatrices(br, et.brlen[br], mi)
    return eng


def run_engine(eng, et, sites=True):
    eng.update_partials(phylo.split_ops(et.ops))
    return eng.root_loglik(et.root, want_sites=sites, want_blocks=True)


def oracle_for(et, states, init_table, rates, probs, pi, models, model_of_node=None, scaling=False,
               pmats=None):
    C = len(rates)
    S = init_table.shape[1]
    if pmats is None:
        pmats = np.zeros((et.n_nodes, C, S, S))
        for n in range(et.n_nodes):
            if n == et.root:
                continue
            m = models[0] if model_of_node is None else models[model_of_node[n]]
            for c in range(C):
                pmats[n, c] = oracle.reversible_pij(m.Q, m.pi, et.brlen[n] * rates[c])
    ss, sons, lr = et.son_arrays()
    lnl, site, _, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, init_table, pmats, probs, pi,
                                         use_patterns=False, scaling=scaling, want_sites=True)
    return lnl, site


def engine_pmats(eng, et):
    """The engine's own transition matrices (K4 output), so that the oracle checks the
    pruning on identical P(t) inputs (SURVEY 8(d) parity check)."""
    pm = np.zeros((et.n_nodes, eng.C, eng.S, eng.S))
    for n in range(et.n_nodes):
        if n != et.root:
            pm[n] = eng.get_pmatrix(n)
    return pm


def check(lnl_g, site_g, lnl_o, site_o, rel=REL):
    assert np.all(np.isfinite(site_g))
    assert abs(lnl_g - lnl_o) <= rel * abs(lnl_o), (lnl_g, lnl_o)
    assert np.allclose(site_g, site_o, rtol=rel, atol=0)


# ---------------------------------------------------------------- transition matrices (K4)

@pytest.mark.parametrize("name", ["T92", "GTR", "LG08", "YN98"])
def test_pmatrix_kernel_vs_expm(name):
    """K4 against the scipy expm fixtures; YN98 runs the 64-state pmat64s_kernel that
    config 4's bench line times (C = 1, stop states as null rows)."""
    f = np.load(os.path.join(GOLD, "pmatrix.npz"))
    m = {"T92": phylo.t92(3.0, 0.5), "GTR": phylo.gtr(a=1.2, b=0.4, c=0.6, d=0.8, e=0.5, piA=0.30, piC=0.20,
                                                          piG=0.25, piT=0.25), "LG08": phylo.lg08(),
         "YN98": phylo.yn98(2.0, 0.3)}[name]
    ts = f[f"{name}_t"]
    et = phylo.engine_tree(phylo.balanced_tree(8))
    eng = plk.Engine(0, m.S, 1, 256, et.n_tips, et.n_internal, 1)
    eng.set_category_rates(np.ones(1), np.ones(1))
    eng.set_eigen(0, m.V, m.Vinv, m.lam)
    br = np.arange(len(ts), dtype=np.int32)
    eng.update_pmatrices(br, ts)
    for i, P in enumerate(f[f"{name}_P"]):
        assert np.allclose(eng.get_pmatrix(i)[0], P, atol=1e-13)


@pytest.mark.parametrize("name", ["GTR", "LG08", "YN98"])
def test_dpmatrix_kernel_vs_expm(name):
    """dP/dt and d2P/dt2 from K4 (PLK_DERIV_DP | PLK_DERIV_D2P) against Q expm(Qt) and
    Q^2 expm(Qt) fixtures (getdPij_dt / getd2Pij_dt2, Model/AbstractSubstitutionModel.cpp:
    499-641), one class of rate 1; and r_c / r_c^2 scaling with Gamma classes."""
    f = np.load(os.path.join(GOLD, "pmatrix.npz"))
    m = {"GTR": phylo.gtr(a=1.2, b=0.4, c=0.6, d=0.8, e=0.5, piA=0.30, piC=0.20, piG=0.25, piT=0.25),
         "LG08": phylo.lg08(), "YN98": phylo.yn98(2.0, 0.3)}[name]
    ts = f[f"{name}_t"]
    et = phylo.engine_tree(phylo.balanced_tree(8))
    eng = plk.Engine(0, m.S, 1, 256, et.n_tips, et.n_internal, 1)
    eng.set_category_rates(np.ones(1), np.ones(1))
    eng.set_eigen(0, m.V, m.Vinv, m.lam)
    br = np.arange(len(ts), dtype=np.int32)
    eng.update_pmatrices(br, ts, deriv_mask=plk.PLK_DERIV_P | plk.PLK_DERIV_DP | plk.PLK_DERIV_D2P)
    scale = max(1.0, float(np.abs(f[f"{name}_Q"]).max()))
    for i in range(len(ts)):
        assert np.allclose(eng.get_dpmatrix(i, 1)[0], f[f"{name}_dP"][i], atol=1e-13 * scale)
        assert np.allclose(eng.get_dpmatrix(i, 2)[0], f[f"{name}_d2P"][i], atol=1e-13 * scale ** 2)
    rates, probs = phylo.gamma_rates(4, 0.5)
    e4 = plk.Engine(0, m.S, 4, 256, et.n_tips, et.n_internal, 1)
    e4.set_category_rates(rates, probs)
    e4.set_eigen(0, m.V, m.Vinv, m.lam)
    e4.update_pmatrices(np.array([0], dtype=np.int32), np.array([0.3]), deriv_mask=7)
    Q = f[f"{name}_Q"]
    for c, r in enumerate(rates):
        E = m.pij(0.3 * r)
        assert np.allclose(e4.get_dpmatrix(0, 1)[c], r * (Q @ E), atol=1e-12 * scale * r)
        assert np.allclose(e4.get_dpmatrix(0, 2)[c], r * r * (Q @ Q @ E), atol=1e-12 * (scale * r) ** 2)


def test_pmatrix_derivatives():
    m = phylo.gtr(a=1.2, b=0.4, c=0.6, d=0.8, e=0.5, piA=0.30, piC=0.20, piG=0.25, piT=0.25)
    eng = plk.Engine(0, 4, 4, 256, 4, 2, 1)
    rates, probs = phylo.gamma_rates(4, 0.5)
    eng.set_category_rates(rates, probs)
    eng.set_eigen(0, m.V, m.Vinv, m.lam)
    eng.update_pmatrices(np.array([0, 1], dtype=np.int32), np.array([0.1, 0.7]),
                         deriv_mask=plk.PLK_DERIV_P | plk.PLK_DERIV_DP | plk.PLK_DERIV_D2P)
    P = eng.get_pmatrix(1)
    for c, r in enumerate(rates):
        assert np.allclose(P[c], m.pij(0.7 * r), atol=1e-14)


# ---------------------------------------------------------------- reference goldens through the engine

def _ref_case(key):
    with open(os.path.join(GOLD, "reference.json")) as f:
        case = json.load(f)[key]
    et = phylo.engine_tree(phylo.Tree.from_newick(case["newick"]), unroot=case["unroot"])
    states = np.stack([phylo.DNA.encode(case["sequences"][n]) for n in et.tip_names])
    m = phylo.t92(case["model"]["kappa"], case["model"]["theta"])
    if case["rates"]["name"] == "Gamma":
        rates, probs = phylo.gamma_rates(case["rates"]["n"], case["rates"]["alpha"])
    else:
        rates, probs = np.ones(1), np.ones(1)
    return case, et, states, m, rates, probs


@pytest.mark.parametrize("key,golden,tol", [("test_likelihood", 85.030942031997312824, 1e-9),
                                             ("test_likelihood_clock", 94.3957, 5e-5),
                                             ("example1", 43.259398988513, 1e-9)])
def test_reference_goldens(key, golden, tol):
    case, et, states, m, rates, probs = _ref_case(key)
    eng = engine_for(et, 4, len(rates), states.shape[1], states, phylo.DNA.init_table, rates, probs, m.pi, [m])
    lnl, site, _ = run_engine(eng, et)
    assert abs(-lnl - golden) < tol
    lo, so = oracle_for(et, states, phylo.DNA.init_table, rates, probs, m.pi, [m])
    check(lnl, site, lo, so)


def test_closed_form_pmatrix_path():
    """T92 P(t) computed on the host in closed form and handed over with plk_set_pmatrix."""
    case, et, states, m, rates, probs = _ref_case("test_likelihood")
    C = len(rates)
    eng = plk.Engine(0, 4, C, states.shape[1], et.n_tips, et.n_internal, 1, plk.PLK_FLAG_NONNEG_GUARD)
    eng.set_code_table(phylo.DNA.init_table)
    for i in range(et.n_tips):
        eng.set_tip_codes(i, states[i].astype(np.uint8))
    eng.set_category_rates(rates, probs)
    eng.set_root_frequencies(m.pi)
    pm = np.zeros((et.n_nodes, C, 4, 4))
    for n in range(et.n_nodes):
        if n != et.root:
            pm[n] = np.stack([oracle.t92_pij(3.0, 0.5, et.brlen[n] * r) for r in rates])
            eng.set_pmatrix(n, pm[n])
    lnl, site, _ = run_engine(eng, et)
    lo, so = oracle_for(et, states, phylo.DNA.init_table, rates, probs, m.pi, [m], pmats=pm)
    check(lnl, site, lo, so)
    assert abs(-lnl - 85.030942031997312824) < 1e-9


# ---------------------------------------------------------------- committed pruning fixtures

@pytest.mark.parametrize("name,alph", [("T92", phylo.DNA), ("GTR", phylo.DNA), ("GTRamb", phylo.DNA),
                                        ("LG08", phylo.PROTEIN), ("YN98", phylo.CODON)])
@pytest.mark.parametrize("extra", [0, plk.PLK_FLAG_LNL_ONLY])
def test_pruning_fixtures(name, alph, extra):
    f = np.load(os.path.join(GOLD, "pruning.npz"))
    g = {k[len(name) + 1:]: f[k] for k in f.files if k.startswith(name + "_")}
    # rebuild the engine tree from the fixture arrays
    n_nodes = len(g["leaf_row"])
    n_tips = int((g["leaf_row"] >= 0).sum())
    ops = [(p, tuple(int(x) for x in g["sons"][g["son_start"][p]:g["son_start"][p + 1]]))
           for p in range(n_tips, n_nodes)]
    et = phylo.EngineTree(n_tips, n_nodes - n_tips, int(g["root"]), [], ops, g["brlen"], {}, [], [])
    Q, pi = g["Q"], g["pi"]
    V, Vinv, lam = phylo.reversible_eigen(Q, pi)
    m = phylo.Model(name, Q.shape[0], Q, pi, V, Vinv, lam)
    eng = engine_for(et, m.S, len(g["rates"]), g["states"].shape[1], g["states"], alph.init_table, g["rates"],
                     g["probs"], pi, [m], flags=plk.PLK_FLAG_NONNEG_GUARD | extra)
    lnl, site, _ = run_engine(eng, et)
    assert np.allclose(site, g["site_lnl"], rtol=REL, atol=0)
    assert abs(lnl - float(g["lnl"])) <= REL * abs(lnl)


# ---------------------------------------------------------------- seeded random problems vs the oracle

def _random_problem(S, C, n_taxa, n_patterns, seed, alpha=0.5, amb=False, lo=0.01, hi=0.3):
    rng = np.random.default_rng(seed)
    tree = phylo.balanced_tree(n_taxa, seed=seed, lo=lo, hi=hi)
    et = phylo.engine_tree(tree)
    if S == 4:
        m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5))
        alph = phylo.DNA
    elif S == 20:
        m = phylo.lg08()
        alph = phylo.PROTEIN
    else:
        E = rng.uniform(0.1, 2.0, (S, S))
        E = E + E.T
        pi = rng.dirichlet(np.ones(S) * 5)
        Q = phylo.reversible_generator(E, pi)
        V, Vinv, lam = phylo.reversible_eigen(Q, pi)
        m = phylo.Model("rand", S, Q, pi, V, Vinv, lam)
        alph = phylo.CODON if S == 64 else phylo.Alphabet("R", S, {}, np.eye(S))
    rates, probs = phylo.gamma_rates(C, alpha)
    wl = workload.Workload("r", et, [m], None, rates, probs, m.pi, alph, n_patterns, False, True, seed)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    if amb:
        mask = rng.random(states.shape) < 0.15
        states[mask] = rng.integers(S, alph.n_codes, size=mask.sum())
    return et, m, alph, rates, probs, states


@pytest.mark.parametrize("S,C,n_taxa,n_patterns", [
    (4, 4, 16, 5000), (4, 1, 9, 1000), (4, 2, 12, 777), (4, 8, 10, 300), (4, 4, 3, 1), (4, 4, 33, 129),
    (20, 4, 12, 600), (20, 1, 7, 250), (64, 1, 8, 300), (64, 1, 5, 130), (64, 2, 10, 400), (64, 4, 3, 1)])
def test_random_vs_oracle(S, C, n_taxa, n_patterns):
    et, m, alph, rates, probs, states = _random_problem(S, C, n_taxa, n_patterns, seed=S * 1000 + C * 10 + n_taxa)
    eng = engine_for(et, S, C, n_patterns, states, alph.init_table, rates, probs, m.pi, [m])
    lnl, site, _ = run_engine(eng, et)
    lo, so = oracle_for(et, states, alph.init_table, rates, probs, m.pi, [m])
    check(lnl, site, lo, so)


def _random_topology(n, rng, lo, hi, poly=0.1):
    """A random rooted tree: subtrees joined at random (a coalescent-like shape, unbalanced),
    now and then three or four at once (a polytomy), branch lengths uniform in [lo, hi]."""
    parts = [f"t{i}" for i in range(n)]
    while len(parts) > 1:
        k = 2 if len(parts) < 4 or rng.random() > poly else int(rng.integers(3, 5))
        idx = sorted(rng.choice(len(parts), size=min(k, len(parts)), replace=False), reverse=True)
        kids = [parts.pop(int(i)) for i in idx]
        parts.append("(" + ",".join(f"{c}:{rng.uniform(lo, hi):.5f}" for c in kids) + ")")
    return phylo.Tree.from_newick(parts[0] + ";")


@pytest.mark.parametrize("seed", range(48))
def test_random_topologies_vs_oracle(seed):
    """Random unbalanced trees (random joins, polytomies, rooted or unrooted), random
    GTR / LG08 / YN98 models with one to three of them over the branches, 1-4 rate classes,
    every traversal mode (per-subtree compression for one model), with and without
    rescaling (long branches) and ambiguity codes, against the oracle at 1e-12 per pattern
    on the engine's own P(t) -- the fragment cutting, tiers, cherry tables and shape sharing
    of the generated kernels on shapes no config has."""
    rng = np.random.default_rng(1000 + seed)
    S = 20 if seed % 4 == 3 else 64 if seed % 8 == 5 else 4
    C = 1 if S == 64 else int(rng.choice([1, 2, 3, 4]))
    n_taxa = int(rng.integers(3, 41 if S == 20 else 31 if S == 64 else 301))
    n = int(rng.choice([1, 77, 700, 2500]))
    scaling = bool(rng.random() < 0.4)
    lo, hi = (0.3, 1.2) if scaling else (0.01, 0.3)
    tree = _random_topology(n_taxa, rng, lo, hi)
    unroot = bool(rng.random() < 0.5)
    et = phylo.engine_tree(tree, unroot=unroot)
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
    wl = workload.Workload("f", et, models, mon, rates, probs, models[0].pi, alph, n, scaling, True, seed)
    states = wl.simulate(0, n).astype(np.int32)
    if rng.random() < 0.5:  # ambiguity / gap codes
        mask = rng.random(states.shape) < 0.1
        states[mask] = rng.integers(S, alph.n_codes, size=mask.sum())
    mode = ["lnl_only", "materialize", "levelwise", "subtree"][seed % 4 if n_models == 1 else seed % 3]
    flags = plk.PLK_FLAG_NONNEG_GUARD | (plk.PLK_FLAG_SUBTREE_PATTERNS if mode == "subtree" else MODES[mode]) | \
        (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, S, C, n, states, alph.init_table, rates, probs, models[0].pi, models, model_of_node=mon,
                     flags=flags)
    lnl, site, _ = run_engine(eng, et)
    lo_, so = oracle_for(et, states, alph.init_table, rates, probs, models[0].pi, models, model_of_node=mon,
                         scaling=scaling, pmats=engine_pmats(eng, et))
    check(lnl, site, lo_, so)
    lnl2, site2, _ = run_engine(eng, et)  # a second traversal: the same doubles
    assert lnl2 == lnl and np.array_equal(site2, site)


def test_ambiguity_codes_vs_oracle():
    et, m, alph, rates, probs, states = _random_problem(4, 4, 20, 3000, seed=5, amb=True)
    eng = engine_for(et, 4, 4, 3000, states, alph.init_table, rates, probs, m.pi, [m])
    lnl, site, _ = run_engine(eng, et)
    lo, so = oracle_for(et, states, alph.init_table, rates, probs, m.pi, [m])
    check(lnl, site, lo, so)


def test_polytomy_accumulate_vs_oracle():
    t = phylo.Tree.from_newick("((a:0.1,b:0.2,c:0.05,d:0.3,e:0.12):0.1,(f:0.2,g:0.1):0.05,h:0.3,i:0.2);")
    et = phylo.engine_tree(t)
    m = phylo.gtr(1.2, 0.4, 0.6, 0.8, 0.5, 0.3, 0.2, 0.25, 0.25)
    rates, probs = phylo.gamma_rates(4, 0.5)
    wl = workload.Workload("p", et, [m], None, rates, probs, m.pi, phylo.DNA, 1000, False, True, 9)
    states = wl.simulate(0, 1000).astype(np.int32)
    assert any(len(ch) > 3 for _, ch in et.ops)
    eng = engine_for(et, 4, 4, 1000, states, phylo.DNA.init_table, rates, probs, m.pi, [m])
    lnl, site, _ = run_engine(eng, et)
    lo, so = oracle_for(et, states, phylo.DNA.init_table, rates, probs, m.pi, [m])
    check(lnl, site, lo, so)


@pytest.mark.parametrize("S", [4, 20, 64])
def test_scaling_vs_oracle_deep_tree(S):
    """Trees where the unscaled reference underflows: both sides use exact 2^256 rescaling."""
    et, m, alph, rates, probs, states = _random_problem(S, 4, 256, 700, seed=11 + S, lo=0.2, hi=0.5)
    eng = engine_for(et, S, 4, 700, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_SCALING | plk.PLK_FLAG_NONNEG_GUARD)
    lnl, site, _ = run_engine(eng, et)
    lo, so = oracle_for(et, states, alph.init_table, rates, probs, m.pi, [m], scaling=True)
    check(lnl, site, lo, so)
    assert lnl < -745 * 10  # deep enough that the scaling matters


def test_nonhomogeneous_vs_oracle():
    wl = workload.make_workload("nh_gtr_g4_dna_2M_512", n_patterns=2000)
    et = wl.et
    # shrink: keep the tree but only 2000 patterns; oracle at 512 taxa is still fast
    states = wl.simulate(0, 2000).astype(np.int32)
    eng = engine_for(et, 4, 4, 2000, states, phylo.DNA.init_table, wl.rates, wl.probs, wl.root_freqs, wl.models,
                     model_of_node=wl.model_of_node, flags=plk.PLK_FLAG_SCALING)
    lnl, site, _ = run_engine(eng, et)
    lo, so = oracle_for(et, states, phylo.DNA.init_table, wl.rates, wl.probs, wl.root_freqs, wl.models,
                        model_of_node=wl.model_of_node, scaling=True)
    check(lnl, site, lo, so)


# ---------------------------------------------------------------- sharding / determinism

def test_sharded_block_sums_bitwise():
    et, m, alph, rates, probs, states = _random_problem(4, 4, 24, 3 * 4096 + 1000, seed=21)
    P = states.shape[1]
    eng = engine_for(et, 4, 4, P, states, alph.init_table, rates, probs, m.pi, [m])
    lnl, _, blocks = run_engine(eng, et, sites=False)
    cut = 2 * 4096
    e1 = engine_for(et, 4, 4, cut, states[:, :cut], alph.init_table, rates, probs, m.pi, [m])
    e2 = engine_for(et, 4, 4, P - cut, states[:, cut:], alph.init_table, rates, probs, m.pi, [m])
    _, _, b1 = run_engine(e1, et, sites=False)
    _, _, b2 = run_engine(e2, et, sites=False)
    allb = np.concatenate([b1, b2])
    assert np.array_equal(allb, blocks)
    s = 0.0
    for v in allb:
        s += v
    assert s == lnl


def test_repeat_evaluation_bitwise():
    et, m, alph, rates, probs, states = _random_problem(4, 4, 32, 10000, seed=4)
    eng = engine_for(et, 4, 4, 10000, states, alph.init_table, rates, probs, m.pi, [m])
    a = run_engine(eng, et)
    b = run_engine(eng, et)
    assert a[0] == b[0] and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("S,C,flags", [(4, 4, plk.PLK_FLAG_LNL_ONLY), (4, 2, 0), (4, 4, plk.PLK_FLAG_LEVELWISE),
                                         (20, 4, plk.PLK_FLAG_LNL_ONLY)])
def test_evaluate_equals_three_calls(S, C, flags):
    """plk_evaluate (one call) == plk_update_pmatrices + plk_update_partials +
    plk_root_loglik, bitwise, including the block sums the JIT kernel forms itself."""
    et, m, alph, rates, probs, states = _random_problem(S, C, 40, 9000, seed=12)
    eng = engine_for(et, S, C, 9000, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | flags)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    ops = phylo.split_ops(et.ops)
    for scale in (1.0, 1.3):   # a second evaluation at other branch lengths
        t = et.brlen[br] * scale
        lnl_e, blocks_e = eng.evaluate(br, t, ops, et.root)
        eng.update_pmatrices(br, t)
        eng.update_partials(ops)
        lnl_3, _, blocks_3 = eng.root_loglik(et.root, want_blocks=True)
        assert lnl_e == lnl_3 and np.array_equal(blocks_e, blocks_3)
        lo, so = oracle_for(et, states, alph.init_table, rates, probs, m.pi, [m],
                            pmats=engine_pmats(eng, et))
        assert abs(lnl_e - lo) <= REL * abs(lo)


@pytest.mark.parametrize("C,scaling,n_patterns", [(4, False, 9000), (1, False, 4096), (4, True, 5000),
                                                   (2, False, 130)])
def test_pmat4_and_block_sums(C, scaling, n_patterns):
    """The 4-state K4 (pmat4_kernel: a thread per row of P): P, r dP, r^2 d2P against
    V diag(e^{lambda r t}) V^-1 and its derivatives at 1e-13; through the traversal the lnL
    against the oracle for one, several and ragged blocks; a second root reduction without a
    new traversal returns the same block sums."""
    et, m, alph, rates, probs, states = _random_problem(4, C, 40, n_patterns, seed=77, amb=True)
    flags = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY | (plk.PLK_FLAG_SCALING if scaling else 0)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    ops = phylo.split_ops(et.ops)
    eng = engine_for(et, 4, C, n_patterns, states, alph.init_table, rates, probs, m.pi, [m], flags=flags)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    for b in br[:: max(1, len(br) // 7)]:
        P, dP, d2P = eng.get_pmatrix(int(b)), eng.get_dpmatrix(int(b), 1), eng.get_dpmatrix(int(b), 2)
        for c in range(C):
            e = np.exp(m.lam * rates[c] * et.brlen[b])
            want = (m.V * e) @ m.Vinv
            wd = (m.V * (e * m.lam * rates[c])) @ m.Vinv
            wd2 = (m.V * (e * (m.lam * rates[c]) ** 2)) @ m.Vinv
            assert np.max(np.abs(P[c] - want)) <= 1e-13
            assert np.max(np.abs(dP[c] - wd)) <= 1e-13 * max(1.0, np.max(np.abs(wd)))
            assert np.max(np.abs(d2P[c] - wd2)) <= 1e-13 * max(1.0, np.max(np.abs(wd2)))
    res = []
    for scale in (1.0, 1.7):
        lnl, blocks = eng.evaluate(br, et.brlen[br] * scale, ops, et.root)
        lnl2, _, blocks2 = eng.root_loglik(et.root, want_blocks=True)
        assert lnl2 == lnl and np.array_equal(blocks2, blocks)
        assert abs(float(np.add.accumulate(blocks)[-1]) - lnl) <= 1e-12 * abs(lnl)
        res.append(lnl)
    assert eng.kernel_path() == "jit_tree4"
    eng.evaluate(br, et.brlen[br], ops, et.root)
    lo, _ = oracle_for(et, states, alph.init_table, rates, probs, m.pi, [m], scaling=scaling)
    assert abs(res[0] - lo) <= 1e-10 * abs(lo)


@pytest.mark.parametrize("S,C", [(4, 4), (20, 2)])
def test_pmat_request_paths_bitwise(S, C):
    """A P(t) request of more than 160 branches goes through mapped pinned staging, smaller
    ones ride in the kernel arguments: the same branches requested at once (staged) and in
    chunks of 100 (inline) give the same transition matrices and lnL bitwise (NH: a model
    index per branch)."""
    et, m, alph, rates, probs, states = _random_problem(S, C, 120, 700, seed=5)
    rng = np.random.default_rng(9)
    models = [m] + [phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5)) for _ in range(2)] \
        if S == 4 else [m]
    mon = rng.integers(0, len(models), et.n_nodes).astype(np.int32)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    assert len(br) > 160
    ops = phylo.split_ops(et.ops)
    out = []
    for chunk in (len(br), 100):
        eng = engine_for(et, S, C, 700, states, alph.init_table, rates, probs, m.pi, models, model_of_node=mon,
                         flags=plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY)
        res = []
        for scale in (0.7, 1.4):
            for k in range(0, len(br), chunk):
                eng.update_pmatrices(br[k:k + chunk], et.brlen[br[k:k + chunk]] * scale, mon[br[k:k + chunk]])
            eng.update_partials(ops)
            lnl, _, blocks = eng.root_loglik(et.root, want_blocks=True)
            res.append((lnl, blocks, np.stack([eng.get_pmatrix(int(b)) for b in br])))
        out.append(res)
        del eng
    for (l0, b0, p0), (l1, b1, p1) in zip(out[0], out[1]):
        assert l0 == l1 and np.array_equal(b0, b1) and np.array_equal(p0, p1)


@pytest.mark.parametrize("S,C,n_taxa,scaling", [(4, 4, 64, False), (4, 4, 40, True), (20, 4, 40, True),
                                                 (64, 1, 24, False)])
def test_zero_and_long_branches_vs_oracle(S, C, n_taxa, scaling):
    """Branch lengths the P(t) kernels treat specially: t = 0 (getPij_t returns the identity,
    AbstractSubstitutionModel.cpp:428-431) on internal and tip branches, and t = 60
    (every row at the stationary distribution, P far from the identity) -- through the
    benched lnL-only fused kernels, against the oracle on the engine's own P(t) at 1e-12
    and on the oracle's P(t) at 1e-10."""
    et, m, alph, rates, probs, states = _random_problem(S, C, n_taxa, 1500, seed=S + n_taxa, amb=True)
    rng = np.random.default_rng(S)
    # zero: a sixth of the internal branches and one tip in each of a few cherries (never
    # both tips of a cherry, which could make a site likelihood exactly 0)
    internal = rng.permutation([n for n in range(et.n_tips, et.n_nodes) if n != et.root])
    zero = list(internal[: len(internal) // 6])
    for parent, kids in et.ops[:4]:
        if all(k < et.n_tips for k in kids):
            zero.append(int(kids[0]))
    long_ = [int(n) for n in internal[len(internal) // 6: len(internal) // 6 + 3]]
    et.brlen[zero] = 0.0
    et.brlen[long_] = 60.0
    pick = np.array(zero)
    flags = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY | (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, S, C, 1500, states, alph.init_table, rates, probs, m.pi, [m], flags=flags)
    lnl, site, _ = run_engine(eng, et)
    for b in pick:
        assert np.array_equal(eng.get_pmatrix(int(b)), np.broadcast_to(np.eye(S), (C, S, S)))
    lo, so = oracle_for(et, states, alph.init_table, rates, probs, m.pi, [m], scaling=scaling,
                        pmats=engine_pmats(eng, et))
    check(lnl, site, lo, so)
    lo2, _ = oracle_for(et, states, alph.init_table, rates, probs, m.pi, [m], scaling=scaling)
    assert abs(lnl - lo2) <= 1e-10 * abs(lo2)


def test_get_partials_matches_recomputation():
    et, m, alph, rates, probs, states = _random_problem(4, 4, 6, 300, seed=8)
    eng = engine_for(et, 4, 4, 300, states, alph.init_table, rates, probs, m.pi, [m])
    run_engine(eng, et)
    # first op's partial = product over its children of P . L
    p, ch = et.ops[0]
    L = eng.get_partials(p)
    acc = np.ones((300, 4, 4))
    for c in ch:
        P = eng.get_pmatrix(c)
        Lc = alph.init_table[states[c]][:, None, :] if c < et.n_tips else eng.get_partials(c)
        acc *= np.einsum("cxy,icy->icx", P, np.broadcast_to(Lc, (300, 4, 4)))
    assert np.allclose(L, acc, rtol=1e-13, atol=0)


# ---------------------------------------------------------------- errors (reference exception behaviour)

def test_errors():
    eng = plk.Engine(0, 4, 4, 100, 4, 2, 1)
    eng.set_code_table(phylo.DNA.init_table)
    with pytest.raises(plk.PlkError) as ei:
        eng.set_tip_codes(0, np.full(100, 200, dtype=np.uint8))
    assert ei.value.code == -6          # BadIntException analogue
    with pytest.raises(plk.PlkError) as ei:
        eng.update_partials([(4, (0, 1), 0)])
    assert ei.value.code == -5          # P matrices not set yet
    with pytest.raises(plk.PlkError) as ei:
        eng.update_partials([(1, (0, 2), 0)])
    assert ei.value.code == -1          # parent is a tip


# ---------------------------------------------------------------- full-size config 2 (properties)

@pytest.mark.slow
def test_config2_full_size_properties():
    """BASELINE config 2 at full size (1M patterns, 64 taxa): oracle on a 20k-pattern
    prefix (patterns are independent), bitwise shard invariance and determinism."""
    wl = workload.make_workload("gtr_g4_dna_1M_64")
    ev = workload.Evaluator(wl, 0, 0, wl.n_patterns)
    lnl, _, blocks = ev.step()
    lnl2, _, _ = ev.step()
    assert np.isfinite(lnl) and lnl == lnl2
    _, sites, _ = ev.eng.root_loglik(wl.et.root, want_sites=True)
    n = 20000
    states = wl.simulate(0, n).astype(np.int32)
    lo, so = oracle_for(wl.et, states, phylo.DNA.init_table, wl.rates, wl.probs, wl.root_freqs, wl.models)
    assert np.allclose(sites[:n], so, rtol=REL, atol=0)
    # 2-way shard at a block boundary
    cut = 61 * 4096
    e1 = workload.Evaluator(wl, 0, 0, cut)
    b1 = e1.step()[2]
    del e1
    e2 = workload.Evaluator(wl, 0, cut, wl.n_patterns)
    b2 = e2.step()[2]
    assert np.array_equal(np.concatenate([b1, b2]), blocks)


# ---------------------------------------------------------------- fused 4-state traversal modes

MODES = {"materialize": 0, "lnl_only": plk.PLK_FLAG_LNL_ONLY, "levelwise": plk.PLK_FLAG_LEVELWISE}


def _caterpillar(n, seed=3, lo=0.02, hi=0.2):
    rng = np.random.default_rng(seed)
    s = "t0:%.4f" % rng.uniform(lo, hi)
    for i in range(1, n - 1):
        s = "(%s,t%d:%.4f):%.4f" % (s, i, rng.uniform(lo, hi), rng.uniform(lo, hi))
    return phylo.Tree.from_newick("(%s,t%d:%.4f);" % (s, n - 1, rng.uniform(lo, hi)))


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("C,tree_kind,n_patterns,scaling", [
    (4, "balanced64", 3000, False), (1, "balanced64", 777, False), (2, "balanced64", 1000, True),
    (4, "caterpillar40", 900, False), (4, "caterpillar40", 900, True), (1, "caterpillar40", 300, True),
    (4, "balanced300", 513, True)])
def test_s4_modes_vs_oracle(mode, C, tree_kind, n_patterns, scaling):
    if tree_kind.startswith("balanced"):
        tree = phylo.balanced_tree(int(tree_kind[8:]), seed=17, lo=0.05, hi=0.4)
    else:
        tree = _caterpillar(int(tree_kind[11:]))
    et = phylo.engine_tree(tree)
    rng = np.random.default_rng(C * 7 + n_patterns)
    m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5))
    rates, probs = phylo.gamma_rates(C, 0.5) if C > 1 else (np.ones(1), np.ones(1))
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.DNA, n_patterns, scaling, True, 5)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    mask = rng.random(states.shape) < 0.05
    states[mask] = rng.integers(4, 15, size=mask.sum())       # ambiguity codes
    flags = plk.PLK_FLAG_NONNEG_GUARD | MODES[mode] | (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, 4, C, n_patterns, states, phylo.DNA.init_table, rates, probs, m.pi, [m], flags=flags)
    lnl, site, blocks = run_engine(eng, et)
    lo, so = oracle_for(et, states, phylo.DNA.init_table, rates, probs, m.pi, [m], scaling=scaling)
    check(lnl, site, lo, so)
    # partials of an interior node are available in every mode (recomputed on demand)
    p, ch = et.ops[len(et.ops) // 2]
    L = eng.get_partials(p)
    assert np.all(np.isfinite(L)) and L.shape == (n_patterns, C, 4)
    # a second evaluation is bitwise identical
    lnl2, site2, _ = run_engine(eng, et)
    assert lnl2 == lnl and np.array_equal(site2, site)


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("C,tree_kind,n_patterns,scaling", [
    (4, "balanced64", 700, False), (1, "balanced64", 333, True), (2, "caterpillar30", 400, True),
    (4, "caterpillar30", 300, False), (3, "balanced100", 257, True)])
def test_s20_modes_vs_oracle(mode, C, tree_kind, n_patterns, scaling):
    """20 states in every traversal mode (jit_treeM lnL-only / materialising, levelwise K2),
    against the oracle."""
    if tree_kind.startswith("balanced"):
        tree = phylo.balanced_tree(int(tree_kind[8:]), seed=19, lo=0.05, hi=0.4)
    else:
        tree = _caterpillar(int(tree_kind[11:]))
    et = phylo.engine_tree(tree)
    m = phylo.lg08()
    rates, probs = phylo.gamma_rates(C, 0.7) if C > 1 else (np.ones(1), np.ones(1))
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.PROTEIN, n_patterns, scaling, True, 6)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    rng = np.random.default_rng(n_patterns)
    mask = rng.random(states.shape) < 0.05
    states[mask] = rng.integers(20, phylo.PROTEIN.n_codes, size=mask.sum())   # B / Z / X ...
    flags = plk.PLK_FLAG_NONNEG_GUARD | MODES[mode] | (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, 20, C, n_patterns, states, phylo.PROTEIN.init_table, rates, probs, m.pi, [m], flags=flags)
    lnl, site, _ = run_engine(eng, et)
    # pruning on identical P(t): per-pattern 1e-12
    lo, so = oracle_for(et, states, phylo.PROTEIN.init_table, rates, probs, m.pi, [m], scaling=scaling,
                        pmats=engine_pmats(eng, et))
    check(lnl, site, lo, so)
    # end to end (GPU eigen-reconstructed P vs the oracle's own Jacobi P): north-star 1e-10 on lnL
    # (small P entries of the 20-state model carry ~1e-16 absolute = up to 1e-10 relative noise)
    lo2, _ = oracle_for(et, states, phylo.PROTEIN.init_table, rates, probs, m.pi, [m], scaling=scaling)
    assert abs(lnl - lo2) <= 1e-10 * abs(lo2)
    p, ch = et.ops[len(et.ops) // 2]
    L = eng.get_partials(p)
    assert np.all(np.isfinite(L)) and L.shape == (n_patterns, C, 20)
    lnl2, site2, _ = run_engine(eng, et)
    assert lnl2 == lnl and np.array_equal(site2, site)


@pytest.mark.parametrize("C,tree_kind,n_patterns,scaling,mode,extra", [(*c, "")[:6] for c in [
    (4, "balanced64", 3000, False, "lnl_only"), (4, "balanced64", 1000, False, "materialize"),
    (2, "balanced64", 700, True, "lnl_only"), (1, "caterpillar40", 300, True, "materialize"),
    (4, "caterpillar40", 900, False, "lnl_only"), (4, "balanced300", 513, True, "lnl_only"),
    (4, "caterpillar200long", 600, True, "lnl_only"), (2, "caterpillar200long", 300, True, "materialize"),
    # cherry pair tables (every cherry with 4 codes; within a small budget) and G groups per
    # workgroup with a ragged last super-block
    (4, "balanced64", 3000, False, "lnl_only", "acgt"), (4, "balanced64", 1000, False, "materialize", "acgt G=3"),
    (4, "balanced64", 2000, False, "lnl_only", "acgt G=4 PAIR_KB=20"), (2, "balanced300", 513, True, "lnl_only", "G=3"),
    (4, "balanced300", 700, True, "materialize", "acgt G=4"), (4, "balanced64", 700, False, "lnl_only", "PAIR_KB=0"),
    (1, "caterpillar40", 300, True, "materialize", "acgt G=3"),
    # rescaling cherry contribution units: a code whose vector is 1e-80 drives cherry
    # partials below 2^-256, so the tables' precomputed joint checks must fire
    (4, "balanced64", 1500, True, "lnl_only", "tiny"), (2, "balanced300", 900, True, "lnl_only", "tiny G=3"),
    (4, "balanced64", 700, True, "lnl_only", "tiny CIW=0")]])
def test_jit_tree4_bitwise_equals_interpreter(C, tree_kind, n_patterns, scaling, mode, extra, monkeypatch):
    """The tree-specialised kernel (plk_jit.hpp, hiprtc) against the interpreter
    (tree4_kernel) on the same program: lnL, per-pattern lnL, block sums and every
    interior partial bitwise; and the oracle at 1e-12.  The long-branch caterpillar
    drives partials below 2^-256 (rescaling in both kernels)."""
    for kv in extra.split():
        if "=" in kv:
            k, v = kv.split("=")
            set_tune(monkeypatch, "JIT_" + k, v)
    if tree_kind.startswith("balanced"):
        tree = phylo.balanced_tree(int(tree_kind[8:]), seed=23, lo=0.05, hi=0.4)
    elif tree_kind.endswith("long"):
        tree = _caterpillar(int(tree_kind[11:-4]), seed=5, lo=0.5, hi=1.5)
    else:
        tree = _caterpillar(int(tree_kind[11:]), seed=5)
    et = phylo.engine_tree(tree)
    rng = np.random.default_rng(C * 11 + n_patterns)
    m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5))
    rates, probs = phylo.gamma_rates(C, 0.5) if C > 1 else (np.ones(1), np.ones(1))
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.DNA, n_patterns, scaling, True, 5)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    init = phylo.DNA.init_table
    if "tiny" in extra.split():
        init = np.array(init, dtype=np.float64, copy=True)
        init[4] = 1e-80
        mask = rng.random(states.shape) < 0.3
        states[mask] = 4
    elif "acgt" not in extra.split():
        mask = rng.random(states.shape) < 0.05
        states[mask] = rng.integers(4, 15, size=mask.sum())
    flags = plk.PLK_FLAG_NONNEG_GUARD | MODES[mode] | (plk.PLK_FLAG_SCALING if scaling else 0)
    res = {}
    for kernel in ("0", "1"):
        set_tune(monkeypatch, "JIT", kernel)
        eng = engine_for(et, 4, C, n_patterns, states, init, rates, probs, m.pi, [m], flags=flags)
        lnl, site, blocks = run_engine(eng, et)
        assert eng.kernel_path() == ("jit_tree4" if kernel == "1" else "tree4")
        parts = np.stack([eng.get_partials(p) for p, _ in et.ops])
        res[kernel] = (lnl, site, blocks, parts)
        del eng
    (l0, s0, b0, p0), (l1, s1, b1, p1) = res["0"], res["1"]
    assert l0 == l1 and np.array_equal(s0, s1) and np.array_equal(b0, b1) and np.array_equal(p0, p1)
    if tree_kind.endswith("long") or "tiny" in extra.split():
        assert s1.min() < -256 * np.log(2)   # partials did go through rescaling
    lo, so = oracle_for(et, states, init, rates, probs, m.pi, [m], scaling=scaling)
    check(l1, s1, lo, so)


@pytest.mark.parametrize("C,tree_kind,n_patterns,guard,tune", [
    (4, "balanced64", 3000, True, ""), (4, "balanced64", 777, False, ""), (2, "balanced64", 5000, True, "JIT_G=8"),
    (1, "balanced64", 1500, True, ""), (4, "balanced64", 4100, True, "JIT_QUAD_KB=40"),
    (4, "balanced300", 2000, True, ""), (2, "balanced64", 600, True, "JIT_G=3"), (4, "caterpillar40", 900, True, ""),
    (4, "random120", 2500, True, ""), (2, "balanced64", 70000, True, ""),
    # staged code rows and one pattern per lane (the shapes before direct codes)
    (4, "balanced64", 3000, True, "JIT_DC=0 JIT_PW=1"), (2, "balanced300", 2000, True, "JIT_DC=0"),
    (4, "balanced64", 5000, False, "JIT_PW=1"), (4, "balanced64", 9000, True, "JIT_G=5"),
    # table rows two / three fetchers ahead (PLK_TUNE JIT_RD)
    (4, "balanced64", 3000, True, "JIT_RD=2"), (2, "balanced300", 2000, False, "JIT_RD=3"),
    # fewer patterns than one super-block / one group (the idle groups recompute group 0, store nothing)
    (4, "balanced64", 7, True, ""), (2, "balanced64", 129, False, ""), (1, "balanced64", 1, True, ""),
    # the P(t) load stream of the classes-in-the-wave kernel with one class per wave
    (4, "balanced64", 3000, True, "JIT_PS1=1"),
    # 3 / 2 codes in use (U^4 = 81 / 16 rows: quad rows in the plain order)
    (4, "balanced64:u3", 3000, True, ""), (2, "balanced64:u2", 2000, False, "")])
def test_jit_tree4_quads_bitwise(C, tree_kind, n_patterns, guard, tune, monkeypatch):
    """One class per workgroup with quad units (plk_jit.hpp JitUnit / JitShape::cls: a node whose
    two children are unstored cherries is one table of U^4 rows, the classes' root terms meet in
    cls_root_kernel): lnL, per-pattern lnL and block sums bitwise those of the interpreter
    (tree4_kernel) and of the classes-in-one-workgroup kernel without quads (JIT_QUAD_KB=0), on
    balanced, multi-tier, caterpillar (no quads) and random trees, a partial quad budget, both
    root rules, direct codes (DC, two patterns per lane: the default) and staged code rows; the
    oracle at 1e-12.  ACGT data (4 codes in use: U^4 = 256 rows)."""
    tree_kind, _, ucodes = tree_kind.partition(":u")
    if tree_kind.startswith("balanced"):
        tree = phylo.balanced_tree(int(tree_kind[8:]), seed=23, lo=0.05, hi=0.4)
    elif tree_kind.startswith("random"):
        tree = _random_topology(int(tree_kind[6:]), np.random.default_rng(5), 0.05, 0.4, poly=0.0)
    else:
        tree = _caterpillar(int(tree_kind[11:]), seed=5)
    et = phylo.engine_tree(tree)
    rng = np.random.default_rng(C * 13 + n_patterns)
    m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5))
    rates, probs = phylo.gamma_rates(C, 0.5) if C > 1 else (np.ones(1), np.ones(1))
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.DNA, n_patterns, False, True, 5)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    if ucodes:
        states %= int(ucodes)   # only the first ucodes nucleotide codes in use
    flags = (plk.PLK_FLAG_NONNEG_GUARD if guard else 0) | plk.PLK_FLAG_LNL_ONLY
    res = {}
    for name, extra in (("quads", ""), ("noquads", "JIT_QUAD_KB=0"), ("interp", "JIT=0")):
        monkeypatch.setenv("PLK_TUNE", ",".join(x for x in (tune.replace(" ", ","), extra) if x))
        eng = engine_for(et, 4, C, n_patterns, states, phylo.DNA.init_table, rates, probs, m.pi, [m], flags=flags)
        lnl, site, blocks = run_engine(eng, et)
        lnl2, site2, blocks2 = run_engine(eng, et)    # a second evaluation: the counters reset
        assert lnl2 == lnl and np.array_equal(site2, site) and np.array_equal(blocks2, blocks)
        res[name] = (lnl, site, blocks, eng.traversal_work()["table_nodes"], eng.kernel_path())
        eng.close()
    (lq, sq, bq, tq, pq), (ln, sn, bn, tn, pn), (li, si, bi, ti, pi_) = res["quads"], res["noquads"], res["interp"]
    assert pq == pn == "jit_tree4" and pi_ == "tree4"
    assert lq == ln == li and np.array_equal(sq, sn) and np.array_equal(sq, si)
    assert np.array_equal(bq, bn) and np.array_equal(bq, bi)
    if not tree_kind.startswith("caterpillar"):
        assert tq > tn   # quads replace three table nodes each where cherries replaced one
    lo, so = oracle_for(et, states, phylo.DNA.init_table, rates, probs, m.pi, [m])
    check(lq, sq, lo, so)   # (positive partials: both root rules are the same sum here)


@pytest.mark.parametrize("C,n_taxa,n_patterns,extra", [(4, 512, 30_000, ""), (4, 64, 5_000, "tiny"),
                                                       (2, 150, 3_000, ""), (4, 64, 700, "ambig")])
def test_jit_tree4_direct_codes_classes_in_wave_bitwise(C, n_taxa, n_patterns, extra, monkeypatch):
    """Every class in the wave (rescaling) with direct codes (PLK_TUNE JIT_DC_CIW=1: each wave
    loads its own patterns' unit codes, up to 32 units in two 16-byte words, one barrier per
    super-block): lnL, per-pattern lnL and block sums bitwise those of the staged code rows,
    over two evaluations; the oracle at 1e-12."""
    tree = phylo.balanced_tree(n_taxa, seed=31, lo=0.05, hi=0.4) if n_taxa != 150 else \
        _random_topology(150, np.random.default_rng(8), 0.05, 0.4, poly=0.0)
    et = phylo.engine_tree(tree)
    rng = np.random.default_rng(C * 17 + n_patterns)
    m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5))
    rates, probs = phylo.gamma_rates(C, 0.5)
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.DNA, n_patterns, True, True, 5)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    init = phylo.DNA.init_table
    if extra == "tiny":
        init = np.array(init, dtype=np.float64, copy=True)
        init[4] = 1e-80
        states[rng.random(states.shape) < 0.3] = 4
    elif extra == "ambig":
        mask = rng.random(states.shape) < 0.05
        states[mask] = rng.integers(4, 15, size=mask.sum())
    flags = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY | plk.PLK_FLAG_SCALING
    res = {}
    for name, tune in (("rows", "JIT_DC_CIW=0"), ("dc", "JIT_DC_CIW=1")):
        monkeypatch.setenv("PLK_TUNE", tune)
        eng = engine_for(et, 4, C, n_patterns, states, init, rates, probs, m.pi, [m], flags=flags)
        a = run_engine(eng, et)
        b = run_engine(eng, et)
        assert a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
        assert eng.kernel_path() == "jit_tree4"
        res[name] = a
        eng.close()
    (l0, s0, b0), (l1, s1, b1) = res["rows"], res["dc"]
    assert l0 == l1 and np.array_equal(s0, s1) and np.array_equal(b0, b1)
    if extra == "tiny":
        assert s1.min() < -256 * np.log(2)   # rescaling fired
    lo, so = oracle_for(et, states, init, rates, probs, m.pi, [m], scaling=True)
    check(l1, s1, lo, so)


@pytest.mark.parametrize("C,n_taxa,n_patterns,scaling", [(4, 64, 320_000, False), (4, 512, 60_000, True)])
def test_jit_tree4_dynamic_superblocks_bitwise(C, n_taxa, n_patterns, scaling, monkeypatch):
    """Dynamic super-blocks (workgroups take super-blocks from a per-fragment counter once
    they walk >= 3 of them): lnL, per-pattern lnL and block sums bitwise equal to the static
    order (PLK_TUNE JIT_DYN=0), over repeated lnL-only evaluations of one engine at
    alternating branch lengths (the counters carry over between launches).  320k patterns
    of a 64-taxon tree: one fragment, ~1 700 super-blocks on ~512 workgroups; the 512-taxon
    tree with rescaling: eight 64-tip fragments, 32 workgroups each over 118 super-blocks."""
    tree = phylo.balanced_tree(n_taxa, seed=29, lo=0.05, hi=0.4)
    et = phylo.engine_tree(tree)
    rng = np.random.default_rng(n_taxa)
    m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5))
    rates, probs = phylo.gamma_rates(C, 0.5)
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.DNA, n_patterns, scaling, True, 9)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    flags = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY | (plk.PLK_FLAG_SCALING if scaling else 0)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    res = {}
    for dyn in ("0", "1"):
        set_tune(monkeypatch, "JIT_DYN", dyn)
        eng = engine_for(et, 4, C, n_patterns, states, phylo.DNA.init_table, rates, probs, m.pi, [m], flags=flags)
        out = []
        for k in range(7):
            eng.update_pmatrices(br, et.brlen[br] * (1.0 + 0.1 * (k % 2)))
            out.append(run_engine(eng, et))
        assert eng.kernel_path() == "jit_tree4"
        res[dyn] = out
        del eng
    for (l0, s0, b0), (l1, s1, b1) in zip(res["0"], res["1"]):
        assert l0 == l1 and np.array_equal(s0, s1) and np.array_equal(b0, b1)
    assert res["1"][0][0] == res["1"][2][0] and res["1"][1][0] == res["1"][3][0]
    sub = slice(0, 2000)
    lo, so = oracle_for(et, states[:, sub], phylo.DNA.init_table, rates, probs, m.pi, [m], scaling=scaling)
    assert np.allclose(res["1"][0][1][sub], so, rtol=REL, atol=0)


def test_jit_same_shape_fragments_share_code(tmp_path, monkeypatch):
    """A balanced tree's 64-tip fragments have one shape: the generated kernel holds one code
    block for all of them (plk_jit.hpp: per-fragment node / slot bases), and the result is
    the oracle's at 1e-12 (the bitwise interpreter tests cover the other shapes)."""
    monkeypatch.setenv("PLK_JIT_DUMP", str(tmp_path))
    C, n = 4, 1500
    tree = phylo.balanced_tree(256, seed=31, lo=0.05, hi=0.4)
    et = phylo.engine_tree(tree, unroot=False)
    rng = np.random.default_rng(256)
    m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5))
    rates, probs = phylo.gamma_rates(C, 0.5)
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.DNA, n, True, True, 3)
    states = wl.simulate(0, n).astype(np.int32)
    flags = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY | plk.PLK_FLAG_SCALING
    eng = engine_for(et, 4, C, n, states, phylo.DNA.init_table, rates, probs, m.pi, [m], flags=flags)
    lnl, site, _ = run_engine(eng, et)
    assert eng.kernel_path() == "jit_tree4"
    srcs = [open(os.path.join(tmp_path, f)).read() for f in os.listdir(tmp_path) if f.endswith(".hip")]
    src = [x for x in srcs if "plk_jit_tree4" in x and "kFragNB" in x][-1]
    labels = len(__import__("re").findall(r"^    case \d+:$", src, __import__("re").M))
    blocks = src.count("const CPd pmf_ = ")
    assert 2 <= blocks < labels, (labels, blocks)   # the same-shape subtrees share a block; the top has its own
    lo, so = oracle_for(et, states, phylo.DNA.init_table, rates, probs, m.pi, [m], scaling=True)
    check(lnl, site, lo, so)


def test_fused20_partials_equal_levelwise():
    et, m, alph, rates, probs, states = _random_problem(20, 4, 40, 500, seed=33)
    outs = []
    for mode in ("materialize", "levelwise", "lnl_only"):
        eng = engine_for(et, 20, 4, 500, states, alph.init_table, rates, probs, m.pi, [m],
                         flags=plk.PLK_FLAG_NONNEG_GUARD | MODES[mode])
        run_engine(eng, et)
        outs.append(np.stack([eng.get_partials(p) for p, _ in et.ops]))
    assert np.allclose(outs[0], outs[1], rtol=1e-12, atol=0)
    assert np.array_equal(outs[0], outs[2])


def test_fused_partials_equal_levelwise():
    et, m, alph, rates, probs, states = _random_problem(4, 4, 24, 1000, seed=31)
    outs = []
    for mode in ("materialize", "levelwise", "lnl_only"):
        eng = engine_for(et, 4, 4, 1000, states, alph.init_table, rates, probs, m.pi, [m],
                         flags=plk.PLK_FLAG_NONNEG_GUARD | MODES[mode])
        run_engine(eng, et)
        outs.append(np.stack([eng.get_partials(p) for p, _ in et.ops]))
    assert np.allclose(outs[0], outs[1], rtol=1e-13, atol=0)
    assert np.array_equal(outs[0], outs[2])


# ---------------------------------------------------------------- analytic branch derivatives (row f1)

@pytest.mark.parametrize("C,mode", [(4, "materialize"), (4, "lnl_only"), (1, "levelwise"), (2, "materialize")])
def test_branch_derivatives_vs_oracle_finite_differences(C, mode):
    et, m, alph, rates, probs, states = _random_problem(4, C, 12, 700, seed=40 + C)
    flags = plk.PLK_FLAG_NONNEG_GUARD | MODES[mode]
    eng = engine_for(et, 4, C, 700, states, alph.init_table, rates, probs, m.pi, [m], flags=flags)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    for b in (0, et.n_tips, et.ops[0][0], br[-1]):
        d1, d2 = eng.branch_derivatives(int(b))

        def lnl_at(t):
            bl = et.brlen.copy()
            bl[b] = t
            e2 = phylo.EngineTree(et.n_tips, et.n_internal, et.root, et.tip_names, et.ops, bl, {}, [], [])
            return oracle_for(e2, states, alph.init_table, rates, probs, m.pi, [m])[0]

        t = et.brlen[b]
        h = 1e-5
        fd1 = (lnl_at(t + h) - lnl_at(t - h)) / (2 * h)
        h2 = 1e-4
        fd2 = (lnl_at(t + h2) - 2 * lnl_at(t) + lnl_at(t - h2)) / h2 ** 2
        assert abs(d1 - fd1) <= 1e-6 * max(1.0, abs(fd1)), (b, d1, fd1)
        assert abs(d2 - fd2) <= 2e-4 * max(1.0, abs(fd2)), (b, d2, fd2)


@pytest.mark.parametrize("S,C,mode,scaling", [(20, 4, "lnl_only", False), (20, 2, "levelwise", True),
                                              (64, 1, "lnl_only", False), (4, 8, "materialize", False)])
def test_branch_derivatives_any_state_count(S, C, mode, scaling):
    """Row f1 beyond DNA: the levelwise path derivatives (dP / d2P substituted on the
    branch, the path to the root recomputed) against central differences of the oracle."""
    n_pat = 300 if S == 64 else 500
    et, m, alph, rates, probs, states = _random_problem(S, C, 10, n_pat, seed=50 + S + C)
    flags = plk.PLK_FLAG_NONNEG_GUARD | MODES[mode] | (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, S, C, n_pat, states, alph.init_table, rates, probs, m.pi, [m], flags=flags)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    pm = engine_pmats(eng, et)
    for b in (0, et.n_tips, br[-1]):
        d1, d2 = eng.branch_derivatives(int(b))

        def lnl_at(t):
            bl = et.brlen.copy()
            bl[b] = t
            e2 = phylo.EngineTree(et.n_tips, et.n_internal, et.root, et.tip_names, et.ops, bl, {}, [], [])
            return oracle_for(e2, states, alph.init_table, rates, probs, m.pi, [m], scaling=scaling)[0]

        t = et.brlen[b]
        h = 1e-5
        fd1 = (lnl_at(t + h) - lnl_at(t - h)) / (2 * h)
        h2 = 1e-4
        fd2 = (lnl_at(t + h2) - 2 * lnl_at(t) + lnl_at(t - h2)) / h2 ** 2
        assert abs(d1 - fd1) <= 1e-6 * max(1.0, abs(fd1)), (b, d1, fd1)
        assert abs(d2 - fd2) <= 2e-4 * max(1.0, abs(fd2)), (b, d2, fd2)
    del pm


@pytest.mark.parametrize("S,C,mode,scaling,n_taxa", [(4, 4, "lnl_only", False, 12), (4, 4, "materialize", True, 3),
                                                     (20, 2, "levelwise", True, 10), (4, 1, "subtree", False, 9)])
def test_root_pair_derivatives_vs_oracle_finite_differences(S, C, mode, scaling, n_taxa):
    """plk_root_pair_derivatives (the reference's BrLenRoot / RootPosition derivatives,
    RNonHomogeneousTreeLikelihood.cpp:391-560, 862-1100): two root sons moved by
    t_a + alpha s, t_b + beta s, against central differences of the oracle along that line.
    n_taxa 3 puts two tips under the root (scratch tip rows)."""
    n_pat = 600
    et, m, alph, rates, probs, states = _random_problem(S, C, n_taxa, n_pat, seed=70 + S + C + n_taxa)
    modes = dict(MODES, subtree=plk.PLK_FLAG_SUBTREE_PATTERNS)
    flags = plk.PLK_FLAG_NONNEG_GUARD | modes[mode] | (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, S, C, n_pat, states, alph.init_table, rates, probs, m.pi, [m], flags=flags)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
    run_engine(eng, et)
    kids = [c for p, ch in et.ops if p == et.root for c in ch]
    a, b = kids[0], kids[1]
    for alpha, beta in ((0.3, 0.7), (0.25, -0.25), (1.0, 0.0)):
        d1, d2 = eng.root_pair_derivatives(int(a), int(b), alpha, beta)

        def lnl_at(s):
            bl = et.brlen.copy()
            bl[a] += alpha * s
            bl[b] += beta * s
            e2 = phylo.EngineTree(et.n_tips, et.n_internal, et.root, et.tip_names, et.ops, bl, {}, [], [])
            return oracle_for(e2, states, alph.init_table, rates, probs, m.pi, [m], scaling=scaling)[0]

        h, h2 = 1e-5, 1e-4
        fd1 = (lnl_at(h) - lnl_at(-h)) / (2 * h)
        fd2 = (lnl_at(h2) - 2 * lnl_at(0.0) + lnl_at(-h2)) / h2 ** 2
        assert abs(d1 - fd1) <= 1e-6 * max(1.0, abs(fd1)), (alpha, beta, d1, fd1)
        assert abs(d2 - fd2) <= 2e-4 * max(1.0, abs(fd2)), (alpha, beta, d2, fd2)
        if beta == 0.0:  # one branch only: the ordinary branch derivative
            e1, e2_ = eng.branch_derivatives(int(a))
            assert abs(d1 - e1) <= 1e-10 * max(1.0, abs(e1)) and abs(d2 - e2_) <= 1e-9 * max(1.0, abs(e2_))
    with pytest.raises(plk.PlkError):
        eng.root_pair_derivatives(int(a), int(a), 0.5, 0.5)


def test_branch_derivatives_require_dp():
    et, m, alph, rates, probs, states = _random_problem(4, 4, 6, 100, seed=3)
    eng = engine_for(et, 4, 4, 100, states, alph.init_table, rates, probs, m.pi, [m])
    run_engine(eng, et)
    with pytest.raises(plk.PlkError) as ei:
        eng.branch_derivatives(0)
    assert ei.value.code == -5


# ---------------------------------------------------------------- per-subtree pattern compression (row f3)

@pytest.mark.parametrize("C,tree_kind,n_patterns,scaling,amb", [
    (4, "balanced64", 5000, False, False), (4, "balanced64", 3000, False, True), (1, "caterpillar40", 700, True, True),
    (2, "balanced300", 900, True, False), (4, "caterpillar200long", 400, True, False)])
def test_subtree_patterns_bitwise_vs_uncompressed(C, tree_kind, n_patterns, scaling, amb):
    """PLK_FLAG_SUBTREE_PATTERNS (the reference's usePatterns=true, links built from the
    data) gives bitwise the uncompressed traversal's lnL, per-site lnL, block sums and every
    node's partial (expanded through the links), computes fewer node updates, and matches
    the oracle's own usePatterns=true path at 1e-12."""
    if tree_kind.startswith("balanced"):
        tree = phylo.balanced_tree(int(tree_kind[8:]), seed=29, lo=0.05, hi=0.4)
    elif tree_kind.endswith("long"):
        tree = _caterpillar(int(tree_kind[11:-4]), seed=7, lo=0.5, hi=1.5)
    else:
        tree = _caterpillar(int(tree_kind[11:]), seed=7)
    et = phylo.engine_tree(tree)
    rng = np.random.default_rng(C * 13 + n_patterns)
    m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5))
    rates, probs = phylo.gamma_rates(C, 0.5) if C > 1 else (np.ones(1), np.ones(1))
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.DNA, n_patterns, scaling, True, 9)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    if amb:
        mask = rng.random(states.shape) < 0.05
        states[mask] = rng.integers(4, 15, size=mask.sum())
    sc = plk.PLK_FLAG_SCALING if scaling else 0
    ref = engine_for(et, 4, C, n_patterns, states, phylo.DNA.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | sc)
    l0, s0, b0 = run_engine(ref, et)
    p0 = np.stack([ref.get_partials(p) for p, _ in et.ops])
    del ref
    eng = engine_for(et, 4, C, n_patterns, states, phylo.DNA.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | sc | plk.PLK_FLAG_SUBTREE_PATTERNS)
    l1, s1, b1 = run_engine(eng, et)
    assert eng.kernel_path() == "subtree_patterns"
    p1 = np.stack([eng.get_partials(p) for p, _ in et.ops])
    assert l0 == l1 and np.array_equal(s0, s1) and np.array_equal(b0, b1) and np.array_equal(p0, p1)
    assert eng.compressed_work() < n_patterns * et.n_internal
    # a second evaluation at other branch lengths reuses the links
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    l2, _ = eng.evaluate(br, et.brlen[br] * 1.2, phylo.split_ops(et.ops), et.root)
    assert np.isfinite(l2) and l2 != l1
    ss, sons, lr = et.son_arrays()
    lo, so, _, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, phylo.DNA.init_table, engine_pmats(eng, et), probs,
                                      m.pi, use_patterns=True, scaling=scaling, want_sites=True)
    check(l2, eng.root_loglik(et.root, want_sites=True)[1], lo, so)


def test_subtree_patterns_follow_new_tip_codes():
    """New tip codes invalidate the links: the compressed engine then agrees with a fresh
    uncompressed engine on the new data."""
    et, m, alph, rates, probs, states = _random_problem(4, 4, 24, 2000, seed=41)
    eng = engine_for(et, 4, 4, 2000, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_SUBTREE_PATTERNS)
    run_engine(eng, et)
    states2 = states.copy()
    states2[3] = np.random.default_rng(1).integers(0, 4, size=states.shape[1])
    eng.set_tip_codes(3, states2[3].astype(np.uint8))
    l1, s1, _ = run_engine(eng, et)
    ref = engine_for(et, 4, 4, 2000, states2, alph.init_table, rates, probs, m.pi, [m])
    l0, s0, _ = run_engine(ref, et)
    assert l0 == l1 and np.array_equal(s0, s1)


@pytest.mark.parametrize("S,C,scaling", [(4, 4, False), (4, 2, True), (20, 2, False), (64, 1, True)])
def test_subtree_patterns_polytomy(S, C, scaling):
    """Per-subtree compression on polytomies of five and four children (the links kernels take
    the children three at a time, their product in order): against the oracle at 1e-12 and
    the uncompressed traversal's lnL (the same products; rescaling can only fire at other
    points, by exact powers of two)."""
    t = phylo.Tree.from_newick("((a:0.1,b:0.2,c:0.05,d:0.3,e:0.12):0.1,(f:0.2,g:0.1,h:0.4,i:0.3):0.05,j:0.3,k:0.2);")
    et = phylo.engine_tree(t)
    assert max(len(ch) for _, ch in et.ops) >= 5
    rng = np.random.default_rng(S + C)
    m = {4: lambda: phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5)), 20: phylo.lg08,
         64: lambda: phylo.yn98(2.0, 0.4)}[S]()
    alph = {4: phylo.DNA, 20: phylo.PROTEIN, 64: phylo.CODON}[S]
    rates, probs = phylo.gamma_rates(C, 0.6) if C > 1 else (np.ones(1), np.ones(1))
    n = 1500
    if scaling:
        et.brlen = et.brlen * 8.0
    wl = workload.Workload("p", et, [m], None, rates, probs, m.pi, alph, n, scaling, True, 17)
    states = wl.simulate(0, n).astype(np.int32)
    sc = plk.PLK_FLAG_SCALING if scaling else 0
    res = []
    for mode in (plk.PLK_FLAG_SUBTREE_PATTERNS, plk.PLK_FLAG_LEVELWISE):
        eng = engine_for(et, S, C, n, states, alph.init_table, rates, probs, m.pi, [m],
                         flags=plk.PLK_FLAG_NONNEG_GUARD | mode | sc)
        res.append(run_engine(eng, et))
        if mode == plk.PLK_FLAG_SUBTREE_PATTERNS:
            assert eng.kernel_path() == "subtree_patterns"
            pm = engine_pmats(eng, et)
    (l1, s1, _), (l2, s2, _) = res
    lo, so = oracle_for(et, states, alph.init_table, rates, probs, m.pi, [m], scaling=scaling, pmats=pm)
    check(l1, s1, lo, so)
    assert np.allclose(s1, s2, rtol=1e-13, atol=0)


@pytest.mark.parametrize("S,C", [(4, 2), (20, 1)])
def test_subtree_patterns_wide_polytomy_rescale(S, C):
    """A root polytomy of nine cherries whose partials sit near 2^-150 (a code whose vector is
    1e-23 on 80 % of the cells): the running product must be rescaled after every
    group of three children in the compressed links kernels as in the uncompressed
    traversal's ACCUMULATE ops -- checked once at the end it underflows to 0 (-inf sites).
    Compressed == uncompressed (bitwise for 4 states: the same arithmetic; 1e-13 for 20),
    both == the oracle (which rescales after every third son the same way) at 1e-12."""
    rng = np.random.default_rng(90 + S)
    clade = lambda k: f"(t{k}a:0.3,t{k}b:0.4):0.2"
    et = phylo.engine_tree(phylo.Tree.from_newick("(" + ",".join(clade(k) for k in range(9)) + ");"))
    assert max(len(ch) for _, ch in et.ops) == 9
    m = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5)) if S == 4 else phylo.lg08()
    alph = phylo.DNA if S == 4 else phylo.PROTEIN
    rates, probs = phylo.gamma_rates(C, 0.6) if C > 1 else (np.ones(1), np.ones(1))
    n = 900
    states = rng.choice(S, size=(et.n_tips, n), p=m.pi).astype(np.int32)
    init = np.array(alph.init_table, dtype=np.float64, copy=True)
    code = alph.n_codes - 1
    init[code] = 1e-23
    states[rng.random(states.shape) < 0.8] = code
    res = []
    for mode in (plk.PLK_FLAG_SUBTREE_PATTERNS, plk.PLK_FLAG_LEVELWISE):
        eng = engine_for(et, S, C, n, states, init, rates, probs, m.pi, [m],
                         flags=plk.PLK_FLAG_NONNEG_GUARD | mode | plk.PLK_FLAG_SCALING)
        res.append(run_engine(eng, et))
        if mode == plk.PLK_FLAG_SUBTREE_PATTERNS:
            assert eng.kernel_path() == "subtree_patterns"
            pm = engine_pmats(eng, et)
    (l1, s1, _), (l2, s2, _) = res
    assert np.all(np.isfinite(s1)) and s1.min() < -3 * 256 * np.log(2)   # several rescales per site
    if S == 4:
        assert l1 == l2 and np.array_equal(s1, s2)
    else:
        assert np.allclose(s1, s2, rtol=1e-13, atol=0)
    lo, so = oracle_for(et, states, init, rates, probs, m.pi, [m], scaling=True, pmats=pm)
    check(l1, s1, lo, so)


def test_subtree_patterns_errors():
    et, m, alph, rates, probs, states = _random_problem(4, 2, 12, 300, seed=43)
    with pytest.raises(plk.PlkError):   # no compressed double-recursive passes
        plk.Engine(0, 4, 2, 300, et.n_tips, et.n_internal, 1,
                   plk.PLK_FLAG_SUBTREE_PATTERNS | plk.PLK_FLAG_DOUBLE_RECURSIVE)
    eng = engine_for(et, 4, 2, 300, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_SUBTREE_PATTERNS)
    run_engine(eng, et)
    ops = phylo.split_ops(et.ops)
    with pytest.raises(plk.PlkError):   # a child produced by an earlier call: links need the whole subtree
        eng.update_partials(ops[-1:])


@pytest.mark.parametrize("S,C,n_taxa,n_patterns,scaling,amb", [
    (20, 4, 24, 900, False, True), (20, 2, 40, 700, True, False), (20, 1, 9, 300, False, False),
    (64, 1, 16, 600, False, True), (64, 1, 30, 400, True, False), (64, 1, 8, 300, False, False)])
def test_subtree_patterns_any_state_count(S, C, n_taxa, n_patterns, scaling, amb):
    """Row f3 beyond DNA: per-subtree compression for 20 and 64 states
    (partials_links_generic_kernel) against the oracle's own usePatterns = true pruning
    at 1e-12 and against the uncompressed levelwise kernels (K2 / K3) at 1e-12 (lnL,
    per-pattern lnL, block sums and every partial expanded through the links)."""
    et, m, alph, rates, probs, states = _random_problem(S, C, n_taxa, n_patterns, seed=90 + S + C, amb=amb)
    sc = plk.PLK_FLAG_SCALING if scaling else 0
    ref = engine_for(et, S, C, n_patterns, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | sc | plk.PLK_FLAG_LEVELWISE)
    l0, s0, b0 = run_engine(ref, et)
    p0 = np.stack([ref.get_partials(p) for p, _ in et.ops])
    del ref
    eng = engine_for(et, S, C, n_patterns, states, alph.init_table, rates, probs, m.pi, [m],
                     flags=plk.PLK_FLAG_NONNEG_GUARD | sc | plk.PLK_FLAG_SUBTREE_PATTERNS)
    l1, s1, b1 = run_engine(eng, et)
    assert eng.kernel_path() == "subtree_patterns"
    p1 = np.stack([eng.get_partials(p) for p, _ in et.ops])
    assert abs(l0 - l1) <= 1e-12 * abs(l0) and np.allclose(s0, s1, rtol=1e-12, atol=0)
    assert np.allclose(b0, b1, rtol=1e-12, atol=0) and np.allclose(p0, p1, rtol=1e-12, atol=1e-300)
    assert eng.compressed_work() < n_patterns * et.n_internal
    ss, sons, lr = et.son_arrays()
    lo, so, _, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, alph.init_table, engine_pmats(eng, et), probs,
                                      m.pi, use_patterns=True, scaling=scaling, want_sites=True)
    check(l1, s1, lo, so)


@pytest.mark.parametrize("S,C", [(4, 4), (20, 2), (64, 1)])
def test_subtree_patterns_derivatives(S, C):
    """Branch derivatives on a compressed handle: the traversal is re-run uncompressed once
    (slots expanded) and the path derivatives equal those of an uncompressed handle; the
    next compressed evaluation is unchanged."""
    et, m, alph, rates, probs, states = _random_problem(S, C, 12, 500, seed=7 + S)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    res = []
    for fl in (0, plk.PLK_FLAG_SUBTREE_PATTERNS):
        eng = engine_for(et, S, C, 500, states, alph.init_table, rates, probs, m.pi, [m],
                         flags=plk.PLK_FLAG_NONNEG_GUARD | fl)
        eng.update_pmatrices(br, et.brlen[br], deriv_mask=7)
        l, _, _ = run_engine(eng, et)
        d = [eng.branch_derivatives(int(b)) for b in (0, et.n_tips, br[-1])]
        l2, _, _ = run_engine(eng, et)
        res.append((l, d, l2))
    (la, da, la2), (lb, db, lb2) = res
    assert abs(la - lb) <= 1e-12 * abs(la) and lb == lb2
    for (a1, a2), (b1, b2) in zip(da, db):
        assert abs(a1 - b1) <= 1e-10 * max(1.0, abs(a1)) and abs(a2 - b2) <= 1e-9 * max(1.0, abs(a2))


@pytest.mark.gpu
@pytest.mark.parametrize("S,C,scaling,variant", [
    (20, 4, True, ""), (20, 2, False, "amb"), (20, 4, True, "tiny"), (64, 1, False, ""), (64, 1, True, "tiny")])
def test_treeM_cherry_tables_vs_oracle(S, C, scaling, variant, monkeypatch):
    """treeM with cherry contribution tables (T_CHERRY rows, plk_treeM.hpp) against the
    oracle.  "tiny": one code's vector is 1e-80, so cherry partials fall below 2^-256 and the
    tables' precomputed joint rescale must fire."""
    et, m, alph, rates, probs, states = _random_problem(S, C, 48 if S == 20 else 24, 700, seed=S + C,
                                                        amb=variant == "amb")
    init = alph.init_table
    if variant == "tiny":
        init = np.array(init, dtype=np.float64, copy=True)
        code = alph.n_codes - 1
        init[code] = 1e-80
        rng = np.random.default_rng(7)
        states[rng.random(states.shape) < 0.3] = code
    flags = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY | (plk.PLK_FLAG_SCALING if scaling else 0)
    set_tune(monkeypatch, "JITM", "0")   # the treeM interpreter (20 states default to jit_treeM)
    eng = engine_for(et, S, C, 700, states, init, rates, probs, m.pi, [m], flags=flags)
    l1, s1, b1 = run_engine(eng, et)
    assert eng.kernel_path() == "treeM"
    assert eng.traversal_work()["table_nodes"] > 0
    if variant == "tiny":
        assert s1.min() < -256 * np.log(2)
    lo, so = oracle_for(et, states, init, rates, probs, m.pi, [m], scaling=scaling)
    check(l1, s1, lo, so, rel=1e-10)


@pytest.mark.gpu
def test_pmat64s_kernel_bitwise():
    """The 64-state K4 (pmat64s_kernel: register-blocked, LDS-staged, split in four row slabs)
    gives the generic kernel's results bitwise (a P-only request runs pmat64s_kernel, a
    P + dP + d2P request the generic pmat_kernel): every P(t) and the traversal's lnL."""
    et, m, alph, rates, probs, states = _random_problem(64, 1, 24, 500, seed=64, amb=True)
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    ops = phylo.split_ops(et.ops)
    out = []
    for mask in (plk.PLK_DERIV_P, 7):
        eng = engine_for(et, 64, 1, 500, states, alph.init_table, rates, probs, m.pi, [m],
                         flags=plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY)
        eng.update_pmatrices(br, et.brlen[br], deriv_mask=mask)
        eng.update_partials(ops)
        lnl, site, _ = eng.root_loglik(et.root, want_sites=True)
        out.append((lnl, site, np.stack([eng.get_pmatrix(int(b)) for b in br])))
        del eng
    assert out[0][0] == out[1][0] and np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])


@pytest.mark.parametrize("RX,NB,C,n_taxa,nh", [
    (4, 4, 1, 24, False), (4, 4, 3, 24, True), (4, 4, 1, 100, True), (2, 4, 2, 100, False),
    (2, 2, 1, 24, True), (1, 1, 4, 24, False), (4, 2, 1, 100, False), (1, 4, 1, 100, True),
    (4, 1, 1, 24, True)])
def test_pmat64w_kernel_bitwise(RX, NB, C, n_taxa, nh, monkeypatch):
    """pmat64w_kernel (NB matrices of one model per workgroup sharing every V Vinv product,
    RX rows per wave, PLK_TUNE P64RX / P64NB) against the generic kernel (a P + dP + d2P request)
    and pmat64s_kernel (P64RX=0), bitwise: every P(t), the fused tip tables (through the
    traversal's lnL and site lnL) -- one class or several, one model or a different model
    per branch (runs of one model inside a workgroup), inline requests (<= 160 branches)
    and staged ones (198), and a zero-length branch (identity)."""
    # a 64-code table (n_codes <= 64: the P(t) kernel writes the tip tables) for most cases,
    # the codon alphabet's 65 (the separate tip-table kernel) when NB == 2
    et, m, alph, rates, probs, states = _random_problem(64, C, n_taxa, 300, seed=640 + n_taxa + C, amb=NB == 2)
    if NB != 2:
        alph = phylo.Alphabet("R", 64, {}, np.eye(64))
    models = [m] + ([_random_problem(64, 1, 4, 10, seed=650 + k)[1] for k in range(2)] if nh else [])
    mon = np.random.default_rng(7).integers(0, len(models), et.n_nodes).astype(np.int32) if nh else None
    br = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
    t = et.brlen[br].copy()
    t[len(t) // 3] = 0.0
    ops = phylo.split_ops(et.ops)
    out = []
    for mask, tune in ((7, None), (plk.PLK_DERIV_P, {"P64RX": 0}), (plk.PLK_DERIV_P, {"P64RX": RX, "P64NB": NB})):
        clear_tune(monkeypatch, "P64RX")
        clear_tune(monkeypatch, "P64NB")
        for k, v in (tune or {}).items():
            set_tune(monkeypatch, k, v)
        eng = engine_for(et, 64, C, 300, states, alph.init_table, rates, probs, m.pi, models, model_of_node=mon,
                         flags=plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY)
        eng.update_pmatrices(br, t, None if mon is None else mon[br], deriv_mask=mask)
        eng.update_partials(ops)
        lnl, site, _ = eng.root_loglik(et.root, want_sites=True)
        out.append((lnl, site, np.stack([eng.get_pmatrix(int(b)) for b in br])))
        eng.close()
    assert np.isfinite(out[0][0])
    assert np.array_equal(out[0][2][len(t) // 3], np.stack([np.eye(64)] * C))
    for o in out[1:]:
        assert o[0] == out[0][0] and np.array_equal(o[1], out[0][1]) and np.array_equal(o[2], out[0][2])


# ---------------------------------------------------------------- jit_treeM (20 states, v_mfma_f64_4x4x4_4b)

@pytest.mark.gpu
@pytest.mark.parametrize("C,tree_kind,n_patterns,scaling,mode,variant", [
    (4, "balanced64", 700, False, "lnl_only", ""), (4, "balanced64", 700, True, "materialize", "amb"),
    (1, "balanced64", 333, True, "lnl_only", ""), (2, "caterpillar30", 400, True, "lnl_only", "amb"),
    (3, "balanced100", 257, True, "materialize", ""), (4, "caterpillar30", 300, False, "materialize", ""),
    (4, "balanced160", 513, True, "lnl_only", "amb"), (4, "balanced64", 900, True, "lnl_only", "tiny"),
    (2, "caterpillar30", 500, True, "materialize", "tiny"), (4, "balanced64", 64, False, "lnl_only", "")])
def test_jit_treeM_vs_oracle(C, tree_kind, n_patterns, scaling, mode, variant, monkeypatch):
    """The tree-specialised 20-state kernel (plk_jitm.hpp) against the oracle on identical
    P(t) (per pattern 1e-12), against the treeM interpreter (PLK_JITM=0, 1e-12), and
    self-consistent: a second evaluation and the materialised partials bitwise.  "tiny": a
    code whose vector is 1e-80 forces the joint rescale (cherry tables and in-kernel)."""
    if tree_kind.startswith("balanced"):
        tree = phylo.balanced_tree(int(tree_kind[8:]), seed=31, lo=0.05, hi=0.4)
    else:
        tree = _caterpillar(int(tree_kind[11:]), seed=9)
    et = phylo.engine_tree(tree)
    m = phylo.lg08()
    rates, probs = phylo.gamma_rates(C, 0.6) if C > 1 else (np.ones(1), np.ones(1))
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.PROTEIN, n_patterns, scaling, True, 8)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    rng = np.random.default_rng(C + n_patterns)
    init = phylo.PROTEIN.init_table
    if variant == "amb":
        mask = rng.random(states.shape) < 0.05
        states[mask] = rng.integers(20, phylo.PROTEIN.n_codes, size=mask.sum())
    elif variant == "tiny":
        init = np.array(init, dtype=np.float64, copy=True)
        code = phylo.PROTEIN.n_codes - 1
        init[code] = 1e-80
        states[rng.random(states.shape) < 0.3] = code
    flags = plk.PLK_FLAG_NONNEG_GUARD | MODES[mode] | (plk.PLK_FLAG_SCALING if scaling else 0)
    eng = engine_for(et, 20, C, n_patterns, states, init, rates, probs, m.pi, [m], flags=flags)
    lnl, site, blocks = run_engine(eng, et)
    assert eng.kernel_path() == "jit_treeM"
    lo, so = oracle_for(et, states, init, rates, probs, m.pi, [m], scaling=scaling, pmats=engine_pmats(eng, et))
    check(lnl, site, lo, so)
    if variant == "tiny":
        assert site.min() < -256 * np.log(2)
    lnl2, site2, blocks2 = run_engine(eng, et)
    assert lnl2 == lnl and np.array_equal(site2, site) and np.array_equal(blocks2, blocks)
    parts = np.stack([eng.get_partials(p) for p, _ in et.ops[-4:]])
    assert np.all(np.isfinite(parts))
    # the treeM interpreter on the same inputs
    set_tune(monkeypatch, "JITM", "0")
    ref = engine_for(et, 20, C, n_patterns, states, init, rates, probs, m.pi, [m], flags=flags)
    lr, sr, _ = run_engine(ref, et)
    assert ref.kernel_path() == "treeM"
    check(lnl, site, lr, sr)
    pr = np.stack([ref.get_partials(p) for p, _ in et.ops[-4:]])
    assert np.allclose(parts, pr, rtol=1e-11, atol=1e-300)


@pytest.mark.gpu
@pytest.mark.parametrize("dm,L", [(2, 1), (3, 2), (4, 3), (6, 1)])
def test_jit_treeM_register_depths(dm, L, monkeypatch):
    """Other fragment heights (JITM_DM) and operand fetch lookaheads (JITM_L) give the default
    kernel's results bitwise (different cuts store different partials, but every operation
    per node is the same)."""
    et, m, alph, rates, probs, states = _random_problem(20, 4, 80, 600, seed=77, amb=True)
    flags = plk.PLK_FLAG_NONNEG_GUARD | plk.PLK_FLAG_LNL_ONLY | plk.PLK_FLAG_SCALING
    eng = engine_for(et, 20, 4, 600, states, alph.init_table, rates, probs, m.pi, [m], flags=flags)
    l0, s0, _ = run_engine(eng, et)
    del eng
    set_tune(monkeypatch, "JITM_DM", str(dm))
    set_tune(monkeypatch, "JITM_L", str(L))
    eng = engine_for(et, 20, 4, 600, states, alph.init_table, rates, probs, m.pi, [m], flags=flags)
    l1, s1, _ = run_engine(eng, et)
    assert eng.kernel_path() == "jit_treeM"
    assert np.array_equal(s0, s1) and l0 == l1


