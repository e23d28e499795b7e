"""CPU tests of the host-side logic: the Python helpers (bpp-phyl_amd/phylo.py,
workload.py) and the C++ Bio++ mirror (bpp-phyl_amd/host) against the oracle and
the golden fixtures.  No GPU."""
import json
import os
import subprocess

import numpy as np
import pytest
from scipy.linalg import expm

import oracle
import phylo
import workload
from conftest import run_make

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
HOST = os.path.join(ROOT, "bpp-phyl_amd", "host")


@pytest.fixture(scope="module")
def host_records():
    run_make("-s", "-C", os.path.join(ROOT, "bpp-phyl_amd"))
    run_make("-s", "-j8", "-C", HOST)
    out = subprocess.run([os.path.join(HOST, "bin", "test_host_cpu")], check=True, capture_output=True,
                         text=True).stdout
    return [json.loads(line) for line in out.splitlines() if line.strip()]


def _models(recs):
    return {r["name"]: r for r in recs if r["kind"] == "model"}


# ------------------------------------------------------------------ C++ host mirror

def test_host_gamma_matches_oracle(host_records):
    for r in (x for x in host_records if x["kind"] == "gamma"):
        ro, _ = oracle.gamma_rates(4, r["alpha"])
        assert np.allclose(r["rates"], ro, rtol=1e-12, atol=0)


@pytest.mark.parametrize("name", ["T92", "T92_k2_t03", "GTR", "LG08"])
def test_host_pmatrix_vs_expm_fixture(host_records, name):
    f = np.load(os.path.join(GOLD, "pmatrix.npz"))
    r = _models(host_records)[name]
    S = r["S"]
    assert np.allclose(np.array(r["Q"]).reshape(S, S), f[f"{name}_Q"], atol=1e-14)
    for P, Pe, Pf in zip(r["P"], r["P_eigen"], f[f"{name}_P"]):
        assert np.allclose(np.array(P).reshape(S, S), Pf, atol=1e-13)
        assert np.allclose(np.array(Pe).reshape(S, S), Pf, atol=1e-13)


@pytest.mark.parametrize("name", ["GTR", "LG08"])
def test_host_taylor_branch_vs_expm_fixture(host_records, name):
    """A model whose eigen-system fails the check gets P(t) from the reference's Taylor
    series with scaling and squaring (Model/AbstractSubstitutionModel.cpp:470-492)."""
    f = np.load(os.path.join(GOLD, "pmatrix.npz"))
    r = _models(host_records)[name + "_taylor"]
    S = r["S"]
    for P, Pf in zip(r["P"], f[f"{name}_P"]):
        assert np.allclose(np.array(P).reshape(S, S), Pf, atol=1e-12)


@pytest.mark.parametrize("name,complex_pair", [("L95_complex", True), ("L95_complex2", True),
                                               ("L95_repeated", False), ("L95_rate", True)])
def test_host_l95_nonreversible_pij(host_records, name, complex_pair):
    """L95 (Model/Nucleotide/L95.cpp:56-119) is non-reversible: its eigen-system comes from
    the general real decomposition (complex pairs as (Re v, Im v) column pairs, the
    reference's EigenValue layout) and P(t), dP/dt take the block form of
    Model/AbstractSubstitutionModel.cpp:440-467, 505-537 -- checked against scipy's expm
    of r t Q.  d2P/dt2 follows the reference's block expression (:581-611), restated here
    from the printed eigen-system; off the pair blocks it is r^2 Q^2 P."""
    r = _models(host_records)[name]
    S = 4
    Q = np.array(r["Q"]).reshape(S, S)
    pi = np.array(r["pi"])
    rate = 1.7 if name == "L95_rate" else 1.0
    assert r["nonsingular"] and r["diagonalizable"] == (not complex_pair)
    assert abs(-np.dot(np.diag(Q), pi) - 1) < 1e-13        # normalised
    assert np.allclose(pi @ Q, 0, atol=1e-13)               # pi stationary
    if complex_pair:  # (the repeated-eigenvalue point is the symmetric corner of L95)
        assert not np.allclose(pi[:, None] * Q, (pi[:, None] * Q).T)  # not reversible
    wr, wi = np.array(r["wr"]), np.array(r["wi"])
    V, Vi = np.array(r["V"]).reshape(S, S), np.array(r["Vi"]).reshape(S, S)
    assert np.allclose(V @ Vi, np.eye(S), atol=1e-12)
    ev = list(np.linalg.eigvals(Q))
    for z in wr + 1j * wi:  # the same spectrum (matched one to one)
        j = int(np.argmin([abs(z - e) for e in ev]))
        assert abs(z - ev.pop(j)) < 1e-10
    if complex_pair:
        k = int(np.argmax(wi))
        assert wi[k] > 0 and wi[k + 1] == -wi[k] and wr[k + 1] == wr[k]
    for t, P, dP, d2P in zip(r["t"], r["P"], r["dP"], r["d2P"]):
        E = expm(rate * t * Q)
        assert np.allclose(np.array(P).reshape(S, S), E, atol=1e-12)
        assert np.allclose(np.array(dP).reshape(S, S), rate * Q @ E, atol=1e-11)
        # the reference's d2 block form
        l = rate * t
        dia, up = np.zeros(S), np.zeros(S - 1)
        i = 0
        while i < S:
            e = np.exp(wr[i] * l)
            if wi[i] != 0 and i + 1 < S:
                a, b = wr[i], wi[i]
                s, c = np.sin(b * l), np.cos(b * l)
                dia[i] = dia[i + 1] = rate ** 2 * ((a * a - b * b) * c - 2 * a * b * s) * e
                up[i] = rate ** 2 * ((a * a - b * b) * s - 2 * a * b * c) * e
                i += 2
            else:
                dia[i] = rate ** 2 * wr[i] ** 2 * e
                i += 1
        T = np.diag(dia) + np.diag(up, 1) - np.diag(up, -1)
        assert np.allclose(np.array(d2P).reshape(S, S), V @ T @ Vi, atol=1e-11)
        if not complex_pair:
            assert np.allclose(np.array(d2P).reshape(S, S), rate ** 2 * Q @ Q @ E, atol=1e-11)


def test_host_yn98_properties(host_records):
    r = _models(host_records)["YN98"]
    Q = np.array(r["Q"]).reshape(64, 64)
    pi = np.array(r["pi"])
    stops = [48, 50, 56]  # TAA TAG TGA
    assert np.all(pi[stops] == 0) and abs(pi.sum() - 1) < 1e-14
    assert abs(-np.dot(np.diag(Q), pi) - 1) < 1e-13
    for t, P in zip(r["t"], r["P"]):
        P = np.array(P).reshape(64, 64)
        assert np.allclose(P[stops][:, stops], np.eye(3))
        live = [i for i in range(64) if i not in stops]
        assert np.allclose(P[live].sum(1), 1, atol=1e-12)
        D = pi[:, None] * P
        assert np.allclose(D, D.T, atol=1e-14)
        assert np.allclose(P[np.ix_(live, live)], expm(Q[np.ix_(live, live)] * t), atol=1e-12)
        # the oracle's independent Jacobi path
        assert np.allclose(P, oracle.reversible_pij(Q, pi, t), atol=1e-12)


def test_host_yn98_vs_expm_fixture(host_records):
    """The C++ mirror's YN98 (config 4's model) against the fixture built from the
    independent restatement in tests/golden/make_golden.py: generator, frequencies, and
    P(t) through both getPij_t and the eigen-system."""
    f = np.load(os.path.join(GOLD, "pmatrix.npz"))
    r = _models(host_records)["YN98"]
    assert np.allclose(np.array(r["Q"]).reshape(64, 64), f["YN98_Q"], atol=1e-14)
    assert np.allclose(r["pi"], f["YN98_pi"], atol=1e-16)
    for P, Pe, Pf in zip(r["P"], r["P_eigen"], f["YN98_P"]):
        assert np.allclose(np.array(P).reshape(64, 64), Pf, atol=1e-13)
        assert np.allclose(np.array(Pe).reshape(64, 64), Pf, atol=1e-13)


def test_host_trees(host_records):
    trees = [r for r in host_records if r["kind"] == "tree"]
    assert trees[0]["leaves"] == ["A", "B", "C", "D"] and not trees[0]["rooted"]
    assert trees[1]["ids"] == list(range(7))
    assert trees[2]["unrooted"] == "(a:1,b:2,(c:4,d:5):9);"
    # same unroot semantics in the Python helper
    t = phylo.Tree.from_newick(trees[2]["newick"])
    t.unroot()
    assert [n.name for n in t.root.sons[:2]] == ["a", "b"] and abs(t.root.sons[2].dist - 9.0) < 1e-15


def test_host_model_set_naming(host_records):
    r = next(x for x in host_records if x["kind"] == "modelset")
    assert r["n"] == 6
    # the reference's layout (SubstitutionModelSetTools.cpp:81-175): root frequencies first,
    # every model parameter suffixed _<k>, the global kappa's copies aliased to model 1's
    assert r["names"][0] == "GC.theta" and r["names"][1:3] == ["T92.kappa_1", "T92.theta_1"]
    assert "T92.theta_6" in r["names"] and "T92.kappa_6" in r["names"]
    assert r["independent"] == ["GC.theta", "T92.kappa_1"] + [f"T92.theta_{k}" for k in range(1, 7)]
    assert r["kappa_last"] == 2.5 and r["changed_models"] == 6 and r["kappa_nodes"] == 6
    assert len(r["theta2_nodes"]) == 1
    assert r["theta2"] == 0.7 and r["theta1"] == 0.5


def test_host_simulator_joint_distribution(host_records):
    """NonHomogeneousSequenceSimulator (Simulation/NonHomogeneousSequenceSimulator.cpp:306-353,
    433-483): the leaves of a rooted cherry are drawn from sum_c p_c sum_x pi_x P_a P_b."""
    r = next(x for x in host_records if x["kind"] == "simulator")
    assert r["names"] == ["a", "b"]
    emp, want = np.array(r["empirical"]), np.array(r["expected"])
    assert abs(want.sum() - 1.0) < 1e-12 and abs(emp.sum() - 1.0) < 1e-9
    # binomial standard error per cell at n = 200000: 5 sigma
    se = np.sqrt(want * (1 - want) / r["n"])
    assert np.all(np.abs(emp - want) <= 5 * se + 1e-12), np.max(np.abs(emp - want) / se)


# ------------------------------------------------------------------ Python host helpers

def test_newick_postorder_ids():
    t = phylo.Tree.from_newick("((A:0.01, B:0.02):0.03,C:0.01,D:0.1);")
    assert [n.id for n in t.nodes()] == list(range(6))
    assert t.leaf_names() == ["A", "B", "C", "D"]
    et = phylo.engine_tree(t)
    assert et.n_tips == 4 and et.n_internal == 2
    assert et.brlen_names == [f"BrLen{i}" for i in range(5)]


def test_engine_tree_unroots_and_clamps():
    t = phylo.Tree.from_newick("(((s05:0.1,s04:0.0):0.3,s03:0.0):0.26667,s02:0.06667,s01:0.16667);")
    et = phylo.engine_tree(t)
    assert et.brlen.min() == 0.0  # the root entry
    assert sorted(et.brlen)[1] == phylo.MIN_BRLEN  # zero lengths clamped to 1e-6
    t2 = phylo.balanced_tree(64)
    et2 = phylo.engine_tree(t2)
    assert et2.n_internal == 62 and len(et.ops) == et.n_internal


@pytest.mark.parametrize("name", ["T92", "GTR", "LG08", "YN98"])
def test_python_models_vs_expm(name):
    f = np.load(os.path.join(GOLD, "pmatrix.npz"))
    m = {"T92": phylo.t92(3.0, 0.5), "GTR": phylo.gtr(1.2, 0.4, 0.6, 0.8, 0.5, 0.30, 0.20, 0.25, 0.25),
         "LG08": phylo.lg08(), "YN98": phylo.yn98(2.0, 0.3)}[name]
    if name == "YN98":
        assert np.allclose(m.Q, f["YN98_Q"], atol=1e-14) and np.allclose(m.pi, f["YN98_pi"], atol=1e-16)
    for t, P in zip(f[f"{name}_t"], f[f"{name}_P"]):
        assert np.allclose(m.pij(t), P, atol=1e-13)


def test_split_ops_polytomy():
    ops = phylo.split_ops([(10, (0, 1, 2, 3, 4))])
    assert ops == [(10, (0, 1, 2), 0), (10, (3, 4), 1)]


def test_simulation_is_shard_invariant():
    wl = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=5000)
    a = wl.simulate(0, 5000)
    b = np.concatenate([wl.simulate(0, 1234), wl.simulate(1234, 5000)], axis=1)
    assert np.array_equal(a, b)
    assert a.min() >= 0 and a.max() <= 3
    # empirical base composition close to the model's stationary frequencies
    freq = np.bincount(a.ravel(), minlength=4) / a.size
    assert np.allclose(freq, wl.models[0].pi, atol=0.02)


def test_algorithmic_bytes_cfg2():
    wl = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=10)
    assert wl.algorithmic_bytes_per_pattern() == 15944
    assert abs(wl.algorithmic_bytes_per_pattern() / wl.et.n_internal - 257.16) < 0.01


def test_host_pseudonewton_conjugate_gradient(host_records):
    """optimizeNumericalParameters2 (OPTIMIZATION_NEWTON) on a host-only function whose
    Newton moves overshoot by orders of magnitude (sqrt(1 + x^2) + sqrt(1 + y^2) from
    (10, -7)): the fourth Felsenstein-Churchill correction is the conjugate-gradient search
    of PseudoNewtonOptimizer.cpp:151-170, and the optimiser reaches the minimum (0, 0)."""
    r = next(x for x in host_records if x["kind"] == "pn_cg")
    assert abs(r["f"] - 2.0) < 1e-8 and abs(r["x"]) < 1e-3 and abs(r["y"]) < 1e-3, r
    assert r["evals"] < 2000, r


def test_host_global_clock2_optimisers(host_records):
    """optimizeNumericalParametersWithGlobalClock2 (OptimizationTools.cpp:484-539) on the same
    host-only function behind the clock interface: the default OPTIMIZATION_GRADIENT (conjugate
    gradient over two-point derivatives, interval 1e-7) and OPTIMIZATION_NEWTON both reach (0, 0)."""
    recs = {r["method"]: r for r in host_records if r["kind"] == "clock2"}
    assert set(recs) == {"gradient", "newton"}, recs
    for r in recs.values():
        assert abs(r["f"] - 2.0) < 1e-7 and abs(r["x"]) < 1e-3 and abs(r["y"]) < 1e-3, r
        assert r["evals"] < 5000, r


# ------------------------------------------------------------------ the reference's own tests

REF_TESTS = ("test_likelihood", "test_likelihood_clock", "test_likelihood_nh")
REF_DIR = "/root/reference/test"


@pytest.mark.parametrize("name", REF_TESTS)
def test_reference_likelihood_test_compiles_and_links_unchanged(name, tmp_path):
    """The drop-in: /root/reference/test/<name>.cpp, read where it lies and never
    copied, compiles and links against the Bio++ mirror (libbpp_phyl_amd over libplk) with no
    extra include, define or source.  Running it needs the GPU (tests/test_gpu_host.py)."""
    src = os.path.join(REF_DIR, name + ".cpp")
    if not os.path.exists(src):
        pytest.skip("reference tree absent")
    run_make("-s", "-C", os.path.join(ROOT, "bpp-phyl_amd"))
    run_make("-s", "-j8", "-C", HOST, "libbpp_phyl_amd.so")
    exe = str(tmp_path / name)
    r = subprocess.run(["g++", "-std=c++17", "-O0", "-w", "-I" + os.path.join(HOST, "include"),
                        "-I" + os.path.join(ROOT, "include"), "-o", exe, src, "-L" + HOST, "-lbpp_phyl_amd",
                        "-L" + os.path.join(ROOT, "bpp-phyl_amd"), "-lplk"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    assert os.path.getsize(exe) > 0
