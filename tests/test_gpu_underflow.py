"""plk_root_underflow (include/plk.h): the root reductions of an unscaled handle flag a site
likelihood below 2^-255.  A clear flag proves that a rescaling handle would have returned
bitwise the same lnL (no node's joint maximum can then have fallen below the 2^-256
rescaling threshold), which is what lets the Bio++ mirror evaluate unscaled first and fall
back to a rescaling engine only when the flag is set (tests/cpp/test_likelihood_gpu.cpp:
shortBranchScalingCase, unscaledFirstCase).  Checked on every kernel that reduces a root:
jit_tree4, jit_treeM, treeM (64 states), and root_kernel after a levelwise traversal."""
import numpy as np
import pytest

import phylo
import plk
import workload

pytestmark = pytest.mark.gpu


def _engine(wl, n, states, flags):
    et = wl.et
    base = plk.PLK_FLAG_NONNEG_GUARD if wl.guard else 0
    eng = plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, len(wl.models), base | flags)
    eng.set_code_table(wl.alphabet.init_table)
    for i in range(et.n_tips):
        eng.set_tip_codes(i, phylo.states_to_codes(states[i]))
    eng.set_category_rates(wl.rates, wl.probs)
    eng.set_root_frequencies(wl.root_freqs)
    for k, m in enumerate(wl.models):
        eng.set_eigen(k, m.V, m.Vinv, m.lam)
    return eng


def _evaluate(eng, wl, scale):
    et = wl.et
    br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
    mi = None if wl.model_of_node is None else wl.model_of_node[br].astype(np.int32)
    return eng.evaluate(br, et.brlen[br] * scale, phylo.split_ops(et.ops), et.root, mi)


@pytest.mark.parametrize("config,flags,path", [
    ("gtr_g4_dna_1M_64", plk.PLK_FLAG_LNL_ONLY, "jit_tree4"),
    ("gtr_g4_dna_1M_64", plk.PLK_FLAG_LEVELWISE, "levelwise"),
    ("lg08_g4_protein_200k_256", plk.PLK_FLAG_LNL_ONLY, "jit_treeM"),
    ("yn98_codon_50k_128", plk.PLK_FLAG_LNL_ONLY, "treeM"),
    ("gtr_g4_dna_1M_64", 0, "jit_tree4"),
    ("gtr_g4_dna_1M_64", plk.PLK_FLAG_SUBTREE_PATTERNS, "subtree_patterns"),
    ("lg08_g4_protein_200k_256", plk.PLK_FLAG_SUBTREE_PATTERNS, "subtree_patterns"),
    ("nh_gtr_g4_dna_2M_512", plk.PLK_FLAG_LNL_ONLY, "jit_tree4"),
    ("nh_gtr_g4_dna_2M_512", plk.PLK_FLAG_LEVELWISE, "levelwise")])
def test_clear_flag_means_scaled_result_bitwise(config, flags, path):
    """Short branches: no site likelihood near 2^-255 -> flag 0, and the rescaling handle's
    lnL and block sums equal the unscaled handle's bitwise -- on full traversals and on an
    incremental one (one branch moved, its ancestors' ops only, as the mirror's optimiser
    evaluates); with the per-subtree compression the mirror's usePatterns default runs, and
    the NH workload's root rule (no guards, clamp).  Incremental where the mirror uses it
    (materialising and levelwise handles)."""
    n = 3000
    wl = workload.make_workload(config, n_patterns=n)
    if wl.S > 4 or wl.et.n_tips > 64:
        # (128 / 256 tips of proteins or codons: a twentieth of the lengths keeps every site
        # likelihood far above 2^-255; the alignment is simulated on the shortened tree)
        wl.et.brlen = wl.et.brlen * 0.05
    states = wl.simulate(0, n)
    un = _engine(wl, n, states, flags)
    sc = _engine(wl, n, states, flags | plk.PLK_FLAG_SCALING)
    l0, b0 = _evaluate(un, wl, 1.0)
    l1, b1 = _evaluate(sc, wl, 1.0)
    assert un.kernel_path() == path
    assert not un.root_underflow()
    assert l0 == l1 and np.array_equal(b0, b1)
    with pytest.raises(plk.PlkError):
        sc.root_underflow()  # a scaled handle's reduction carries no flag
    if flags & (plk.PLK_FLAG_LNL_ONLY | plk.PLK_FLAG_SUBTREE_PATTERNS):
        return   # lnL-only (partials in registers) and compressed handles take full op lists only
        # (the mirror evaluates incrementally on neither: Likelihood.cpp evaluateTree)
    # incremental: one branch 1.5x longer, only its ancestors recomputed
    et = wl.et
    ops = [(p, tuple(ch)) for p, ch in et.ops]
    parent = {c: p for p, ch in ops for c in ch}
    b = ops[len(ops) // 3][1][0]
    path, v = set(), b
    while v in parent:
        v = parent[v]
        path.add(v)
    inc = phylo.split_ops([op for op in ops if op[0] in path])
    br = np.array([b], dtype=np.int32)
    mi = None if wl.model_of_node is None else wl.model_of_node[br].astype(np.int32)
    li0, bi0 = un.evaluate(br, et.brlen[br] * 1.5, inc, et.root, mi)
    li1, bi1 = sc.evaluate(br, et.brlen[br] * 1.5, inc, et.root, mi)
    assert not un.root_underflow()
    assert li0 == li1 and np.array_equal(bi0, bi1) and li0 != l0


@pytest.mark.parametrize("config,flags", [
    ("nh_gtr_g4_dna_2M_512", plk.PLK_FLAG_LNL_ONLY),
    ("lg08_g4_protein_200k_256", plk.PLK_FLAG_LNL_ONLY),
    ("nh_gtr_g4_dna_2M_512", plk.PLK_FLAG_LEVELWISE)])
def test_long_branches_raise_the_flag(config, flags):
    """Long branches on a 256 / 512-taxon tree: site likelihoods near prod(pi), far below
    2^-255 -- the unscaled handle flags them (its lnL may then differ from the rescaled one,
    which stays finite)."""
    n = 2000
    wl = workload.make_workload(config, n_patterns=n)
    states = wl.simulate(0, n)
    un = _engine(wl, n, states, flags)
    _evaluate(un, wl, 50.0)
    assert un.root_underflow()
    sc = _engine(wl, n, states, flags | plk.PLK_FLAG_SCALING)
    l_sc, _ = _evaluate(sc, wl, 50.0)
    assert np.isfinite(l_sc)


@pytest.mark.parametrize("flags", [plk.PLK_FLAG_LNL_ONLY, plk.PLK_FLAG_LEVELWISE])
def test_flag_follows_each_evaluation(flags):
    """64 taxa: branches shrunk to 1e-6 of the simulation's make every mismatch cost ~ln(1e-6),
    and sites with a dozen of them fall below 2^-255 (flag set); the next evaluation at the
    simulation's lengths clears it."""
    n = 3000
    wl = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=n)
    states = wl.simulate(0, n)
    un = _engine(wl, n, states, flags)
    _evaluate(un, wl, 1e-6)
    assert un.root_underflow()
    _evaluate(un, wl, 1.0)
    assert not un.root_underflow()
    _evaluate(un, wl, 1e-6)
    assert un.root_underflow()


def test_multi_device_flag_is_the_or_of_the_shards():
    n = 3 * 4096 + 5
    wl = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=n)
    states = wl.simulate(0, n)
    et = wl.et
    eng = plk.Engine([0, 0, 0], wl.S, wl.C, n, et.n_tips, et.n_internal, len(wl.models),
                     plk.PLK_FLAG_LNL_ONLY | plk.PLK_FLAG_NONNEG_GUARD)
    eng.set_code_table(wl.alphabet.init_table)
    for i in range(et.n_tips):
        eng.set_tip_codes(i, phylo.states_to_codes(states[i]))
    eng.set_category_rates(wl.rates, wl.probs)
    eng.set_root_frequencies(wl.root_freqs)
    for k, m in enumerate(wl.models):
        eng.set_eigen(k, m.V, m.Vinv, m.lam)
    _evaluate(eng, wl, 1.0)
    assert not eng.root_underflow()
    _evaluate(eng, wl, 1e-6)
    assert eng.root_underflow()


@pytest.mark.parametrize("flags", [plk.PLK_FLAG_LNL_ONLY, plk.PLK_FLAG_LEVELWISE])
def test_comm_flag_travels_in_the_exchange_record(flags, monkeypatch):
    """Under a communicator the flag is global: wave_sums_to_blocks writes it into this rank's
    exchange record (plk_exchange.hpp: block sums, zero padding, flag) and root_finish ORs every
    rank's.  One rank with PLK_TEST_COMM_PAD=5 (five padding doubles, as a rank with fewer blocks
    than the widest carries): lnL, block sums and the flag equal the plain handle's, evaluation
    after evaluation, flag set and cleared."""
    n = 3 * 4096 + 5
    wl = workload.make_workload("gtr_g4_dna_1M_64", n_patterns=n)
    states = wl.simulate(0, n)
    ref = _engine(wl, n, states, flags)
    monkeypatch.setenv("PLK_TEST_COMM_PAD", "5")
    eng = _engine(wl, n, states, flags)
    eng.comm_init(1, 0, plk.comm_get_id())
    for scale, want in ((1.0, False), (1e-6, True), (1.0, False), (1e-6, True)):
        l0, b0 = _evaluate(ref, wl, scale)
        l1, b1 = _evaluate(eng, wl, scale)
        assert l0 == l1 and np.array_equal(b0, b1)
        assert ref.root_underflow() == want and eng.root_underflow() == want
