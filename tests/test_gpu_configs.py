"""GPU parity of exactly what the bench lines time: every BASELINE.json GPU config
 through workload.Evaluator with the bench's default flags
(PLK_FLAG_LNL_ONLY: the fused traversal with cherry tables), at the config's own tree,
model and rate classes, against the CPU oracle.

  - pruning on the engine's own P(t) (plk_get_pmatrix): per-pattern relative 1e-12;
  - end to end (the oracle's independent Jacobi P(t), oracle.reversible_pij on the
    model's generator): total lnL relative 1e-10 (north_star), per pattern 1e-9;
  - the kernel that served the traversal is the one the bench line names;
  - at full size: the oracle on every pattern (per pattern and the total), bitwise
    determinism, and bitwise invariance of the block sums under a 2-way shard.

Config 4 (YN98, 64 stored states with TAA/TAG/TGA as null states, C = 1) runs the
treeM<64> traversal, the cherry contribution tables and pmat64w_kernel, i.e. the path
that profiles/*cfg4* time; reference chain Model/Codon/YN98.cpp:51-78 ->
Model/Codon/AbstractCodonSubstitutionModel.cpp:174-190.
"""
import numpy as np
import pytest

import oracle
import phylo
import plk
import workload

pytestmark = pytest.mark.gpu

REL = 1e-12

# config -> (patterns for the oracle comparison, kernel path of the bench's mode)
CASES = {
    "gtr_g4_dna_1M_64": (20000, "jit_tree4"),
    "lg08_g4_protein_200k_256": (1500, "jit_treeM"),
    "yn98_codon_50k_128": (3000, "treeM"),
    "nh_gtr_g4_dna_2M_512": (4000, "jit_tree4"),
}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if plk.device_count() < 1:
        pytest.fail("no GPU visible: gpu-marked tests must run on the MI355X box")


def test_library_built_from_these_sources():
    """On the box: the libplk.so these tests load was built from the shipped sources."""
    assert plk.build_id() == plk.source_hash()


def _model_of(wl, n):
    return wl.models[0] if wl.model_of_node is None else wl.models[wl.model_of_node[n]]


def _oracle(wl, states, pmats=None, brlen=None, use_patterns=False):
    et = wl.et
    bl = et.brlen if brlen is None else brlen
    if pmats is None:
        pmats = np.zeros((et.n_nodes, wl.C, wl.S, wl.S))
        for n in range(et.n_nodes):
            if n != et.root:
                m = _model_of(wl, n)
                for c in range(wl.C):
                    pmats[n, c] = oracle.reversible_pij(m.Q, m.pi, bl[n] * wl.rates[c])
    ss, sons, lr = et.son_arrays()
    lnl, site, _, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, wl.alphabet.init_table, pmats, wl.probs,
                                         wl.root_freqs, use_patterns=use_patterns, scaling=wl.scaling, want_sites=True)
    return lnl, site


def _engine_pmats(eng, et):
    pm = np.zeros((et.n_nodes, eng.C, eng.S, eng.S))
    for n in range(et.n_nodes):
        if n != et.root:
            pm[n] = eng.get_pmatrix(n)
    return pm


@pytest.mark.parametrize("config", sorted(CASES))
def test_bench_mode_vs_oracle(config):
    n, path = CASES[config]
    wl = workload.make_workload(config, n_patterns=n)
    states = wl.simulate(0, n).astype(np.int32)
    if wl.alphabet.name == "Codon":
        assert not np.isin(states, phylo.STOP_CODONS).any()      # stop codons have pi = 0
    ev = workload.Evaluator(wl, 0, 0, n, states=states, extra_flags=plk.PLK_FLAG_LNL_ONLY)
    for scale in (1.0, 1.15):    # a second evaluation at other branch lengths (new P(t), same program)
        bl = wl.et.brlen * scale
        lnl, _, blocks = ev.step(bl)
        assert ev.eng.kernel_path() == path
        lnl_r, sites, _ = ev.eng.root_loglik(wl.et.root, want_sites=True)
        assert lnl_r == lnl and np.all(np.isfinite(sites))
        # pruning on identical P(t)
        lo, so = _oracle(wl, states, pmats=_engine_pmats(ev.eng, wl.et))
        assert abs(lnl - lo) <= REL * abs(lo), (lnl, lo)
        assert np.allclose(sites, so, rtol=REL, atol=0)
        # end to end: the oracle's own P(t) from the model's generator
        lo2, so2 = _oracle(wl, states, brlen=bl)
        assert abs(lnl - lo2) <= 1e-10 * abs(lo2), (lnl, lo2)
        assert np.allclose(sites, so2, rtol=1e-9, atol=0)


# the oracle over every pattern of the full-size workload (the reference's per-subtree
# compression keeps it at a few seconds per config on the box's host core)
FULL = {
    "gtr_g4_dna_1M_64": None,
    "lg08_g4_protein_200k_256": None,
    "yn98_codon_50k_128": None,
    "nh_gtr_g4_dna_2M_512": None,
}


@pytest.mark.slow
@pytest.mark.parametrize("config", sorted(FULL))
def test_bench_mode_full_size(config):
    """The bench's workload at its full per-GPU size in the bench's mode: finite and
    deterministic, the oracle on every pattern (1e-12 per pattern and on the total, the
    ragged last super-block and block included), and block sums bitwise invariant under a
    2-way shard at a block boundary (the multi-GPU exchange's premise)."""
    wl = workload.make_workload(config)
    P = wl.n_patterns
    states = wl.simulate(0, P)
    ev = workload.Evaluator(wl, 0, 0, P, states=states, extra_flags=plk.PLK_FLAG_LNL_ONLY)
    lnl, _, blocks = ev.step()
    lnl2, _, blocks2 = ev.step()
    assert np.isfinite(lnl) and lnl == lnl2 and np.array_equal(blocks, blocks2)
    assert ev.eng.kernel_path() == CASES[config][1]
    _, sites, _ = ev.eng.root_loglik(wl.et.root, want_sites=True)
    n = FULL[config] or P
    edge = min(256, n // 4)
    mid = np.random.default_rng(11).choice(np.arange(edge, P - edge), size=n - 2 * edge, replace=False)
    idx = np.sort(np.concatenate([np.arange(edge), mid, np.arange(P - edge, P)]))
    lo, so = _oracle(wl, states[:, idx].astype(np.int32), pmats=_engine_pmats(ev.eng, wl.et), use_patterns=True)
    assert np.allclose(sites[idx], so, rtol=REL, atol=0)
    if n == P:  # every pattern: the total too
        assert abs(lnl - lo) <= REL * abs(lo), (lnl, lo)
    del ev
    cut = (P // 4096 // 2) * 4096
    parts = []
    for a, b in ((0, cut), (cut, P)):
        e = workload.Evaluator(wl, 0, a, b, states=states[:, a:b], extra_flags=plk.PLK_FLAG_LNL_ONLY)
        parts.append(e.step()[2])
        del e
    assert np.array_equal(np.concatenate(parts), blocks)
    s = 0.0
    for v in blocks:
        s += v
    assert s == lnl
