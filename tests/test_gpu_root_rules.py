"""The root reduction's two rules on the MI355X, through every root
reduction libplk has: the fused roots of plk_jit_tree4, tree4, plk_jit_treeM and treeM
(20 and 64 states), and root_kernel after the levelwise and per-subtree-compression
traversals.

  - PLK_FLAG_NONNEG_GUARD set: RHomogeneousTreeLikelihood's rule, terms <= 0 dropped per
    state and per class (L/RHomogeneousTreeLikelihood.cpp:192-216);
  - clear: RNonHomogeneousTreeLikelihood's rule, every term added and the site sum clamped
    l < 0 -> 0 before the log (L/RNonHomogeneousTreeLikelihood.cpp:198-221, clamp :206).

Inputs (tests/negroot.py): transition matrices with a negative shift of one row on the
root's first son and on tip 0, uploaded with plk_set_pmatrix, so that root terms are
negative -- "mixed" (both rules finite and different) and "clamp" (NH site sums < 0, which
the clamp turns into log(0) = -inf instead of NaN).  The oracle runs the rule the flag
names (orc_tree_loglik_rule) on the same matrices.  Per test: the numpy census saw <= 0
terms, GPU == oracle per site at 1e-12 (-inf at the same sites, no NaN) and on the total,
and the two rules give different lnL on the GPU -- the branch fired.  With scaling, one
code's vector is 1e-80, so the joint rescale fires too (negative values included).
"""
import numpy as np
import pytest

import negroot
import phylo
import plk
from conftest import set_tune

pytestmark = pytest.mark.gpu
REL = 1e-12

# path -> (S, C, n_taxa, traversal flags, PLK_TUNE keys)
PATHS = {
    "jit_tree4": (4, 4, 16, plk.PLK_FLAG_LNL_ONLY, {}),              # unscaled: one class per workgroup, quads
    "jit_tree4_noquad": (4, 4, 16, plk.PLK_FLAG_LNL_ONLY, {"JIT_QUAD_KB": "0"}),   # every class in the wave
    "tree4": (4, 4, 16, plk.PLK_FLAG_LNL_ONLY, {"JIT": "0"}),
    "levelwise": (4, 3, 16, plk.PLK_FLAG_LEVELWISE, {}),
    "subtree_patterns": (4, 2, 16, plk.PLK_FLAG_SUBTREE_PATTERNS, {}),
    "jit_treeM": (20, 2, 16, plk.PLK_FLAG_LNL_ONLY, {}),
    "treeM": (20, 2, 16, plk.PLK_FLAG_LNL_ONLY, {"JITM": "0"}),
    "treeM64": (64, 1, 8, plk.PLK_FLAG_LNL_ONLY, {}),
    "levelwise20": (20, 2, 16, plk.PLK_FLAG_LEVELWISE, {}),
}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if plk.device_count() < 1:
        pytest.fail("no GPU visible: gpu-marked tests must run on the MI355X box")


def _engine(et, S, C, n, init, states, rates, probs, pi, pm, flags):
    eng = plk.Engine(0, S, C, n, et.n_tips, et.n_internal, 1, flags)
    eng.set_code_table(init)
    for i in range(et.n_tips):
        eng.set_tip_codes(i, states[i].astype(np.uint8))
    eng.set_category_rates(rates, probs)
    eng.set_root_frequencies(pi)
    for b in range(et.n_nodes):
        if b != et.root:
            eng.set_pmatrix(b, pm[b])
    return eng


@pytest.mark.parametrize("kind", ["mixed", "clamp"])
@pytest.mark.parametrize("scaling", [False, True])
@pytest.mark.parametrize("path", sorted(PATHS))
def test_root_rules_vs_oracle(path, scaling, kind, monkeypatch):
    S, C, n_taxa, tflags, tune = PATHS[path]
    for k, v in tune.items():
        set_tune(monkeypatch, k, v)
    n = 500
    et, m, init, states, rates, probs, pi, pm = negroot.problem(S, C, n_taxa, n, seed=100 + S + C + n_taxa,
                                                                 tiny=scaling)
    delta, pm2, census = negroot.choose(et, states, init, pm, pi, probs, kind)
    assert census["neg_terms"] > 0                       # the root saw terms <= 0
    expect_path = {"levelwise20": "levelwise", "treeM64": "treeM", "jit_tree4_noquad": "jit_tree4"}.get(path, path)
    got = {}
    for guard in (True, False):
        flags = tflags | (plk.PLK_FLAG_NONNEG_GUARD if guard else 0) | (plk.PLK_FLAG_SCALING if scaling else 0)
        eng = _engine(et, S, C, n, init, states, rates, probs, pi, pm2, flags)
        eng.update_partials(phylo.split_ops(et.ops))
        lnl, site, _ = eng.root_loglik(et.root, want_sites=True, want_blocks=True)
        assert eng.kernel_path() == expect_path
        if path == "jit_tree4" and not scaling:   # quads ran (three table nodes each; 8 cherries here)
            assert eng.traversal_work()["table_nodes"] > et.n_tips // 2
        eng.close()
        lo, so = negroot.oracle_sites(et, states, init, pm2, probs, pi, scaling, nh_root=not guard)
        negroot.same_sites(site, so, REL)
        if np.isfinite(lo):
            assert abs(lnl - lo) <= REL * abs(lo), (lnl, lo)
        else:
            assert lnl == lo
        if scaling:
            assert np.nanmin(np.where(np.isfinite(so), so, np.nan)) < -256 * np.log(2)   # rescaled
        got[guard] = (lnl, site)
    (lh, sh), (ln, sn) = got[True], got[False]
    fin = np.isfinite(sn)
    assert np.any(sh[fin] != sn[fin])                    # the per-term guards fired
    if kind == "clamp":
        assert ln == -np.inf and np.any(np.isneginf(sn) & np.isfinite(sh))   # the clamp fired
    else:
        assert np.isfinite(ln) and ln < lh
