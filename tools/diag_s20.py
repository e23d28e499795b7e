import sys, os
# Diagnostic: S=20 per-site error of each engine mode vs the oracle, with independent and with identical P(t).
sys.path.insert(0, "tests"); sys.path.insert(0, "bpp-phyl_amd"); sys.path.insert(0, "oracle")
import numpy as np
import test_gpu_parity as T
import phylo, workload, plk
for mode in ("levelwise", "materialize", "lnl_only"):
  for amb in (True, False):
    C, n_patterns = 4, 700
    tree = phylo.balanced_tree(64, seed=19, lo=0.05, hi=0.4)
    et = phylo.engine_tree(tree)
    m = phylo.lg08()
    rates, probs = phylo.gamma_rates(C, 0.7)
    wl = workload.Workload("m", et, [m], None, rates, probs, m.pi, phylo.PROTEIN, n_patterns, False, True, 6)
    states = wl.simulate(0, n_patterns).astype(np.int32)
    if amb:
        rng = np.random.default_rng(n_patterns)
        mask = rng.random(states.shape) < 0.05
        states[mask] = rng.integers(20, phylo.PROTEIN.n_codes, size=mask.sum())
    flags = plk.PLK_FLAG_NONNEG_GUARD | T.MODES[mode]
    eng = T.engine_for(et, 20, C, n_patterns, states, phylo.PROTEIN.init_table, rates, probs, m.pi, [m], flags=flags)
    lnl, site, _ = T.run_engine(eng, et)
    lo, so = T.oracle_for(et, states, phylo.PROTEIN.init_table, rates, probs, m.pi, [m])
    l2, s2 = T.oracle_for(et, states, phylo.PROTEIN.init_table, rates, probs, m.pi, [m], pmats=T.engine_pmats(eng, et))
    r2 = np.abs(site - s2) / np.abs(s2)
    print(mode, "amb", amb, "same-P: lnl rel", abs(lnl - l2) / abs(l2), "max site rel", r2.max(), flush=True)
    r = np.abs(site - so) / np.abs(so)
    i = int(np.argmax(r))
    print(mode, "amb", amb, "lnl rel", abs(lnl - lo) / abs(lo), "max site rel", r.max(), "at", i, site[i], so[i], "n>1e-12", int((r > 1e-12).sum()), flush=True)
