"""Repeat test_multi_device_handle_bitwise[lg08] with fresh handles and report mismatches
(intermittent -inf seen once on the multi handle)."""
import sys, numpy as np
sys.path.insert(0, "bpp-phyl_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import plk, phylo, workload
from test_gpu_multi import _setup
n = 2 * 4096 + 7
wl = workload.make_workload("lg08_g4_protein_200k_256", n_patterns=n)
et = wl.et
states = wl.simulate(0, n)
base = (plk.PLK_FLAG_SCALING if wl.scaling else 0) | (plk.PLK_FLAG_NONNEG_GUARD if wl.guard else 0) | plk.PLK_FLAG_LNL_ONLY
br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
ops = phylo.split_ops(et.ops)
w = np.random.default_rng(3).integers(1, 5, size=n).astype(np.float64)
bad = 0
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 15):
    one = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    multi = _setup(plk.Engine([0, 0], wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
    one.set_pattern_weights(w); multi.set_pattern_weights(w)
    for scale in (1.0, 0.8):
        t = et.brlen[br] * scale
        l1, b1 = one.evaluate(br, t, ops, et.root, None)
        lm, bm = multi.evaluate(br, t, ops, et.root, None)
        if not (l1 == lm and np.array_equal(b1, bm)):
            bad += 1
            r1 = one.root_loglik(et.root, want_sites=True); rm = multi.root_loglik(et.root, want_sites=True)
            d = np.where(r1[1] != rm[1])[0]
            print("MISMATCH it", it, "scale", scale, l1, lm, "sites", len(d), d[:8], rm[1][d[:4]], flush=True)
    del one, multi
print("done, mismatches:", bad, flush=True)
