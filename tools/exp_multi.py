import sys, os, numpy as np
sys.path.insert(0, "bpp-phyl_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import plk, phylo, workload
from test_gpu_multi import _setup
n = 8199
wl = workload.make_workload("lg08_g4_protein_200k_256", n_patterns=n)
et = wl.et
states = wl.simulate(0, n)
base = (plk.PLK_FLAG_SCALING if wl.scaling else 0) | (plk.PLK_FLAG_NONNEG_GUARD if wl.guard else 0) | plk.PLK_FLAG_LNL_ONLY
br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
ops = phylo.split_ops(et.ops)
one = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
multi = _setup(plk.Engine([0, 0], wl.S, wl.C, n, et.n_tips, et.n_internal, 1, base), wl, states)
l1, b1 = one.evaluate(br, et.brlen[br], ops, et.root, None)
lm, bm = multi.evaluate(br, et.brlen[br], ops, et.root, None)
print("one", l1, one.kernel_path(), "multi", lm, multi.kernel_path())
bad = np.where(~np.isfinite(bm) | (b1 != bm))[0]
print("blocks", len(b1), "differ at", bad[:10], b1[bad[:3]] if len(bad) else None, bm[bad[:3]] if len(bad) else None)
r1 = one.root_loglik(et.root, want_sites=True)
rm = multi.root_loglik(et.root, want_sites=True)
d = np.where(r1[1] != rm[1])[0]
print("sites differ", len(d), d[:10], d[-5:] if len(d) else None, rm[1][d[:5]] if len(d) else None)
