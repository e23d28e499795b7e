import sys, numpy as np
sys.path.insert(0, "bpp-phyl_amd"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import plk, phylo, workload
from test_gpu_multi import _setup
wl = workload.make_workload("lg08_g4_protein_200k_256", n_patterns=8199)
et = wl.et
states = wl.simulate(0, 8199)
base = (plk.PLK_FLAG_SCALING if wl.scaling else 0) | (plk.PLK_FLAG_NONNEG_GUARD if wl.guard else 0) | plk.PLK_FLAG_LNL_ONLY
br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
ops = phylo.split_ops(et.ops)
for lo, hi in ((0, 8199), (0, 4096), (4096, 8199)):
    n = hi - lo
    st = states[:, lo:hi]
    e = _setup(plk.Engine(0, wl.S, wl.C, n, et.n_tips, et.n_internal, len(wl.models), base), wl, st)
    l, b = e.evaluate(br, et.brlen[br], ops, et.root, None)
    print(lo, hi, l, e.kernel_path(), flush=True)
