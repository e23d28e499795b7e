"""Debug: NH (per-branch models) lnL-only traversals with quads vs without, after a model change."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "bpp-phyl_amd"), os.path.join(os.path.dirname(__file__), "..", "..", "tests")]
import numpy as np
import phylo, plk, workload

et = phylo.engine_tree(phylo.balanced_tree(64, seed=3, lo=0.02, hi=0.1), unroot=False)
rng = np.random.default_rng(1)
models = [phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5)) for _ in range(et.n_nodes)]
mon = np.arange(et.n_nodes, dtype=np.int32)
rates, probs = phylo.gamma_rates(4, 0.8)
pi = np.array([0.3, 0.2, 0.2, 0.3])
n = 3000
wl = workload.Workload("nh", et, models, mon, rates, probs, pi, phylo.DNA, n, False, False, 7)
states = wl.simulate(0, n).astype(np.int32)
br = np.array([v for v in range(et.n_nodes) if v != et.root], dtype=np.int32)
ops = phylo.split_ops(et.ops)

def run(tune, flags):
    os.environ["PLK_TUNE"] = tune
    eng = plk.Engine(0, 4, 4, n, et.n_tips, et.n_internal, len(models), flags)
    eng.set_code_table(phylo.DNA.init_table)
    for i in range(et.n_tips):
        eng.set_tip_codes(i, states[i].astype(np.uint8))
    eng.set_category_rates(rates, probs)
    eng.set_root_frequencies(pi)
    for k, m in enumerate(models):
        eng.set_eigen(k, m.V, m.Vinv, m.lam)
    out = []
    l0, _ = eng.evaluate(br, et.brlen[br], ops, et.root, mon[br])
    out.append(l0)
    # a model change on one tip branch and one internal branch: re-upload eigen, P(t) of that branch only, full ops
    for b in (5, et.n_tips + 7):
        m2 = phylo.gtr(*rng.uniform(0.3, 2.0, 5), *rng.dirichlet(np.ones(4) * 5)) if False else models[(b * 7) % len(models)]
        eng.set_eigen(int(mon[b]), m2.V, m2.Vinv, m2.lam)
        l1, _ = eng.evaluate(np.array([b], dtype=np.int32), et.brlen[[b]], ops, et.root, mon[[b]])
        out.append(l1)
    eng.set_root_frequencies(np.array([0.25, 0.25, 0.2, 0.3]))
    l2, _ = eng.evaluate(np.zeros(0, dtype=np.int32), np.zeros(0), ops, et.root, np.zeros(0, dtype=np.int32))
    out.append(l2)
    print(tune or "default", hex(flags), eng.kernel_path(), [repr(x) for x in out], flush=True)
    eng.close()
    return out

LO = plk.PLK_FLAG_LNL_ONLY
a = run("", LO)
b = run("JIT_QUAD_KB=0", LO)
c = run("", LO | plk.PLK_FLAG_SCALING)
d = run("JIT=0", LO)
print("quad==noquad", [x == y for x, y in zip(a, b)], "noquad==interp", [x == y for x, y in zip(b, d)])
