"""Host cost of plk_update_pmatrices by request size (PLK_DEBUG_HOST breakdown)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bpp-phyl_amd"))
import phylo, plk, workload
wl = workload.make_workload("nh_gtr_g4_dna_2M_512", n_patterns=8192)
ev = workload.Evaluator(wl, 0, 0, 8192, sim_device="cpu")
br_all = ev.branches
for n in (100, 160, 161, 400, 1022):
    br = br_all[:n].copy(); t = wl.et.brlen[br].copy(); mod = ev.model_idx[:n].copy()
    for _ in range(5):
        ev.eng.update_pmatrices(br, t, mod)
    ev.eng.synchronize()
    ev.eng.reset_timing()
    ts = []
    for _ in range(50):
        t0 = time.perf_counter(); ev.eng.update_pmatrices(br, t, mod); t1 = time.perf_counter()
        ev.eng.synchronize(); ts.append((t1 - t0) * 1e6)
    print(f"n={n}: call {np.median(ts):.2f} us (python incl.)", flush=True)
    ev.eng.reset_timing()
