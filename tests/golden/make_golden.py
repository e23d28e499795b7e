"""Generate the committed golden fixtures under tests/golden/.

Three kinds of vectors:
  reference.json  -- known answers quoted verbatim from the reference's own tests
                     (test/test_likelihood.cpp:108, test/test_likelihood_clock.cpp:115)
                     plus the inputs those tests use (trees, alignments, model params).
  pmatrix.npz     -- P(t) = expm(Q t) via scipy.linalg.expm (Pade, independent of every
                     eigen-decomposition in this repo) for T92, GTR, LG08 and YN98
                     generators built from the reference's parameterisations.  The YN98
                     generator is restated here from the reference chain on its own
                     (yn98_Q below), not taken from phylo.yn98, so the fixture also pins
                     the product's codon generator.
  pruning.npz     -- per-site log-likelihoods of small seeded trees/alignments computed
                     here by a straightforward numpy pruning (per-site, no pattern
                     compression) on the expm matrices above, for T92, GTR and LG08 with
                     Gamma rates, including ambiguity codes.

Run from the repo root:  python tests/golden/make_golden.py
(numpy + scipy only; nothing here touches /root/reference at run time -- the LG08
numbers come from bpp-phyl_amd/lg08_data.py, the published matrix).
"""
import json
import os
import sys

import numpy as np
from scipy.linalg import expm

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "bpp-phyl_amd"))
import phylo  # noqa: E402  (host helpers: Newick, alphabets, generators)

REFERENCE = {
    "test_likelihood": {
        "source": "test/test_likelihood.cpp:91-108",
        "newick": "((A:0.01, B:0.02):0.03,C:0.01,D:0.1);",
        "sequences": {"A": "AAATGGCTGTGCACGTC", "B": "GACTGGATCTGCACGTC",
                      "C": "CTCTGGATGTGCACGTG", "D": "AAATGGCGGTGCGCCTA"},
        "model": {"name": "T92", "kappa": 3.0, "theta": 0.5},
        "rates": {"name": "Gamma", "n": 4, "alpha": 1.0},
        "unroot": True,
        "initial_minus_lnl": 85.030942031997312824,
        "final_minus_lnl": 65.72293577214308868406,
        "tolerance_reference": 1e-3,
    },
    "test_likelihood_clock": {
        "source": "test/test_likelihood_clock.cpp:99-115",
        "newick": "(((A:0.01, B:0.01):0.02,C:0.03):0.01,D:0.04);",
        "sequences": {"A": "AAATGGCTGTGCACGTC", "B": "AACTGGATCTGCATGTC",
                      "C": "ATCTGGACGTGCACGTG", "D": "CAACGGGAGTGCGCCTA"},
        "model": {"name": "T92", "kappa": 3.0, "theta": 0.5},
        "rates": {"name": "Constant"},
        "unroot": False,
        "initial_minus_lnl": 94.3957,
        "final_minus_lnl": 71.2657,
        "tolerance_reference": 1e-3,
    },
    "example1": {
        "source": "test/example1.ph + test/example1.mp.dnd (config 1 of BASELINE.json; gaps mapped to N)",
        "newick": "(((s05:0.10000,s04:0.00000):0.30000,s03:0.00000):0.26667,s02:0.06667,s01:0.16667);",
        "sequences": {"s01": "ATGCGTCTTA", "s02": "ACGCNTCTTA", "s03": "AAGCNTCCGA",
                      "s04": "TAGGNTCCGT", "s05": "TAGGNTCCCT"},
        "model": {"name": "T92", "kappa": 3.0, "theta": 0.5},
        "rates": {"name": "Gamma", "n": 4, "alpha": 1.0},
        "unroot": True,
        "initial_minus_lnl": None,   # no reference golden: restatement-derived
    },
}


def t92_Q(kappa, theta):
    return phylo.t92(kappa, theta).Q


# Standard genetic code in the reference's codon numbering 16*n1 + 4*n2 + n3 over ACGT
# (bpp-seq StandardGeneticCode; '*' = stop: TAA = 48, TAG = 50, TGA = 56).
STD_CODE = "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV*Y*YSSSS*CWCLFLF"


def yn98_Q(kappa, omega):
    """YN98 generator on 64 codon states, restated from the reference chain:
    YN98 (Model/Codon/YN98.cpp:51-78) = CodonDistanceFrequenciesSubstitutionModel over
    K80(kappa) on every codon position; AbstractWordSubstitutionModel::fillBasicGenerator
    (Model/AbstractWordSubstitutionModel.cpp:355-390) puts the nucleotide rate on codons that
    differ at exactly one position; AbstractCodonSubstitutionModel::completeMatrices
    (Model/Codon/AbstractCodonSubstitutionModel.cpp:174-190) zeroes stop rows/columns and
    multiplies by getCodonsMulRate = (omega if non-synonymous,
    AbstractCodonDistanceSubstitutionModel.cpp:80-88) x pi_j
    (AbstractCodonFrequenciesSubstitutionModel.cpp:82-85); F3X4 with equal nucleotide
    frequencies gives pi = 1/61 on sense codons.  Normalised to -sum pi_i Q_ii = 1
    (Model/AbstractSubstitutionModel.cpp:645-690); K80's own scale cancels there."""
    sense = np.array([a != "*" for a in STD_CODE])
    pi = sense / sense.sum()
    Q = np.zeros((64, 64))
    transition = {(0, 2), (2, 0), (1, 3), (3, 1)}   # A<->G, C<->T
    for i in range(64):
        for j in range(64):
            if i == j or not (sense[i] and sense[j]):
                continue
            di = [(i >> s) & 3 for s in (4, 2, 0)]
            dj = [(j >> s) & 3 for s in (4, 2, 0)]
            pos = [k for k in range(3) if di[k] != dj[k]]
            if len(pos) != 1:
                continue
            r = kappa if (di[pos[0]], dj[pos[0]]) in transition else 1.0
            if STD_CODE[i] != STD_CODE[j]:
                r *= omega
            Q[i, j] = r * pi[j]
    Q[np.diag_indices(64)] = -Q.sum(axis=1)
    return Q / -(np.diag(Q) @ pi), pi


def np_pruning(et, states, init_table, Pfun, C, probs, pi):
    """Per-site pruning, straightforward numpy: partial[node] = prod_son P_son @ L_son."""
    n_sites = states.shape[1]
    S = init_table.shape[1]
    L = {}
    for i in range(et.n_tips):
        L[i] = np.broadcast_to(init_table[states[i]][:, None, :], (n_sites, C, S)).copy()
    for p, ch in et.ops:
        acc = np.ones((n_sites, C, S))
        for c in ch:
            P = Pfun(c)  # [C][S][S]
            acc *= np.einsum("cxy,icy->icx", P, L[c])
        L[p] = acc
    root = L[et.root]
    site = np.log(np.einsum("ics,s,c->i", root, pi, probs))
    return site


def main():
    rng = np.random.default_rng(20261015)
    out = {}
    # ---- P(t) fixtures
    gtr_par = dict(a=1.2, b=0.4, c=0.6, d=0.8, e=0.5, piA=0.30, piC=0.20, piG=0.25, piT=0.25)
    mods = {"T92": phylo.t92(3.0, 0.5), "T92_k2_t03": phylo.t92(2.0, 0.3), "GTR": phylo.gtr(**gtr_par),
            "LG08": phylo.lg08()}
    ts = np.array([1e-6, 0.01, 0.1, 0.5, 2.0, 10.0])
    for name, m in mods.items():
        out[f"{name}_Q"] = m.Q
        out[f"{name}_pi"] = m.pi
        out[f"{name}_t"] = ts
        out[f"{name}_P"] = np.stack([expm(m.Q * t) for t in ts])
    # YN98(kappa=2, omega=0.3), config 4's model: expm on the full 64 x 64 generator (stop
    # rows and columns are zero, so their rows of P(t) are unit rows)
    Qy, piy = yn98_Q(2.0, 0.3)
    out["YN98_Q"], out["YN98_pi"], out["YN98_t"] = Qy, piy, ts
    out["YN98_P"] = np.stack([expm(Qy * t) for t in ts])
    # first and second derivatives in t: dP/dt = Q expm(Q t), d2P/dt2 = Q^2 expm(Q t)
    # (getdPij_dt / getd2Pij_dt2, Model/AbstractSubstitutionModel.cpp:499-641)
    for name in ("GTR", "LG08", "YN98"):
        Q = out[f"{name}_Q"]
        out[f"{name}_dP"] = np.stack([Q @ expm(Q * t) for t in ts])
        out[f"{name}_d2P"] = np.stack([Q @ Q @ expm(Q * t) for t in ts])
    np.savez_compressed(os.path.join(HERE, "pmatrix.npz"), **out)

    # ---- pruning fixtures on small seeded problems
    prn = {}
    cases = [("T92", mods["T92"], 6, 40, 4, 1.0, phylo.DNA),
             ("GTR", mods["GTR"], 9, 60, 4, 0.5, phylo.DNA),
             ("GTRamb", mods["GTR"], 7, 50, 4, 0.7, phylo.DNA),
             ("LG08", mods["LG08"], 8, 30, 4, 0.5, phylo.PROTEIN),
             ("YN98", phylo.Model("YN98", 64, Qy, piy, None, None, None), 7, 40, 1, None, phylo.CODON)]
    for name, m, ntaxa, nsites, C, alpha, alph in cases:
        tree = phylo.balanced_tree(ntaxa, seed=int(rng.integers(1 << 30)), lo=0.02, hi=0.3)
        et = phylo.engine_tree(tree)
        rates, probs = phylo.gamma_rates(C, alpha) if C > 1 else (np.ones(1), np.ones(1))
        sim = m if m.V is not None else phylo.Model(name, m.S, m.Q, m.pi, *phylo.reversible_eigen(m.Q, m.pi))
        states = phylo.simulate(et, [sim], None, rates, nsites, seed=int(rng.integers(1 << 30)))
        if name == "GTRamb":   # sprinkle ambiguity codes (4..14)
            mask = rng.random(states.shape) < 0.1
            states[mask] = rng.integers(4, 15, size=mask.sum())
        Pm = {c: np.stack([expm(m.Q * et.brlen[c] * r) for r in rates]) for c in range(et.n_nodes) if c != et.root}
        site = np_pruning(et, states, alph.init_table, lambda c: Pm[c], C, probs, m.pi)
        ss, sons, lr = et.son_arrays()
        prn[f"{name}_son_start"] = ss
        prn[f"{name}_sons"] = sons
        prn[f"{name}_leaf_row"] = lr
        prn[f"{name}_root"] = np.array(et.root)
        prn[f"{name}_brlen"] = et.brlen
        prn[f"{name}_states"] = states.astype(np.int32)
        prn[f"{name}_rates"] = rates
        prn[f"{name}_probs"] = probs
        prn[f"{name}_Q"] = m.Q
        prn[f"{name}_pi"] = m.pi
        prn[f"{name}_site_lnl"] = site
        prn[f"{name}_lnl"] = np.array(site.sum())
    np.savez_compressed(os.path.join(HERE, "pruning.npz"), **prn)
    with open(os.path.join(HERE, "reference.json"), "w") as f:
        json.dump(REFERENCE, f, indent=1)
    print("wrote reference.json, pmatrix.npz, pruning.npz")


if __name__ == "__main__":
    main()
