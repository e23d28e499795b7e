"""Synthetic workloads of BASELINE.json / SURVEY.md 8(d) and the evaluation step.

A workload is (tree, model(s), Gamma rates, alignment).  Alignments are simulated
with a counter-based generator (splitmix64 of (seed, node, site)), so any pattern
range [start, end) can be generated independently and a site's state does not
depend on how the patterns are sharded across GPUs.  Every simulated column is
treated as one pattern of weight 1, so P is exact.

One evaluation ("step") is what RHomogeneousTreeLikelihood::fireParameterChanged
does (Likelihood/RHomogeneousTreeLikelihood.cpp:255-283): all transition matrices
(K4), the full postorder traversal (K1/K2/K3), the root reduction (K5).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

import phylo
import plk

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniforms(seed: int, stream: int, start: int, end: int) -> np.ndarray:
    idx = np.arange(start, end, dtype=np.uint64)
    with np.errstate(over="ignore"):
        key = idx + np.uint64((seed * 1000003 + stream) & 0xFFFFFFFF) * np.uint64(1 << 32)
    z = _splitmix(_splitmix(key))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


@dataclass
class Workload:
    name: str
    et: phylo.EngineTree
    models: List[phylo.Model]
    model_of_node: Optional[np.ndarray]   # per engine node (NH), None = homogeneous
    rates: np.ndarray
    probs: np.ndarray
    root_freqs: np.ndarray
    alphabet: phylo.Alphabet
    n_patterns: int
    scaling: bool
    guard: bool                            # homogeneous (<= 0 guards) vs NH clamp
    seed: int = 42

    @property
    def S(self) -> int:
        return self.models[0].S

    @property
    def C(self) -> int:
        return len(self.rates)

    def units_per_traversal(self, n_patterns: Optional[int] = None) -> int:
        """Site-pattern x node partial updates of one full traversal (P x I)."""
        return (self.n_patterns if n_patterns is None else n_patterns) * self.et.n_internal

    def algorithmic_bytes_per_pattern(self) -> int:
        """16*C*S*I + N + 8 (fp64 partials written + read once, 1-B leaves, 8-B weight)."""
        S_live = self.S if self.alphabet.name != "Codon" else 61
        return 16 * self.C * S_live * self.et.n_internal + self.et.n_tips + 8

    def algorithmic_flops_per_pattern(self) -> int:
        """2*C*S^2 per internal child, 0 per leaf child (code lookup),
        (k-1)*C*S to combine k children."""
        S_live = self.S if self.alphabet.name != "Codon" else 61
        nt = self.et.n_tips
        f = 0
        for _, ch in self.et.ops:
            f += sum(2 * self.C * S_live * S_live for c in ch if c >= nt) + (len(ch) - 1) * self.C * S_live
        return f

    def simulate(self, start: int, end: int, device=None) -> np.ndarray:
        """States [n_tips][end-start] for sites [start, end).  device: a torch device to run
        the same counter-based generator on (bitwise the same states; config 5's 2M patterns
        x 1023 nodes take minutes in numpy and well under a second on the GPU)."""
        if device is not None:
            return self._simulate_torch(start, end, device)
        et, S = self.et, self.S
        n = end - start
        cls = np.minimum((uniforms(self.seed, 1, start, end) * self.C).astype(np.int64), self.C - 1)
        state = np.empty((et.n_nodes, n), dtype=np.int16)
        cum0 = np.cumsum(self.root_freqs)
        state[et.root] = np.searchsorted(cum0, uniforms(self.seed, 2, start, end), side="right").clip(0, S - 1)
        for p, ch in reversed(et.ops):
            for c in ch:
                m = self.models[0] if self.model_of_node is None else self.models[self.model_of_node[c]]
                cum = np.cumsum(np.stack([m.pij(et.brlen[c] * r) for r in self.rates]), axis=2)
                rows = cum[cls, state[p]]
                u = uniforms(self.seed, 16 + c, start, end)
                state[c] = (u[:, None] > rows).sum(axis=1).clip(0, S - 1)
        return state[: et.n_tips]

    def _simulate_torch(self, start: int, end: int, device) -> np.ndarray:
        """simulate() in torch: uint64 splitmix on int64 tensors (wrapping multiply, logical
        shifts masked), the same cumulative rows and comparisons, so the states are bitwise
        those of the numpy generator (tests/test_host.py checks it)."""
        import torch

        et, S, C = self.et, self.S, self.C
        n = end - start
        dev = torch.device(device)
        idx = torch.arange(start, end, dtype=torch.int64, device=dev)

        def uni(stream):
            key = idx + _signed(((self.seed * 1000003 + stream) & 0xFFFFFFFF) << 32)
            z = _splitmix_t(_splitmix_t(key))
            return _lsr(z, 11).to(torch.float64) * (1.0 / 9007199254740992.0)

        cls = torch.clamp((uni(1) * C).to(torch.int64), max=C - 1)
        state = torch.empty((et.n_nodes, n), dtype=torch.int16, device=dev)
        cum0 = torch.from_numpy(np.cumsum(self.root_freqs)).to(dev)
        state[et.root] = torch.searchsorted(cum0, uni(2), right=True).clamp(0, S - 1)
        for p, ch in reversed(et.ops):
            for c in ch:
                m = self.models[0] if self.model_of_node is None else self.models[self.model_of_node[c]]
                cum = torch.from_numpy(np.cumsum(np.stack([m.pij(et.brlen[c] * r) for r in self.rates]),
                                                 axis=2)).to(dev)
                rows = cum[cls, state[p].long()]
                state[c] = (uni(16 + c)[:, None] > rows).sum(dim=1).clamp(0, S - 1)
        return state[: et.n_tips].cpu().numpy()


def _signed(v: int) -> int:
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= (1 << 63) else v


def _lsr(z, k: int):
    """Logical right shift of int64 tensors holding uint64 bit patterns."""
    return (z >> k) & ((1 << (64 - k)) - 1)


def _splitmix_t(x):
    z = x + _signed(0x9E3779B97F4A7C15)
    z = (z ^ _lsr(z, 30)) * _signed(0xBF58476D1CE4E5B9)
    z = (z ^ _lsr(z, 27)) * _signed(0x94D049BB133111EB)
    return z ^ _lsr(z, 31)


def _gtr_cfg2() -> phylo.Model:
    return phylo.gtr(a=1.2, b=0.4, c=0.6, d=0.8, e=0.5, piA=0.30, piC=0.20, piG=0.25, piT=0.25)


CONFIGS = {
    # config 2: "DNA GTR+G4, 4 states, 1M synthetic site patterns, 64-taxon balanced tree, 1 MI355X"
    "gtr_g4_dna_1M_64": dict(model="GTR", alpha=0.5, C=4, n_taxa=64, n_patterns=1_000_000, scaling=False, cpu_sample=100_000),
    # config 3: "Protein LG+G4, 20 states, 200k patterns, 256 taxa"
    "lg08_g4_protein_200k_256": dict(model="LG08", alpha=0.5, C=4, n_taxa=256, n_patterns=200_000, scaling=True, cpu_sample=8_000),
    # config 4: "Codon YN98, 61 states, 50k patterns, 128 taxa" (64 stored states, 3 null stops)
    "yn98_codon_50k_128": dict(model="YN98", alpha=None, C=1, n_taxa=128, n_patterns=50_000, scaling=False, cpu_sample=2_000),
    # config 5: per-branch GTR, 512 taxa, rooted; 2M patterns = 250k per GPU x 8 (weak-scaled per GPU;
    # bench.py --scaling strong keeps the 2M (global_patterns) fixed and splits it over the ranks)
    "nh_gtr_g4_dna_2M_512": dict(model="NHGTR", alpha=1.0, C=4, n_taxa=512, n_patterns=250_000, scaling=True, cpu_sample=10_000,
                                 global_patterns=2_000_000),
}


def make_workload(name: str, n_patterns: Optional[int] = None, seed: int = 42,
                  n_classes: Optional[int] = None) -> Workload:
    """n_classes: A/B experiments only -- the config's model with another Gamma class count."""
    cfg = dict(CONFIGS[name])
    if n_classes is not None:
        cfg["C"] = n_classes
        if cfg["alpha"] is None:
            cfg["alpha"] = 1.0
    tree = phylo.balanced_tree(cfg["n_taxa"], seed=seed)
    rates, probs = phylo.gamma_rates(cfg["C"], cfg["alpha"]) if cfg["C"] > 1 else (np.ones(1), np.ones(1))
    P = cfg["n_patterns"] if n_patterns is None else n_patterns
    if cfg["model"] == "GTR":
        m = _gtr_cfg2()
        et = phylo.engine_tree(tree, unroot=True)
        return Workload(name, et, [m], None, rates, probs, m.pi, phylo.DNA, P, cfg["scaling"], True, seed)
    if cfg["model"] == "LG08":
        m = phylo.lg08()
        et = phylo.engine_tree(tree, unroot=True)
        return Workload(name, et, [m], None, rates, probs, m.pi, phylo.PROTEIN, P, cfg["scaling"], True, seed)
    if cfg["model"] == "YN98":
        m = phylo.yn98(2.0, 0.3)
        et = phylo.engine_tree(tree, unroot=True)
        return Workload(name, et, [m], None, rates, probs, m.pi, phylo.CODON, P, cfg["scaling"], True, seed)
    if cfg["model"] == "NHGTR":
        et = phylo.engine_tree(tree, unroot=False)
        u = uniforms(seed, 7, 0, et.n_nodes)
        models = []
        for i in range(et.n_nodes):
            theta = 0.3 + 0.4 * u[i]          # GC content theta ~ U(0.3, 0.7) per branch
            models.append(phylo.gtr(a=1.2, b=0.4, c=0.6, d=0.8, e=0.5, piA=(1 - theta) / 2, piC=theta / 2,
                                    piG=theta / 2, piT=(1 - theta) / 2))
        root_freqs = np.array([0.3, 0.2, 0.2, 0.3])  # GC root frequencies (theta = 0.4)
        return Workload(name, et, models, np.arange(et.n_nodes), rates, probs, root_freqs, phylo.DNA, P,
                        cfg["scaling"], False, seed)
    raise KeyError(name)


class Evaluator:
    """One libplk engine holding the patterns [start, end) of a workload."""

    def __init__(self, wl: Workload, device, start: int, end: int, states: Optional[np.ndarray] = None,
                 extra_flags: int = 0, sim_device=None):
        """device: a HIP device, or a list of them (one plk_create_multi handle sharding the
        patterns); sim_device: a torch device for the alignment simulation (bitwise the same
        states as numpy, Workload.simulate)."""
        self.wl = wl
        self.start, self.end = start, end
        et = wl.et
        flags = (plk.PLK_FLAG_SCALING if wl.scaling else 0) | (plk.PLK_FLAG_NONNEG_GUARD if wl.guard else 0) | extra_flags
        self.eng = plk.Engine(device, wl.S, wl.C, end - start, et.n_tips, et.n_internal, len(wl.models), flags)
        self.eng.set_code_table(wl.alphabet.init_table)
        st = wl.simulate(start, end, device=sim_device) if states is None else states
        for i in range(et.n_tips):
            self.eng.set_tip_codes(i, phylo.states_to_codes(st[i]))
        self.eng.set_category_rates(wl.rates, wl.probs)
        self.eng.set_root_frequencies(wl.root_freqs)
        for k, m in enumerate(wl.models):
            self.eng.set_eigen(k, m.V, m.Vinv, m.lam)
        self.branches = np.array([n for n in range(et.n_nodes) if n != et.root], dtype=np.int32)
        self.model_idx = None if wl.model_of_node is None else wl.model_of_node[self.branches].astype(np.int32)
        self.ops = phylo.split_ops(et.ops)
        self.n_blocks = (end - start + plk.BLOCK - 1) // plk.BLOCK
        self.t_tree = et.brlen[self.branches]  # the tree's own branch lengths, per branch of the request

    def step(self, brlen: Optional[np.ndarray] = None):
        """One evaluation: P(t) of every branch (the tree's lengths, or `brlen` per node),
        the traversal and the root reduction (plk_evaluate)."""
        et = self.wl.et
        t = self.t_tree if brlen is None else brlen[self.branches]
        lnl, blocks = self.eng.evaluate(self.branches, t, self.ops, et.root, self.model_idx)
        return lnl, None, blocks
