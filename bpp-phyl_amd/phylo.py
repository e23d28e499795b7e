"""Host-side helpers for the MI355X pruning engine (Python mirror of the Bio++ host layer).

Everything here runs on the host and prepares inputs for libplk (include/plk.h):
trees (Newick -> postorder ids -> unroot), alphabets and leaf codes, substitution
models (generator + eigen-system), discrete Gamma rates, the postorder op list, and
the seeded synthetic workloads of SURVEY.md 8(d).  Reference citations are relative
to /root/reference/src/Bpp/Phyl/.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

# ---------------------------------------------------------------------------
# Alphabets (bpp-seq state integers).  DNA: A C G T = 0..3, ambiguity codes
# M R W S Y K V H D B N = 4..14, gap = -1.  getInitValue(s, state) = 1 if s is in
# the alias set of `state` (Model/AbstractSubstitutionModel.cpp:98-112).
# ---------------------------------------------------------------------------

DNA_CHARS = "ACGTMRWSYKVHDBN"
_DNA_ALIAS = {
    "A": "A", "C": "C", "G": "G", "T": "T", "M": "AC", "R": "AG", "W": "AT", "S": "CG",
    "Y": "CT", "K": "GT", "V": "ACG", "H": "ACT", "D": "AGT", "B": "CGT", "N": "ACGT",
}
_DNA_EXTRA = {"U": 3, "X": 14, "O": 14, "0": 14, "?": 14, "-": -1, ".": -1}

PROTEIN_CHARS = "ARNDCQEGHILKMFPSTWYV"
_PROT_ALIAS = {"B": "ND", "Z": "QE", "J": "IL", "X": PROTEIN_CHARS}
_PROT_EXTRA_ORDER = "BZJX"

NUC = "ACGT"
# NCBI standard genetic code, codon index = 16*n1 + 4*n2 + n3 over ACGT.
_STD_CODE_AA = "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV*Y*YSSSS*CWCLFLF"


@dataclass
class Alphabet:
    name: str
    n_states: int
    chars: Dict[str, int]          # character (or triplet) -> state int
    init_table: np.ndarray         # [n_codes][S] getInitValue table

    @property
    def n_codes(self) -> int:
        return self.init_table.shape[0]

    def encode(self, seq: str) -> np.ndarray:
        """Sequence string -> state ints (gaps -> -1)."""
        if self.name == "Codon":
            s = seq.upper()
            return np.array([self.chars.get(s[i:i + 3], -1) for i in range(0, len(s), 3)], dtype=np.int32)
        return np.array([self.chars.get(ch, -1) for ch in seq.upper()], dtype=np.int32)


def _dna() -> Alphabet:
    chars = {c: i for i, c in enumerate(DNA_CHARS)}
    chars.update(_DNA_EXTRA)
    tab = np.zeros((len(DNA_CHARS), 4))
    for i, c in enumerate(DNA_CHARS):
        for a in _DNA_ALIAS[c]:
            tab[i, NUC.index(a)] = 1.0
    return Alphabet("DNA", 4, chars, tab)


def _protein() -> Alphabet:
    chars = {c: i for i, c in enumerate(PROTEIN_CHARS)}
    for k, c in enumerate(_PROT_EXTRA_ORDER):
        chars[c] = 20 + k
    chars.update({"-": -1, "?": 23, "*": -1, ".": -1})
    tab = np.zeros((24, 20))
    for i in range(20):
        tab[i, i] = 1.0
    for k, c in enumerate(_PROT_EXTRA_ORDER):
        for a in _PROT_ALIAS[c]:
            tab[20 + k, PROTEIN_CHARS.index(a)] = 1.0
    return Alphabet("Protein", 20, chars, tab)


def _codon() -> Alphabet:
    chars = {}
    for i in range(64):
        chars[NUC[i // 16] + NUC[(i // 4) % 4] + NUC[i % 4]] = i
    chars["NNN"] = 64
    tab = np.zeros((65, 64))
    for i in range(64):
        tab[i, i] = 1.0
    tab[64, :] = 1.0
    return Alphabet("Codon", 64, chars, tab)


DNA = _dna()
PROTEIN = _protein()
CODON = _codon()

# ---------------------------------------------------------------------------
# Trees: TreeTemplateTools::parenthesisToTree (TreeTemplateTools.cpp:335-354):
# nodes are created recursively and ids reset to the postorder index
# (TreeTemplateTools.h:354-361, TreeTemplate::resetNodesId).
# ---------------------------------------------------------------------------


@dataclass
class Node:
    id: int = -1
    name: Optional[str] = None
    dist: Optional[float] = None
    sons: List["Node"] = field(default_factory=list)
    father: Optional["Node"] = None

    def is_leaf(self) -> bool:
        return not self.sons

    def add_son(self, s: "Node") -> None:
        s.father = self
        self.sons.append(s)


def _split_top(content: str) -> List[str]:
    out, depth, cur = [], 0, []
    for ch in content:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    out.append("".join(cur))
    return out


def _parse_node(desc: str) -> Node:
    desc = desc.strip()
    node = Node()
    if desc.startswith("("):
        close = desc.rfind(")")
        inner, tail = desc[1:close], desc[close + 1:]
        for part in _split_top(inner):
            node.add_son(_parse_node(part))
    else:
        tail = desc
    if ":" in tail:
        label, length = tail.split(":", 1)
        node.dist = float(length)
    else:
        label = tail
    label = label.strip()
    if node.sons:
        pass  # internal labels are bootstrap values in Bio++; ignored here
    else:
        node.name = label
    return node


def postorder(root: Node) -> List[Node]:
    out: List[Node] = []
    stack = [(root, False)]
    while stack:
        n, done = stack.pop()
        if done:
            out.append(n)
        else:
            stack.append((n, True))
            for s in reversed(n.sons):
                stack.append((s, False))
    return out


class Tree:
    def __init__(self, root: Node):
        self.root = root

    @staticmethod
    def from_newick(text: str) -> "Tree":
        semi = text.rfind(";")
        if semi < 0:
            raise ValueError("Bad format: no semi-colon found.")
        t = Tree(_parse_node(text[:semi].replace("\n", "").replace(" ", "")))
        for i, n in enumerate(postorder(t.root)):
            n.id = i
        return t

    def nodes(self) -> List[Node]:
        return postorder(self.root)

    def leaves(self) -> List[Node]:
        return [n for n in self.nodes() if n.is_leaf()]

    def leaf_names(self) -> List[str]:
        return [n.name for n in self.leaves()]

    def is_rooted(self) -> bool:
        return len(self.root.sons) == 2

    def unroot(self) -> bool:
        """TreeTemplate::unroot (TreeTemplate.h:244-300)."""
        if not self.is_rooted():
            raise ValueError("Tree::unroot: tree is not rooted")
        son1, son2 = self.root.sons
        if son1.is_leaf() and son2.is_leaf():
            return False
        if son1.is_leaf():
            self.root.sons = [son2, son1]
            son1, son2 = son2, son1
        if son1.dist is not None:
            son2.dist = son1.dist + son2.dist if son2.dist is not None else son1.dist
            son1.dist = None
        self.root.sons = []
        son1.father = None
        son1.add_son(son2)
        self.root = son1
        return True

    def copy(self) -> "Tree":
        def cp(n: Node) -> Node:
            m = Node(n.id, n.name, n.dist)
            for s in n.sons:
                m.add_son(cp(s))
            return m
        return Tree(cp(self.root))


def balanced_tree(n_leaves: int, seed: int = 42, lo: float = 0.01, hi: float = 0.1) -> Tree:
    """Complete balanced rooted binary tree t0..t{N-1}, branch lengths U(lo, hi)."""
    rng = np.random.default_rng(seed)
    level = [Node(name=f"t{i}") for i in range(n_leaves)]
    while len(level) > 1:
        nxt = []
        for i in range(0, len(level) - 1, 2):
            p = Node()
            p.add_son(level[i])
            p.add_son(level[i + 1])
            nxt.append(p)
        if len(level) % 2:
            nxt.append(level[-1])
        level = nxt
    t = Tree(level[0])
    for i, n in enumerate(t.nodes()):
        n.id = i
        if n is not t.root:
            n.dist = float(rng.uniform(lo, hi))
    return t


# ---------------------------------------------------------------------------
# Engine layout: tips [0, n_tips), internal nodes after, ops in postorder.
# Branch lengths are clamped to [1e-6, 1e4] as the reference does
# (Likelihood/AbstractHomogeneousTreeLikelihood.cpp:163-165, 305-337).
# ---------------------------------------------------------------------------

MIN_BRLEN, MAX_BRLEN = 1e-6, 1e4


@dataclass
class EngineTree:
    n_tips: int
    n_internal: int
    root: int                          # engine index of the root
    tip_names: List[str]
    ops: List[Tuple[int, Tuple[int, ...]]]   # (parent, children) postorder
    brlen: np.ndarray                  # [n_nodes] branch length above each node (root: 0)
    engine_of_id: Dict[int, int]
    brlen_names: List[str]             # BrLen<i> names in reference order (postorder minus root)
    brlen_engine: List[int]            # engine node of BrLen<i>

    @property
    def n_nodes(self) -> int:
        return self.n_tips + self.n_internal

    # tree arrays for the oracle (son lists by engine index)
    def son_arrays(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        sons: List[List[int]] = [[] for _ in range(self.n_nodes)]
        for p, ch in self.ops:
            sons[p].extend(ch)
        start = np.zeros(self.n_nodes + 1, dtype=np.int32)
        for i in range(self.n_nodes):
            start[i + 1] = start[i] + len(sons[i])
        flat = np.array([c for s in sons for c in s], dtype=np.int32)
        leaf_row = np.array([i if i < self.n_tips else -1 for i in range(self.n_nodes)], dtype=np.int32)
        return start, flat, leaf_row


def engine_tree(tree: Tree, unroot: bool = True) -> EngineTree:
    """Mirror of AbstractHomogeneousTreeLikelihood::init_ (:140-166): copy, unroot if
    rooted (checkRooted), nodes_ = postorder minus root.  NH trees keep the root."""
    t = tree.copy()
    if unroot and t.is_rooted():
        t.unroot()
    nodes = t.nodes()
    tips = [n for n in nodes if n.is_leaf()]
    internal = [n for n in nodes if not n.is_leaf()]
    eng: Dict[int, int] = {}
    for i, n in enumerate(tips):
        eng[id(n)] = i
    for i, n in enumerate(internal):
        eng[id(n)] = len(tips) + i
    ops = [(eng[id(n)], tuple(eng[id(s)] for s in n.sons)) for n in internal]
    brlen = np.zeros(len(nodes))
    names, beng = [], []
    for i, n in enumerate(nodes[:-1]):   # nodes_.pop_back(): root is last in postorder
        d = MIN_BRLEN if n.dist is None else min(max(n.dist, MIN_BRLEN), MAX_BRLEN)
        brlen[eng[id(n)]] = d
        names.append(f"BrLen{i}")
        beng.append(eng[id(n)])
    return EngineTree(
        n_tips=len(tips), n_internal=len(internal), root=eng[id(t.root)],
        tip_names=[n.name for n in tips], ops=ops, brlen=brlen,
        engine_of_id={n.id: eng[id(n)] for n in nodes}, brlen_names=names, brlen_engine=beng)


def split_ops(ops: Sequence[Tuple[int, Tuple[int, ...]]]) -> List[Tuple[int, Tuple[int, ...], int]]:
    """Split polytomies into <=3-child ops; follow-ups carry PLK_OP_ACCUMULATE."""
    out = []
    for p, ch in ops:
        for k in range(0, len(ch), 3):
            out.append((p, tuple(ch[k:k + 3]), 0 if k == 0 else 1))
    return out


# ---------------------------------------------------------------------------
# Discrete Gamma (mean of category, alpha = beta), exact quantiles via scipy.
# bpp-core uses AS91 (chi2 quantile) + AS32 (incomplete gamma); the oracle carries
# that restatement.  Differences are < 1e-9 relative on the rates.
# ---------------------------------------------------------------------------


def gamma_rates(n: int, alpha: float) -> Tuple[np.ndarray, np.ndarray]:
    if n == 1:
        return np.ones(1), np.ones(1)
    from scipy.special import gammainc, gammaincinv
    bounds = gammaincinv(alpha, np.arange(1, n) / n) / alpha
    cum = np.concatenate([[0.0], gammainc(alpha + 1.0, alpha * bounds), [1.0]])
    rates = np.diff(cum) * n
    return rates, np.full(n, 1.0 / n)


# ---------------------------------------------------------------------------
# Substitution models -> (generator Q, frequencies pi, eigen-system V, Vinv, lambda)
# ---------------------------------------------------------------------------


@dataclass
class Model:
    name: str
    S: int
    Q: np.ndarray
    pi: np.ndarray
    V: np.ndarray
    Vinv: np.ndarray
    lam: np.ndarray

    def pij(self, t: float) -> np.ndarray:
        """getPij_t: V diag(exp(lambda t)) Vinv (Model/AbstractSubstitutionModel.cpp:426-438)."""
        if t == 0:
            return np.eye(self.S)
        return (self.V * np.exp(self.lam * t)) @ self.Vinv


def reversible_generator(exch: np.ndarray, pi: np.ndarray) -> np.ndarray:
    """hadamardMult(S, pi) + setDiagonal + normalize (Model/AbstractSubstitutionModel.cpp:645-703)."""
    Q = exch * pi[None, :]
    np.fill_diagonal(Q, 0.0)
    np.fill_diagonal(Q, -Q.sum(axis=1))
    scale = -np.dot(np.diag(Q), pi)
    return Q / scale


def reversible_eigen(Q: np.ndarray, pi: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Eigen-system of a reversible generator via the symmetric form D^1/2 Q D^-1/2.
    Null (stop) states are kept out of the decomposition and get unit eigenvectors
    with eigenvalue 0 (Model/AbstractSubstitutionModel.cpp:184-273)."""
    S = Q.shape[0]
    null = np.array([abs(Q[i, i]) < 1e-12 and np.all(np.abs(Q[:, i]) < 1e-12) for i in range(S)])
    live = np.where(~null)[0]
    sq = np.sqrt(pi[live])
    B = sq[:, None] * Q[np.ix_(live, live)] / sq[None, :]
    B = 0.5 * (B + B.T)
    lam_l, U = np.linalg.eigh(B)
    V = np.zeros((S, S))
    Vinv = np.zeros((S, S))
    lam = np.zeros(S)
    n = len(live)
    V[np.ix_(live, np.arange(n))] = U / sq[:, None]
    Vinv[np.ix_(np.arange(n), live)] = U.T * sq[None, :]
    lam[:n] = lam_l
    for k, i in enumerate(np.where(null)[0]):
        V[i, n + k] = 1.0
        Vinv[n + k, i] = 1.0
    # exact zero for the stationary eigenvalue (:358-361)
    lam[np.argmin(np.abs(lam[:n]))] = 0.0
    return V, Vinv, lam


def t92(kappa: float = 3.0, theta: float = 0.5) -> Model:
    """T92 with the reference's closed-form eigen-system (Model/Nucleotide/T92.cpp:81-187)."""
    piA = piT = (1 - theta) / 2
    piC = piG = theta / 2
    r = 2.0 / (1 + 2 * theta * kappa - 2 * theta * theta * kappa)
    Q = np.array([
        [-(1 + theta * kappa) / 2, theta / 2, kappa * theta / 2, (1 - theta) / 2],
        [(1 - theta) / 2, -(1 + (1 - theta) * kappa) / 2, theta / 2, kappa * (1 - theta) / 2],
        [kappa * (1 - theta) / 2, theta / 2, -(1 + (1 - theta) * kappa) / 2, (1 - theta) / 2],
        [(1 - theta) / 2, kappa * theta / 2, theta / 2, -(1 + theta * kappa) / 2]]) * r
    lam = np.array([0.0, -r * (1 + kappa) / 2, -r * (1 + kappa) / 2, -r])
    Vinv = np.array([
        [-(theta - 1) / 2, theta / 2, theta / 2, -(theta - 1) / 2],
        [0.0, -(theta - 1), 0.0, theta - 1],
        [theta, 0.0, -theta, 0.0],
        [-(theta - 1) / 2, -theta / 2, theta / 2, (theta - 1) / 2]])
    V = np.array([
        [1.0, 0.0, 1.0, 1.0],
        [1.0, 1.0, 0.0, -1.0],
        [1.0, 0.0, (theta - 1) / theta, 1.0],
        [1.0, theta / (theta - 1), 0.0, -1.0]])
    return Model("T92", 4, Q, np.array([piA, piC, piG, piT]), V, Vinv, lam)


def gtr(a=1.0, b=1.0, c=1.0, d=1.0, e=1.0, piA=0.25, piC=0.25, piG=0.25, piT=0.25) -> Model:
    """GTR in the Bio++ parameterisation (Model/Nucleotide/GTR.cpp:84-124): A<->G = 1,
    a = C<->T, b = A<->T, c = G<->T, d = A<->C, e = C<->G."""
    theta = piG + piC
    theta1 = piA / (1 - theta)
    theta2 = piG / theta
    pA = theta1 * (1 - theta)
    pC = (1 - theta2) * theta
    pG = theta2 * theta
    pT = (1 - theta1) * (1 - theta)
    p = 2 * (a * pC * pT + b * pA * pT + c * pG * pT + d * pA * pC + e * pC * pG + pA * pG)
    E = np.array([[0, d, 1, b], [d, 0, e, a], [1, e, 0, c], [b, a, c, 0]], dtype=float) / p
    pi = np.array([pA, pC, pG, pT])
    Q = reversible_generator(E, pi)
    V, Vinv, lam = reversible_eigen(Q, pi)
    return Model("GTR", 4, Q, pi, V, Vinv, lam)


def lg08() -> Model:
    from lg08_data import LG08_EXCHANGEABILITY, LG08_FREQUENCIES
    E = np.array(LG08_EXCHANGEABILITY, dtype=float)
    pi = np.array(LG08_FREQUENCIES, dtype=float)
    Q = reversible_generator(E, pi)
    V, Vinv, lam = reversible_eigen(Q, pi)
    return Model("LG08", 20, Q, pi, V, Vinv, lam)


STOP_CODONS = [i for i, a in enumerate(_STD_CODE_AA) if a == "*"]


def yn98(kappa: float = 2.0, omega: float = 0.3, codon_freqs: Optional[np.ndarray] = None) -> Model:
    """YN98 on the 64-codon state space, stop codons as null states
    (Model/Codon/YN98.cpp:51-78 -> AbstractWordSubstitutionModel::fillBasicGenerator :355-390,
    AbstractCodonSubstitutionModel::completeMatrices :174-190): for codons differing at
    one position, Q_ij = (kappa if transition) * (omega if non-synonymous) * pi_j."""
    pi = np.ones(64) if codon_freqs is None else np.array(codon_freqs, dtype=float)
    pi[STOP_CODONS] = 0.0
    pi /= pi.sum()
    Q = np.zeros((64, 64))
    ts = {(0, 2), (2, 0), (1, 3), (3, 1)}
    for i in range(64):
        for j in range(64):
            if i == j or i in STOP_CODONS or j in STOP_CODONS:
                continue
            a = (i // 16, (i // 4) % 4, i % 4)
            b = (j // 16, (j // 4) % 4, j % 4)
            diff = [k for k in range(3) if a[k] != b[k]]
            if len(diff) != 1:
                continue
            k = diff[0]
            q = kappa if (a[k], b[k]) in ts else 1.0
            if _STD_CODE_AA[i] != _STD_CODE_AA[j]:
                q *= omega
            Q[i, j] = q * pi[j]
    np.fill_diagonal(Q, -Q.sum(axis=1))
    Q /= -np.dot(np.diag(Q), pi)
    V, Vinv, lam = reversible_eigen(Q, pi)
    return Model("YN98", 64, Q, pi, V, Vinv, lam)


# ---------------------------------------------------------------------------
# Seeded simulation (NonHomogeneousSequenceSimulator::simulate semantics,
# Simulation/NonHomogeneousSequenceSimulator.cpp:306-353): root ~ pi, class
# uniform per site, evolve along branches with cumulative P rows.
# ---------------------------------------------------------------------------


def simulate(et: EngineTree, models: Sequence[Model], model_of_node: Optional[np.ndarray], rates: np.ndarray,
             n_sites: int, seed: int = 42, root_freqs: Optional[np.ndarray] = None) -> np.ndarray:
    """Returns states [n_tips][n_sites] (int8/int16) simulated on the engine tree."""
    rng = np.random.default_rng(seed)
    S = models[0].S
    C = len(rates)
    pi0 = models[0].pi if root_freqs is None else root_freqs
    cls = rng.integers(0, C, size=n_sites)
    state = np.empty((et.n_nodes, n_sites), dtype=np.int16)
    state[et.root] = np.searchsorted(np.cumsum(pi0), rng.random(n_sites), side="right").clip(0, S - 1)
    # preorder over ops (reverse postorder)
    for p, ch in reversed(et.ops):
        for c in ch:
            m = models[0] if model_of_node is None else models[model_of_node[c]]
            cum = np.cumsum(np.stack([m.pij(et.brlen[c] * r) for r in rates]), axis=2)  # [C][S][S]
            u = rng.random(n_sites)
            rows = cum[cls, state[p]]                   # [n_sites][S]
            state[c] = (u[:, None] > rows).sum(axis=1).clip(0, S - 1)
    return state[: et.n_tips].copy()


def states_to_codes(states: np.ndarray) -> np.ndarray:
    if states.min() < 0:
        raise ValueError("gap / unknown state: map gaps to the unknown code first (BadIntException)")
    return states.astype(np.uint8)
