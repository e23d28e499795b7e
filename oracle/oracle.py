"""ctypes wrapper of the CPU oracle (oracle/oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product path.
"""
from __future__ import annotations

import ctypes as ct
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load() -> ct.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ct.CDLL(LIB_PATH)
    P = ct.POINTER
    dp, ip = P(ct.c_double), P(ct.c_int32)
    lib.orc_gamma_rates.argtypes = [ct.c_int, ct.c_double, dp, dp]
    lib.orc_t92_pij.argtypes = [ct.c_double, ct.c_double, ct.c_double, dp]
    lib.orc_t92_freqs.argtypes = [ct.c_double, dp]
    lib.orc_reversible_generator.argtypes = [ct.c_int, dp, dp, dp]
    lib.orc_gtr_model.argtypes = [ct.c_double] * 8 + [dp, dp]
    lib.orc_reversible_pij.argtypes = [ct.c_int, dp, dp, ct.c_double, dp]
    lib.orc_tree_loglik.argtypes = [ct.c_int, ct.c_int, ip, ip, ip, ct.c_int, ip, ct.c_int, ct.c_int, ct.c_int, dp,
                                    dp, dp, dp, ct.c_int, ct.c_int, ct.c_int, dp, dp, dp, dp]
    lib.orc_tree_loglik_rule.argtypes = [ct.c_int, ct.c_int, ip, ip, ip, ct.c_int, ip, ct.c_int, ct.c_int, ct.c_int,
                                         dp, dp, dp, dp, ct.c_int, ct.c_int, ct.c_int, ct.c_int, dp, dp, dp, dp]
    lib.orc_count_patterns.argtypes = [ct.c_int, ct.c_int, ip]
    lib.orc_dr_derivatives.argtypes = [ct.c_int, ct.c_int, ip, ip, ip, ct.c_int, ip, ct.c_int, ct.c_int, ct.c_int,
                                       dp, dp, dp, dp, dp, dp, dp, dp]
    _lib = lib
    return lib


def _d(a):
    return a.ctypes.data_as(ct.POINTER(ct.c_double))


def _i(a):
    return a.ctypes.data_as(ct.POINTER(ct.c_int32))


def gamma_rates(n: int, alpha: float):
    lib = load()
    r, p = np.empty(n), np.empty(n)
    if lib.orc_gamma_rates(n, alpha, _d(r), _d(p)) != 0:
        raise ValueError("bad gamma parameters")
    return r, p


def t92_pij(kappa: float, theta: float, t: float) -> np.ndarray:
    out = np.empty(16)
    load().orc_t92_pij(kappa, theta, t, _d(out))
    return out.reshape(4, 4)


def t92_freqs(theta: float) -> np.ndarray:
    out = np.empty(4)
    load().orc_t92_freqs(theta, _d(out))
    return out


def gtr_model(a, b, c, d, e, theta, theta1, theta2):
    ex, pi = np.empty(16), np.empty(4)
    load().orc_gtr_model(a, b, c, d, e, theta, theta1, theta2, _d(ex), _d(pi))
    return ex.reshape(4, 4), pi


def reversible_generator(exch: np.ndarray, pi: np.ndarray) -> np.ndarray:
    S = pi.shape[0]
    e = np.ascontiguousarray(exch, dtype=np.float64)
    p = np.ascontiguousarray(pi, dtype=np.float64)
    Q = np.empty(S * S)
    load().orc_reversible_generator(S, _d(e), _d(p), _d(Q))
    return Q.reshape(S, S)


def reversible_pij(Q: np.ndarray, pi: np.ndarray, t: float) -> np.ndarray:
    S = pi.shape[0]
    q = np.ascontiguousarray(Q, dtype=np.float64)
    p = np.ascontiguousarray(pi, dtype=np.float64)
    out = np.empty(S * S)
    load().orc_reversible_pij(S, _d(q), _d(p), t, _d(out))
    return out.reshape(S, S)


def tree_loglik(son_start, sons, leaf_row, root, states, init_table, pmats, class_probs, root_freqs,
                use_patterns=True, scaling=False, n_rep=1, want_sites=False, nh_root=False):
    """pmats: [n_nodes][C][S][S]; states: [n_leaf_rows][n_sites] ints.
    nh_root: RNonHomogeneousTreeLikelihood's root rule (no <= 0 guards, site sum clamped at
    0) instead of RHomogeneousTreeLikelihood's (terms <= 0 dropped).
    Returns (lnL, site_lnl or None, seconds per traversal, seconds for the reduction)."""
    lib = load()
    n_nodes = len(leaf_row)
    states = np.ascontiguousarray(states, dtype=np.int32)
    n_sites = states.shape[1]
    S = init_table.shape[1]
    C = pmats.shape[1]
    lnl = ct.c_double(0)
    tt, tr = ct.c_double(0), ct.c_double(0)
    sites = np.empty(n_sites) if want_sites else None
    args = [np.ascontiguousarray(x, dtype=np.int32) for x in (son_start, sons, leaf_row)]
    it = np.ascontiguousarray(init_table, dtype=np.float64)
    pm = np.ascontiguousarray(pmats, dtype=np.float64)
    cp = np.ascontiguousarray(class_probs, dtype=np.float64)
    rf = np.ascontiguousarray(root_freqs, dtype=np.float64)
    rc = lib.orc_tree_loglik_rule(n_nodes, root, _i(args[0]), _i(args[1]), _i(args[2]), n_sites, _i(states), S, C,
                                  it.shape[0], _d(it), _d(pm), _d(cp), _d(rf), int(use_patterns), int(scaling),
                                  int(nh_root), n_rep, ct.byref(lnl), _d(sites) if want_sites else None,
                                  ct.byref(tt), ct.byref(tr))
    if rc != 0:
        raise ValueError(f"oracle error {rc} (state code not allowed by the model?)")
    return lnl.value, sites, tt.value, tr.value


def dr_derivatives(son_start, sons, leaf_row, root, states, init_table, pmats, dpmats, d2pmats, class_probs,
                   root_freqs):
    """DRHomogeneousTreeLikelihood restatement (orc_dr_derivatives): (d1, d2) per node, d lnL/dt
    and d2 lnL/dt2 of the branch above each node over all sites (flat, unscaled)."""
    lib = load()
    n_nodes = len(leaf_row)
    states = np.ascontiguousarray(states, dtype=np.int32)
    S = init_table.shape[1]
    C = pmats.shape[1]
    args = [np.ascontiguousarray(x, dtype=np.int32) for x in (son_start, sons, leaf_row)]
    it = np.ascontiguousarray(init_table, dtype=np.float64)
    mats = [np.ascontiguousarray(m, dtype=np.float64) for m in (pmats, dpmats, d2pmats)]
    cp = np.ascontiguousarray(class_probs, dtype=np.float64)
    rf = np.ascontiguousarray(root_freqs, dtype=np.float64)
    d1, d2 = np.zeros(n_nodes), np.zeros(n_nodes)
    rc = lib.orc_dr_derivatives(n_nodes, root, _i(args[0]), _i(args[1]), _i(args[2]), states.shape[1], _i(states), S,
                                C, it.shape[0], _d(it), _d(mats[0]), _d(mats[1]), _d(mats[2]), _d(cp), _d(rf),
                                _d(d1), _d(d2))
    if rc != 0:
        raise ValueError(f"oracle error {rc} (state code not allowed by the model?)")
    return d1, d2


def count_patterns(states: np.ndarray) -> int:
    s = np.ascontiguousarray(states, dtype=np.int32)
    return load().orc_count_patterns(s.shape[0], s.shape[1], _i(s))
