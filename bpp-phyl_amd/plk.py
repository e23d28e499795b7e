"""ctypes binding of libplk (include/plk.h) -- the Python side of the C-ABI boundary.

This is the binding a Python maintainer would add for the engine; the C++ Bio++
host mirror (bpp-phyl_amd/host) binds the same symbols directly.  Errors become
PlkError carrying plk_last_error().  There is no fallback: if libplk.so is missing
or no gfx950 device is present, calls fail loudly.
"""
from __future__ import annotations

import ctypes as ct
import os
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PLK_LIB") or os.path.join(_HERE, "libplk.so")  # PLK_LIB: A/B builds

PLK_OK = 0
BLOCK = 4096  # plk_block_size(): patterns per fixed-order root block sum
PLK_FLAG_SCALING = 1
PLK_FLAG_NONNEG_GUARD = 2
PLK_FLAG_LNL_ONLY = 4
PLK_FLAG_LEVELWISE = 8
PLK_FLAG_SUBTREE_PATTERNS = 16
PLK_FLAG_DOUBLE_RECURSIVE = 32
PLK_DERIV_P, PLK_DERIV_DP, PLK_DERIV_D2P = 1, 2, 4
PLK_OP_ACCUMULATE = 1
PLK_TIME_PARTIALS, PLK_TIME_PMAT, PLK_TIME_ROOT, PLK_TIME_TABLES = 1, 2, 4, 8

# every symbol include/plk.h declares
EXPORTS = [
    "plk_abi_version", "plk_build_id", "plk_device_count", "plk_last_error", "plk_create", "plk_destroy",
    "plk_set_code_table", "plk_set_tip_codes", "plk_set_pattern_weights", "plk_set_category_rates",
    "plk_set_root_frequencies", "plk_set_eigen", "plk_update_pmatrices", "plk_set_pmatrix",
    "plk_get_pmatrix", "plk_update_partials", "plk_get_partials", "plk_root_loglik", "plk_block_size",
    "plk_set_timing", "plk_get_timing", "plk_reset_timing", "plk_synchronize", "plk_branch_derivatives",
    "plk_kernel_path", "plk_evaluate", "plk_compressed_work", "plk_all_branch_derivatives",
    "plk_get_timing_ex", "plk_traversal_work", "plk_create_multi", "plk_shard_count", "plk_comm_get_id",
    "plk_comm_init", "plk_get_dpmatrix", "plk_root_pair_derivatives", "plk_get_fanout",
    "plk_root_underflow", "plk_exchange_stride", "plk_exchange_pack", "plk_exchange_reduce",
    "plk_exchange_rank_sums", "plk_clock_records",
]


class PlkError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"plk error {code}: {msg}")
        self.code = code


class plk_op(ct.Structure):
    _fields_ = [("parent", ct.c_int32), ("n_children", ct.c_int32), ("child", ct.c_int32 * 3),
                ("flags", ct.c_int32)]


class plk_timing(ct.Structure):
    _fields_ = [("partials_launches", ct.c_int64), ("partials_ms", ct.c_double), ("pmat_ms", ct.c_double),
                ("root_ms", ct.c_double), ("tables_ms", ct.c_double), ("table_launches", ct.c_int64),
                ("evaluations", ct.c_int64), ("host_us", ct.c_double * 6)]


class plk_work(ct.Structure):
    _fields_ = [("patterns", ct.c_int64), ("node_updates", ct.c_int64), ("table_nodes", ct.c_int64),
                ("table_rows", ct.c_int64), ("useful_flops", ct.c_double), ("issued_flops", ct.c_double),
                ("table_flops", ct.c_double), ("exact", ct.c_int32), ("internal_nodes", ct.c_int32)]


class plk_comm_id(ct.Structure):
    _fields_ = [("internal", ct.c_char * 128)]


_lib = None
ABI_VERSION = 2  # include/plk.h PLK_ABI_VERSION


def load(path: str = LIB_PATH) -> ct.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built (run make -C bpp-phyl_amd); libplk has no CPU fallback")
    lib = ct.CDLL(path)
    P = ct.POINTER
    dp, ip = P(ct.c_double), P(ct.c_int32)
    sig = {
        "plk_abi_version": ([], ct.c_int),
        "plk_build_id": ([], ct.c_char_p),
        "plk_device_count": ([P(ct.c_int)], ct.c_int),
        "plk_last_error": ([ct.c_void_p], ct.c_char_p),
        "plk_create": ([ct.c_int, ct.c_int, ct.c_int, ct.c_int64, ct.c_int, ct.c_int, ct.c_int, ct.c_uint,
                        P(ct.c_void_p)], ct.c_int),
        "plk_destroy": ([ct.c_void_p], ct.c_int),
        "plk_create_multi": ([P(ct.c_int), ct.c_int, ct.c_int, ct.c_int, ct.c_int64, ct.c_int, ct.c_int, ct.c_int,
                              ct.c_uint, P(ct.c_void_p)], ct.c_int),
        "plk_shard_count": ([ct.c_void_p, P(ct.c_int)], ct.c_int),
        "plk_get_fanout": ([ct.c_void_p, ct.c_int, dp, dp, P(ct.c_int64)], ct.c_int),
        "plk_root_underflow": ([ct.c_void_p, P(ct.c_int)], ct.c_int),
        "plk_clock_records": ([ct.c_void_p, dp, ct.c_int, P(ct.c_int)], ct.c_int),
        "plk_comm_get_id": ([P(plk_comm_id)], ct.c_int),
        "plk_exchange_stride": ([P(ct.c_int64), ct.c_int, P(ct.c_int64)], ct.c_int),
        "plk_exchange_pack": ([dp, ct.c_int64, ct.c_int, ct.c_int64, dp], ct.c_int),
        "plk_exchange_reduce": ([dp, P(ct.c_int64), ct.c_int, ct.c_int64, dp, P(ct.c_int)], ct.c_int),
        "plk_exchange_rank_sums": ([dp, ct.c_int, ct.c_int64, dp], ct.c_int),
        "plk_comm_init": ([ct.c_void_p, ct.c_int, ct.c_int, P(plk_comm_id)], ct.c_int),
        "plk_set_code_table": ([ct.c_void_p, ct.c_int, dp], ct.c_int),
        "plk_set_tip_codes": ([ct.c_void_p, ct.c_int, P(ct.c_uint8)], ct.c_int),
        "plk_set_pattern_weights": ([ct.c_void_p, dp], ct.c_int),
        "plk_set_category_rates": ([ct.c_void_p, dp, dp], ct.c_int),
        "plk_set_root_frequencies": ([ct.c_void_p, dp], ct.c_int),
        "plk_set_eigen": ([ct.c_void_p, ct.c_int, dp, dp, dp], ct.c_int),
        "plk_update_pmatrices": ([ct.c_void_p, ct.c_int, ip, ip, dp, ct.c_uint], ct.c_int),
        "plk_set_pmatrix": ([ct.c_void_p, ct.c_int, dp], ct.c_int),
        "plk_get_pmatrix": ([ct.c_void_p, ct.c_int, dp], ct.c_int),
        "plk_get_dpmatrix": ([ct.c_void_p, ct.c_int, ct.c_int, dp], ct.c_int),
        "plk_update_partials": ([ct.c_void_p, P(plk_op), ct.c_int], ct.c_int),
        "plk_get_partials": ([ct.c_void_p, ct.c_int, dp], ct.c_int),
        "plk_root_loglik": ([ct.c_void_p, ct.c_int, dp, dp, dp], ct.c_int),
        "plk_block_size": ([], ct.c_int),
        "plk_set_timing": ([ct.c_void_p, ct.c_int], ct.c_int),
        "plk_get_timing": ([ct.c_void_p, P(ct.c_int64), dp, dp, dp], ct.c_int),
        "plk_get_timing_ex": ([ct.c_void_p, P(plk_timing)], ct.c_int),
        "plk_traversal_work": ([ct.c_void_p, P(plk_work)], ct.c_int),
        "plk_reset_timing": ([ct.c_void_p], ct.c_int),
        "plk_synchronize": ([ct.c_void_p], ct.c_int),
        "plk_branch_derivatives": ([ct.c_void_p, ct.c_int, dp, dp], ct.c_int),
        "plk_root_pair_derivatives": ([ct.c_void_p, ct.c_int, ct.c_int, ct.c_double, ct.c_double, dp, dp], ct.c_int),
        "plk_all_branch_derivatives": ([ct.c_void_p, dp, dp], ct.c_int),
        "plk_kernel_path": ([ct.c_void_p], ct.c_char_p),
        "plk_compressed_work": ([ct.c_void_p, P(ct.c_int64)], ct.c_int),
        "plk_evaluate": ([ct.c_void_p, ct.c_int, ip, ip, dp, P(plk_op), ct.c_int, ct.c_int, dp, dp], ct.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name, None)
        if f is None and os.environ.get("PLK_LIB"):
            continue  # an older A/B build (PLK_LIB) without this entry point
        if f is None:
            raise AttributeError(f"{path}: missing {name}")
        f.argtypes = args
        f.restype = res
    if lib.plk_abi_version() != ABI_VERSION:  # the structs above mirror this version of plk.h
        raise RuntimeError(f"{path}: ABI version {lib.plk_abi_version()}, this binding needs {ABI_VERSION}")
    _lib = lib
    return lib


def source_hash() -> str:
    """The build id libplk.so should report when built from the sources beside it
    (same recipe as bpp-phyl_amd/Makefile: SHA-256 over csrc/*.hip, csrc/*.hpp in sorted
    order, then include/plk.h; first 16 hex digits)."""
    import glob
    import hashlib

    csrc = os.path.join(_HERE, "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp")))
    files.append(os.path.join(os.path.dirname(_HERE), "include", "plk.h"))
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def comm_get_id() -> bytes:
    """plk_comm_get_id (ncclGetUniqueId) on one rank; share the 128 bytes with the others."""
    cid = plk_comm_id()
    lib = load()
    rc = lib.plk_comm_get_id(ct.byref(cid))
    if rc != PLK_OK:
        raise PlkError(rc, lib.plk_last_error(None).decode())
    return ct.string_at(ct.addressof(cid), 128)   # all 128 bytes (a c_char field stops at NUL)


def _chk(rc: int):
    if rc != PLK_OK:
        raise PlkError(rc, load().plk_last_error(None).decode())


# The exchange bookkeeping of the communicator path (csrc/plk_exchange.hpp): host only, usable
# without a GPU.  Record of a rank = its block sums, zero padding, its underflow flag.

def exchange_stride(counts: Sequence[int]) -> int:
    c = np.ascontiguousarray(counts, dtype=np.int64)
    out = ct.c_int64(0)
    _chk(load().plk_exchange_stride(c.ctypes.data_as(ct.POINTER(ct.c_int64)), len(c), ct.byref(out)))
    return out.value


def exchange_pack(block_sums: np.ndarray, uflow: bool, stride: int) -> np.ndarray:
    b = np.ascontiguousarray(block_sums, dtype=np.float64)
    rec = np.full(stride, np.nan)
    _chk(load().plk_exchange_pack(_d(b), len(b), int(bool(uflow)), stride, _d(rec)))
    return rec


def exchange_reduce(gathered: np.ndarray, counts: Sequence[int], stride: int) -> Tuple[float, bool]:
    g = np.ascontiguousarray(gathered, dtype=np.float64).ravel()
    c = np.ascontiguousarray(counts, dtype=np.int64)
    lnl, f = ct.c_double(0), ct.c_int(0)
    _chk(load().plk_exchange_reduce(_d(g), c.ctypes.data_as(ct.POINTER(ct.c_int64)), len(c), stride, ct.byref(lnl),
                                    ct.byref(f)))
    return lnl.value, bool(f.value)


def exchange_rank_sums(gathered: np.ndarray, n_ranks: int) -> np.ndarray:
    g = np.ascontiguousarray(gathered, dtype=np.float64).ravel()
    n = len(g) // n_ranks
    v = np.empty(n)
    _chk(load().plk_exchange_rank_sums(_d(g), n_ranks, n, _d(v)))
    return v


def build_id() -> str:
    return load().plk_build_id().decode()


def _d(a: np.ndarray):
    return a.ctypes.data_as(ct.POINTER(ct.c_double))


def device_count() -> int:
    lib = load()
    n = ct.c_int(0)
    lib.plk_device_count(ct.byref(n))
    return n.value


def make_ops(ops: Sequence[Tuple[int, Sequence[int], int]]):
    arr = (plk_op * len(ops))()
    for i, (p, ch, fl) in enumerate(ops):
        arr[i].parent = p
        arr[i].n_children = len(ch)
        for k, c in enumerate(ch):
            arr[i].child[k] = c
        arr[i].flags = fl
    return arr


class Engine:
    """One libplk handle (one device, one pattern shard)."""

    def __init__(self, device, n_states: int, n_classes: int, n_patterns: int, n_tips: int,
                 n_internal: int, n_models: int = 1, flags: int = PLK_FLAG_NONNEG_GUARD):
        """device: one HIP device, or a list of devices (plk_create_multi: the patterns are
        sharded over them in contiguous block-aligned ranges; same calls, whole-alignment
        arguments)."""
        self.lib = load()
        self.h = ct.c_void_p()
        self.S, self.C, self.P = n_states, n_classes, n_patterns
        self.n_tips, self.n_internal = n_tips, n_internal
        self._ops_cache = None
        self._eval_cache = None
        self._eval_call = None
        if isinstance(device, (list, tuple)):
            devs = (ct.c_int * len(device))(*device)
            rc = self.lib.plk_create_multi(devs, len(device), n_states, n_classes, n_patterns, n_tips, n_internal,
                                           n_models, flags, ct.byref(self.h))
        else:
            rc = self.lib.plk_create(device, n_states, n_classes, n_patterns, n_tips, n_internal, n_models, flags,
                                     ct.byref(self.h))
        if rc != PLK_OK:
            raise PlkError(rc, self.lib.plk_last_error(None).decode())

    def _chk(self, rc: int):
        if rc != PLK_OK:
            raise PlkError(rc, self.lib.plk_last_error(self.h).decode())

    def close(self):
        if self.h:
            self.lib.plk_destroy(self.h)
            self.h = ct.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_code_table(self, table: np.ndarray):
        t = np.ascontiguousarray(table, dtype=np.float64)
        self._chk(self.lib.plk_set_code_table(self.h, t.shape[0], _d(t)))

    def set_tip_codes(self, tip: int, codes: np.ndarray):
        c = np.ascontiguousarray(codes, dtype=np.uint8)
        self._chk(self.lib.plk_set_tip_codes(self.h, tip, c.ctypes.data_as(ct.POINTER(ct.c_uint8))))

    def set_pattern_weights(self, w: np.ndarray):
        w = np.ascontiguousarray(w, dtype=np.float64)
        self._chk(self.lib.plk_set_pattern_weights(self.h, _d(w)))

    def set_category_rates(self, rates: np.ndarray, probs: np.ndarray):
        r = np.ascontiguousarray(rates, dtype=np.float64)
        p = np.ascontiguousarray(probs, dtype=np.float64)
        self._chk(self.lib.plk_set_category_rates(self.h, _d(r), _d(p)))

    def set_root_frequencies(self, pi: np.ndarray):
        p = np.ascontiguousarray(pi, dtype=np.float64)
        self._chk(self.lib.plk_set_root_frequencies(self.h, _d(p)))

    def set_eigen(self, model: int, V: np.ndarray, Vinv: np.ndarray, lam: np.ndarray):
        V = np.ascontiguousarray(V, dtype=np.float64)
        Vi = np.ascontiguousarray(Vinv, dtype=np.float64)
        la = np.ascontiguousarray(lam, dtype=np.float64)
        self._chk(self.lib.plk_set_eigen(self.h, model, _d(V), _d(Vi), _d(la)))

    def update_pmatrices(self, branches: np.ndarray, t: np.ndarray, models: Optional[np.ndarray] = None,
                         deriv_mask: int = PLK_DERIV_P):
        b = np.ascontiguousarray(branches, dtype=np.int32)
        tt = np.ascontiguousarray(t, dtype=np.float64)
        mp = None
        if models is not None:
            m = np.ascontiguousarray(models, dtype=np.int32)
            mp = m.ctypes.data_as(ct.POINTER(ct.c_int32))
        self._chk(self.lib.plk_update_pmatrices(self.h, len(b), b.ctypes.data_as(ct.POINTER(ct.c_int32)), mp,
                                                _d(tt), deriv_mask))

    def set_pmatrix(self, branch: int, P: np.ndarray):
        p = np.ascontiguousarray(P, dtype=np.float64)
        assert p.size == self.C * self.S * self.S
        self._chk(self.lib.plk_set_pmatrix(self.h, branch, _d(p)))

    def get_pmatrix(self, branch: int) -> np.ndarray:
        out = np.empty((self.C, self.S, self.S))
        self._chk(self.lib.plk_get_pmatrix(self.h, branch, _d(out)))
        return out

    def get_dpmatrix(self, branch: int, order: int) -> np.ndarray:
        """r_c dP/dt (order 1) or r_c^2 d2P/dt2 (order 2) of the branch, per class."""
        out = np.empty((self.C, self.S, self.S))
        self._chk(self.lib.plk_get_dpmatrix(self.h, branch, order, _d(out)))
        return out

    def _op_array(self, ops):
        if self._ops_cache is None or self._ops_cache[2] is not ops:  # same list object: reuse its ctypes array
            key = tuple((p, tuple(c), f) for p, c, f in ops)
            if self._ops_cache is None or self._ops_cache[0] != key:
                self._ops_cache = (key, make_ops(ops), ops)
            else:
                self._ops_cache = (key, self._ops_cache[1], ops)
        return self._ops_cache[1]

    def update_partials(self, ops: Sequence[Tuple[int, Sequence[int], int]]):
        arr = self._op_array(ops)
        self._chk(self.lib.plk_update_partials(self.h, arr, len(arr)))

    def evaluate(self, branches: np.ndarray, t: np.ndarray, ops, root: int, models: Optional[np.ndarray] = None):
        """plk_evaluate: P(t) of `branches`, the traversal `ops`, the root reduction in one
        call.  Returns (lnL, block_sums).  The branch / model index arrays are converted
        once per array object (an optimiser loop passes the same ones every time): the
        cache holds strong references to the caller's objects and matches them by
        identity, so a freed array's id can never alias a new one.  Index arrays must not
        be mutated in place between calls (they are treated as immutable)."""
        c = self._eval_cache
        if c is None or c[0] is not branches or c[1] is not models:
            b = np.ascontiguousarray(branches, dtype=np.int32)
            m = None if models is None else np.ascontiguousarray(models, dtype=np.int32)
            nb = (self.P + self.lib.plk_block_size() - 1) // self.lib.plk_block_size()
            blocks, tbuf = np.empty(nb), np.empty(len(b))
            # pointers made once: numpy's ctypes.data_as costs microseconds per call, a
            # visible share of a ~150 us evaluation
            self._eval_cache = (branches, models, b, m, b.ctypes.data_as(ct.POINTER(ct.c_int32)),
                                None if m is None else m.ctypes.data_as(ct.POINTER(ct.c_int32)), blocks,
                                _d(blocks), tbuf, _d(tbuf), ct.c_double(0.0))
        c = self._eval_cache
        _, _, b, _, bp, mp, blocks_buf, blocks_p, tbuf, tbuf_p, lnl = c
        if getattr(t, "shape", None) != tbuf.shape and np.shape(t) != tbuf.shape:
            raise ValueError(f"branch lengths: {np.shape(t)} for {tbuf.shape[0]} branches")
        tbuf[:] = t  # (float64 conversion included)
        # The call's arguments are the same ctypes objects from one evaluation to the next
        # (same op list object, root and index arrays): they are made once, and passed to an
        # entry point without argtypes -- ctypes' per-call argument conversion cost ~2 of the
        # ~3 us of a ten-argument call (the objects are already the C types plk.h declares)
        call = self._eval_call
        if call is None or call[0] is not ops or call[1] != root or call[2] is not c:
            arr = self._op_array(ops)
            fn = self.lib["plk_evaluate"]  # (a fresh function object: lib.plk_evaluate keeps its argtypes)
            fn.restype = ct.c_int
            args = (self.h, ct.c_int(len(b)), bp, mp, tbuf_p, ct.cast(arr, ct.POINTER(plk_op)), ct.c_int(len(arr)),
                    ct.c_int(root), ct.byref(lnl), blocks_p)
            call = self._eval_call = (ops, root, c, fn, args, arr)
        self._chk(call[3](*call[4]))
        return lnl.value, blocks_buf.copy()

    def get_partials(self, node: int) -> np.ndarray:
        out = np.empty((self.P, self.C, self.S))
        self._chk(self.lib.plk_get_partials(self.h, node, _d(out)))
        return out

    def root_loglik(self, root: int, want_sites: bool = False, want_blocks: bool = False):
        lnl = ct.c_double(0.0)
        sites = np.empty(self.P) if want_sites else None
        nb = (self.P + self.lib.plk_block_size() - 1) // self.lib.plk_block_size()
        blocks = np.empty(nb) if want_blocks else None
        self._chk(self.lib.plk_root_loglik(self.h, root, ct.byref(lnl), _d(sites) if want_sites else None,
                                           _d(blocks) if want_blocks else None))
        return lnl.value, sites, blocks

    def root_underflow(self) -> bool:
        """plk_root_underflow (unscaled handles): did the last root reduction meet a site
        likelihood below 2^-255 (or <= 0, or NaN)?  False proves a scaled handle would have
        returned bitwise the same lnL."""
        f = ct.c_int(0)
        self._chk(self.lib.plk_root_underflow(self.h, ct.byref(f)))
        return bool(f.value)

    def clock_records(self) -> np.ndarray:
        """plk_clock_records (PLK_DEBUG_CLOCK=1): per stamped traversal [shader MHz over all
        workgroups, slowest / fastest workgroup MHz, span us, workgroups]; clears them."""
        n = ct.c_int(0)
        self._chk(self.lib.plk_clock_records(self.h, None, 0, ct.byref(n)))
        out = np.zeros((n.value, 5))
        if n.value:
            self._chk(self.lib.plk_clock_records(self.h, _d(out), n.value, ct.byref(n)))
        return out

    def branch_derivatives(self, branch: int):
        """(d lnL/dt, d2 lnL/dt2) for the branch above node `branch`."""
        d1, d2 = ct.c_double(0), ct.c_double(0)
        self._chk(self.lib.plk_branch_derivatives(self.h, branch, ct.byref(d1), ct.byref(d2)))
        return d1.value, d2.value

    def root_pair_derivatives(self, a: int, b: int, alpha: float, beta: float):
        """Directional (d lnL/ds, d2 lnL/ds2) for root sons a, b moved by t_a + alpha s,
        t_b + beta s (the reference's BrLenRoot / RootPosition derivatives)."""
        d1, d2 = ct.c_double(0), ct.c_double(0)
        self._chk(self.lib.plk_root_pair_derivatives(self.h, a, b, alpha, beta, ct.byref(d1), ct.byref(d2)))
        return d1.value, d2.value

    def all_branch_derivatives(self):
        """Double-recursive pass (PLK_FLAG_DOUBLE_RECURSIVE): (d1, d2) arrays indexed by
        node, d lnL/dt and d2 lnL/dt2 of every branch of the last traversal (0 at the root)."""
        n = self.n_tips + self.n_internal
        d1, d2 = np.zeros(n), np.zeros(n)
        self._chk(self.lib.plk_all_branch_derivatives(self.h, _d(d1), _d(d2)))
        return d1, d2

    def set_timing(self, on: bool):
        self._chk(self.lib.plk_set_timing(self.h, (PLK_TIME_PARTIALS | PLK_TIME_PMAT | PLK_TIME_ROOT) if on is True
                                          else int(on)))

    def get_timing(self):
        t = plk_timing()
        self._chk(self.lib.plk_get_timing_ex(self.h, ct.byref(t)))
        return {"launches": t.partials_launches, "partials_ms": t.partials_ms, "pmat_ms": t.pmat_ms,
                "root_ms": t.root_ms, "tables_ms": t.tables_ms, "table_launches": t.table_launches,
                "evaluations": t.evaluations, "host_us": list(t.host_us)}

    def traversal_work(self) -> dict:
        """plk_traversal_work: node updates computed per pattern vs served by tables, and
        the fp64 flops of the last traversal (counted from the program that ran)."""
        w = plk_work()
        self._chk(self.lib.plk_traversal_work(self.h, ct.byref(w)))
        return {k: getattr(w, k) for k, _ in plk_work._fields_}

    def reset_timing(self):
        self._chk(self.lib.plk_reset_timing(self.h))

    def synchronize(self):
        self._chk(self.lib.plk_synchronize(self.h))

    def compressed_work(self) -> int:
        """Node updates the last compressed traversal computed (sum of distinct subtree patterns)."""
        n = ct.c_int64(0)
        self._chk(self.lib.plk_compressed_work(self.h, ct.byref(n)))
        return n.value

    def shard_count(self) -> int:
        n = ct.c_int(0)
        self._chk(self.lib.plk_shard_count(self.h, ct.byref(n)))
        return n.value

    def fanout(self) -> dict:
        """plk_get_fanout: per shard, the mean offsets (us) from posting an evaluation to the
        shard's worker starting it, to its traversal launch call returning and to its stream
        wait returning; the spread (last - first traversal launch), mean and max."""
        ns = self.shard_count()
        off, spread, n = np.zeros(3 * ns), np.zeros(2), ct.c_int64(0)
        self._chk(self.lib.plk_get_fanout(self.h, ns, _d(off), _d(spread), ct.byref(n)))
        o = off.reshape(ns, 3)
        return {"evaluations": n.value, "start_us": o[:, 0].tolist(), "traversal_launched_us": o[:, 1].tolist(),
                "waited_us": o[:, 2].tolist(), "launch_spread_mean_us": float(spread[0]),
                "launch_spread_max_us": float(spread[1])}

    def comm_init(self, n_ranks: int, rank: int, comm_id: bytes):
        """plk_comm_init: RCCL communicator inside the handle; evaluations then return the
        global lnL of all ranks (one all-gather of block sums per evaluation)."""
        if len(comm_id) != 128:
            raise ValueError("a plk_comm_id is 128 bytes")
        cid = plk_comm_id()
        ct.memmove(ct.addressof(cid), bytes(comm_id), 128)   # (a c_char field reads back as a copy)
        self._chk(self.lib.plk_comm_init(self.h, n_ranks, rank, ct.byref(cid)))

    def kernel_path(self) -> str:
        """Kernel that served the last update_partials ("jit_tree4", "tree4", "treeS", "treeM", "levelwise")."""
        return self.lib.plk_kernel_path(self.h).decode()
