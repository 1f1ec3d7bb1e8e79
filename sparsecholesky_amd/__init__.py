"""MI355X-native supernodal sparse Cholesky -- Python mirror of the reference API.

The compute lives in ``libsparsecholesky_amd.so`` (host symbolic analysis in C++,
numeric factorization in hand-written HIP for gfx950), reached through its C ABI
(``include/sparsecholesky.h``) with ctypes.  This module mirrors the reference's
C++ API (evanwporter/SparseCholesky ``include/chol.hpp``) so tests read like the
reference's own gtests:

=========================  ===========================================
reference (chol.hpp)       here
=========================  ===========================================
csc_matrix<T, S>   :134    :class:`csc_matrix`
SChol              :99     :class:`SChol`
triplet_to_csc_matrix :308 :func:`triplet_to_csc_matrix`
etree              :377    :func:`etree`
post_order         :466    :func:`post_order`
col_count          :567    :func:`col_count`
ereach             :725    :func:`ereach`
chol               :750    :func:`chol`   (GPU numeric path)
schol              :874    :func:`schol`
chol_sn            :1407   :func:`chol_sn` (same GPU path; the reference's is broken)
csc_to_dense       :1448   :func:`csc_to_dense`
compute_levels     src/chol.cpp:7     :func:`compute_levels`
compute_supernodes src/chol.cpp:42    :func:`compute_supernodes`
atree              src/chol.cpp:102   :func:`atree`
load_matrix_market_to_csc  mtx_reader.hpp:17  :func:`load_matrix_market_to_csc`
=========================  ===========================================

There is no CPU fallback: :func:`chol` raises if the HIP library or a GPU is
missing.
"""
from __future__ import annotations

import ctypes as C
import enum
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

__all__ = [
    "sym", "csc_matrix", "SChol", "Expected", "lib", "LibraryError",
    "triplet_to_csc_matrix", "build_csc_matrix_from_pattern", "load_matrix_market_to_csc",
    "etree", "post_order", "col_count", "ereach", "schol", "chol", "chol_sn",
    "csc_to_dense", "compute_levels", "compute_supernodes", "atree", "laplacian3d",
    "Symbolic", "Numeric", "Options",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsparsecholesky_amd.so")

SC_OK = 0
_STATUS = {
    -1: "invalid argument", -2: "host allocation failed", -3: "HIP runtime error",
    -4: "device allocation failed", -5: "call out of order", -6: "communication error",
    -7: "not implemented", -8: "matrix is not symmetric", -9: "file could not be opened",
}


class LibraryError(RuntimeError):
    pass


class Options(C.Structure):
    _fields_ = [
        ("struct_size", C.c_int32), ("relax", C.c_int32), ("nrelax", C.c_int32 * 3), ("zrelax", C.c_double * 3),
        ("small_front_max", C.c_int32), ("panel_nb", C.c_int32), ("panel_nb_outer", C.c_int32),
        ("use_graph", C.c_int32), ("relax_wmax", C.c_int32), ("syrk_tile", C.c_int32),
        ("lookahead", C.c_int32), ("inner_order", C.c_int32),
        ("asm_tile_min_m", C.c_int32), ("dist_split", C.c_int32), ("dist_cbb", C.c_int32),
        ("ordering", C.c_int32), ("dist_early", C.c_int32), ("dist_panel", C.c_int32),
        ("cb_gather", C.c_int32),
        ("dist_slab_block", C.c_int32), ("trsm_split_wg", C.c_int32),
        ("syrk_lean_kmax", C.c_int32), ("cb_tail_split", C.c_int32), ("tiny_dense", C.c_int32),
        ("dist_asm", C.c_int32),
        ("dist_pieces", C.c_int32), ("dist_local_pieces", C.c_int32), ("panel_prefactor", C.c_int32),
    ]


class SymbolicStats(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("nnz_A", C.c_int64), ("nnz_L", C.c_int64), ("flops", C.c_double),
        ("etree_depth", C.c_int64), ("n_fundamental", C.c_int64), ("n_supernodes", C.c_int64),
        ("n_levels", C.c_int64), ("max_front_m", C.c_int64), ("max_front_w", C.c_int64),
        ("panel_entries", C.c_int64), ("cb_entries", C.c_int64), ("flops_executed", C.c_double),
        ("flops_syrk_w256", C.c_double), ("n_small_fronts", C.c_int64), ("n_large_fronts", C.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_P = C.c_void_p
_I64 = C.c_int64
_I32 = C.c_int32
_D = C.c_double

# (name, restype, argtypes)
_SIGS = [
    ("sc_version", _I32, []),
    ("sc_status_string", C.c_char_p, [_I64]),
    ("sc_last_error", C.c_char_p, []),
    ("sc_default_options", None, [C.POINTER(Options)]),
    ("sc_analyze", _I64, [_I64, _P, _P, C.POINTER(Options), C.POINTER(_P)]),
    ("sc_symbolic_get_stats", _I64, [_P, C.POINTER(SymbolicStats)]),
    ("sc_nnz_L", _I64, [_P]),
    ("sc_flops", _D, [_P]),
    ("sc_symbolic_pattern", _I64, [_P, _P, _P]),
    ("sc_symbolic_etree", _I64, [_P, _P, _P]),
    ("sc_symbolic_supernodes", _I64, [_P, _P, _P, _P, _P]),
    ("sc_symbolic_perm", _I64, [_P, _P]),
    ("sc_free_symbolic", None, [_P]),
    ("sc_numeric_create", _I64, [_P, _I32, C.POINTER(_P)]),
    ("sc_factor", _I64, [_P, _P]),
    ("sc_factor_device", _I64, [_P, _P, _I32]),
    ("sc_numeric_status", _I64, [_P]),
    ("sc_export_L", _I64, [_P, _P, _P, _P]),
    ("sc_export_L_cols", _I64, [_P, _I64, _I64, _P, _P, _P]),
    ("sc_numeric_stream", _P, [_P]),
    ("sc_numeric_set_profile", _I64, [_P, _I32]),
    ("sc_numeric_timing", _I64, [_P, _P, _I32]),
    ("sc_numeric_level_times", _I64, [_P, _P, _I32]),
    ("sc_numeric_launch_trace", _I64, [_P, _P, _P, _P, _P, _P, _I64]),
    ("sc_numeric_syrk_stats", _I64, [_P, _I32, C.POINTER(_D), C.POINTER(_D), C.POINTER(_I64)]),
    ("sc_numeric_syrk_bytes", _I64, [_P, _I32, C.POINTER(_D)]),
    ("sc_numeric_launch_times", _I64, [_P, _P, _P, _P, _P, _P, _I64]),
    ("sc_free_numeric", None, [_P]),
    ("sc_solve_host", _I64, [_P, _P, _P]),
    ("sc_solve_device", _I64, [_P, _P, _P]),
    ("sc_etree", _I64, [_I64, _P, _P, _P]),
    ("sc_post_order", _I64, [_I64, _P, _P]),
    ("sc_col_count", _I64, [_I64, _P, _P, _P, _P, _P]),
    ("sc_ereach", _I64, [_I64, _P, _P, _P, _I64, _P, _P, _P, _P]),
    ("sc_compute_levels", _I64, [_I64, _P, _P]),
    ("sc_compute_supernodes", _I64, [_I64, _P, _P, _P, _P]),
    ("sc_atree", _I64, [_I64, _P, _P, _P, _P, _I64, _P]),
    ("sc_triplet_to_csc", _I64, [_I64, _I64, _P, _P, _P, _P, _P, _P]),
    ("sc_read_mtx", _I64, [C.c_char_p, C.POINTER(_I64), _P, _P, _P]),
    ("sc_laplacian3d", _I64, [_I64, _I32, _P, _P, _P, _P]),
    ("sc_dist_unique_id", _I64, [_P]),
    ("sc_dist_owner_map", _I64, [_P, _I32, _P, _P]),
    ("sc_numeric_create_dist", _I64, [_P, _I32, _I32, _I32, _P, C.POINTER(_P)]),
    ("sc_dist_schedule", _I64, [_P, _I32, _I32, _P, _P, _P, _P, _I64]),
    ("sc_dist_plan_info", _I64, [_P, _I32, _P, _P, _P, C.POINTER(_I64)]),
    ("sc_dist_steps", _I64, [_P, _I32, _P, _P, _P, _P, _P, _I64]),
    ("sc_numeric_create_dist_host", _I64, [_P, _I32, _I32, _I32, C.c_void_p, _P, C.POINTER(_P)]),
    ("sc_numeric_create_dist_dry", _I64, [_P, _I32, _I32, _I32, C.POINTER(_P)]),
    ("sc_numeric_create_dist_emulated", _I64, [_P, _I32, _I32, _I32, C.POINTER(_P)]),
    ("sc_numeric_memory", _I64, [_P, _P, _I32]),
    ("sc_memory_plan", _I64, [_P, _I32, _P, _P, _P]),
    ("sc_memory_plan_check", _I64, [_P, _I32]),
    ("sc_debug_syrk", _I64, [_P, _I32, _P, _I32, _I32, _I32, _I32]),
    ("sc_debug_bench", _I64, [_I32, _I32, _I32, _I32, _I32, C.POINTER(_D)]),
    ("sc_device_count", _I64, []),
    ("sc_debug_chain_stamps", _I64, [_P, _I32, _P, _I64]),
    ("sc_debug_time_factor", _I64, [_P, C.c_void_p, _I32, C.POINTER(_D)]),
    ("sc_debug_solve_eager", _I64, [_P, _I32]),
    ("sc_debug_hwid", _I64, [_I32, _I32, _I32, _P]),
    ("sc_debug_contention", _I64, [_I32, _I32, _I32, _I32, _I32, _I32, _P]),
]

_lib: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """Load the product library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LibraryError(
                f"{LIB_PATH} missing: build it with `make -C sparsecholesky_amd/csrc` "
                "(or __graft_entry__.build())")
        # torch (when present) bundles its own libamdhip64.so.7; loading it first
        # lets this library bind to the same HIP runtime (same soname) so device
        # pointers and streams are shared instead of two runtimes fighting over
        # the device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, res, args in _SIGS:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return [name for name, _, _ in _SIGS]


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _check(rc: int, what: str):
    if rc < 0:
        msg = lib().sc_last_error()
        raise LibraryError(f"{what}: {_STATUS.get(rc, rc)}" + (f" ({msg.decode()})" if msg else ""))
    return rc


# --------------------------------------------------------------------------
# storage types (chol.hpp:26-299)
# --------------------------------------------------------------------------
class sym(enum.Enum):
    none = 0
    upper = 1
    lower = 2


@dataclass
class csc_matrix:
    """CSC matrix with int64 column pointers (chol.hpp:134 csc_matrix<T,S>)."""
    n_rows: int
    n_cols: int
    p: np.ndarray
    i: np.ndarray
    x: np.ndarray
    S: sym = sym.upper

    def rows(self):
        return self.n_rows

    def cols(self):
        return self.n_cols

    def size(self):
        return self.n_cols

    def capacity(self):
        return int(self.p[-1]) if len(self.p) else 0

    def find_index(self, i: int, j: int) -> int:
        a, b = int(self.p[j]), int(self.p[j + 1])
        k = a + int(np.searchsorted(self.i[a:b], i))
        return k if k < b and self.i[k] == i else -1

    def __getitem__(self, ij):
        i, j = ij
        if self.S == sym.upper and j < i:
            i, j = j, i
        elif self.S == sym.lower and i < j:
            i, j = j, i
        k = self.find_index(i, j)
        return 0.0 if k < 0 else float(self.x[k])

    def transpose(self) -> "csc_matrix":
        n = self.n_cols
        cols = np.repeat(np.arange(n, dtype=np.int32), np.diff(self.p).astype(np.int64))
        order = np.lexsort((cols, self.i))
        tp = np.zeros(self.n_rows + 1, dtype=np.int64)
        np.add.at(tp, self.i.astype(np.int64) + 1, 1)
        tp = np.cumsum(tp)
        St = {sym.upper: sym.lower, sym.lower: sym.upper, sym.none: sym.none}[self.S]
        return csc_matrix(self.n_cols, self.n_rows, tp, cols[order].astype(np.int32),
                          self.x[order].copy(), St)


@dataclass
class SChol:
    """Symbolic factor: pattern of L plus the etree (chol.hpp:99-132)."""
    p: np.ndarray
    i: np.ndarray
    parent: np.ndarray

    def size(self):
        return len(self.p) - 1

    def capacity(self):
        return int(self.p[-1])

    def __getitem__(self, ij):
        i, j = ij
        if i < j:
            i, j = j, i
        a, b = int(self.p[j]), int(self.p[j + 1])
        k = a + int(np.searchsorted(self.i[a:b], i))
        return bool(k < b and self.i[k] == i)


@dataclass
class Expected:
    """std::expected<csc_matrix, std::string> (chol.hpp:750)."""
    _value: Optional[csc_matrix] = None
    _error: Optional[str] = None
    status: int = 0

    def has_value(self):
        return self._value is not None

    def __bool__(self):
        return self.has_value()

    def value(self) -> csc_matrix:
        if self._value is None:
            raise RuntimeError(self._error)
        return self._value

    def error(self) -> str:
        return self._error


# --------------------------------------------------------------------------
# input construction (chol.hpp:308-435, mtx_reader.hpp)
# --------------------------------------------------------------------------
def triplet_to_csc_matrix(ti, tj, tx, n: int) -> csc_matrix:
    ti = np.ascontiguousarray(ti, dtype=np.int32)
    tj = np.ascontiguousarray(tj, dtype=np.int32)
    tx = np.ascontiguousarray(tx, dtype=np.float64)
    assert len(ti) == len(tj) == len(tx)
    Ap = np.zeros(n + 1, dtype=np.int64)
    nnz = _check(lib().sc_triplet_to_csc(n, len(ti), _ptr(ti), _ptr(tj), _ptr(tx), _ptr(Ap), None, None),
                 "triplet_to_csc")
    Ai = np.zeros(max(nnz, 1), dtype=np.int32)
    Ax = np.zeros(max(nnz, 1), dtype=np.float64)
    _check(lib().sc_triplet_to_csc(n, len(ti), _ptr(ti), _ptr(tj), _ptr(tx), _ptr(Ap), _ptr(Ai), _ptr(Ax)),
           "triplet_to_csc")
    return csc_matrix(n, n, Ap, Ai[:nnz], Ax[:nnz], sym.upper)


def build_csc_matrix_from_pattern(pattern) -> csc_matrix:
    """chol.hpp:412-435: every listed (row, col) becomes an upper entry of value 1."""
    ti, tj = [], []
    for r, cols in enumerate(pattern):
        for c in cols:
            a, b = (r, c) if r <= c else (c, r)
            ti.append(a)
            tj.append(b)
    return triplet_to_csc_matrix(ti, tj, np.ones(len(ti)), len(pattern))


def load_matrix_market_to_csc(path: str) -> csc_matrix:
    n = C.c_int64(0)
    nnz = _check(lib().sc_read_mtx(path.encode(), C.byref(n), None, None, None), "read_mtx")
    Ap = np.zeros(n.value + 1, dtype=np.int64)
    Ai = np.zeros(max(nnz, 1), dtype=np.int32)
    Ax = np.zeros(max(nnz, 1), dtype=np.float64)
    _check(lib().sc_read_mtx(path.encode(), C.byref(n), _ptr(Ap), _ptr(Ai), _ptr(Ax)), "read_mtx")
    return csc_matrix(n.value, n.value, Ap, Ai[:nnz], Ax[:nnz], sym.upper)


def laplacian3d(k: int, nd: bool = True, with_perm: bool = False):
    """7-point Laplacian on a k^3 grid in geometric nested-dissection order."""
    nnz = _check(lib().sc_laplacian3d(k, 1 if nd else 0, None, None, None, None), "laplacian3d")
    n = k ** 3
    Ap = np.zeros(n + 1, dtype=np.int64)
    Ai = np.zeros(nnz, dtype=np.int32)
    Ax = np.zeros(nnz, dtype=np.float64)
    perm = np.zeros(n, dtype=np.int32)
    _check(lib().sc_laplacian3d(k, 1 if nd else 0, _ptr(Ap), _ptr(Ai), _ptr(Ax), _ptr(perm)), "laplacian3d")
    A = csc_matrix(n, n, Ap, Ai, Ax, sym.upper)
    return (A, perm) if with_perm else A


# --------------------------------------------------------------------------
# symbolic helpers (chol.hpp:371-739, src/chol.cpp)
# --------------------------------------------------------------------------
def etree(A: csc_matrix) -> np.ndarray:
    parent = np.zeros(A.size(), dtype=np.int32)
    _check(lib().sc_etree(A.size(), _ptr(A.p), _ptr(A.i), _ptr(parent)), "etree")
    return parent


def post_order(parent: np.ndarray) -> np.ndarray:
    parent = np.ascontiguousarray(parent, dtype=np.int32)
    post = np.zeros(len(parent), dtype=np.int32)
    _check(lib().sc_post_order(len(parent), _ptr(parent), _ptr(post)), "post_order")
    return post


def col_count(A: csc_matrix, parent, post) -> np.ndarray:
    parent = np.ascontiguousarray(parent, dtype=np.int32)
    post = np.ascontiguousarray(post, dtype=np.int32)
    cc = np.zeros(A.size(), dtype=np.int64)
    _check(lib().sc_col_count(A.size(), _ptr(A.p), _ptr(A.i), _ptr(parent), _ptr(post), _ptr(cc)), "col_count")
    return cc


def ereach(A: csc_matrix, k: int, parent, s: np.ndarray, w: np.ndarray, x: Optional[np.ndarray] = None) -> int:
    """Fills s[top:] with the reach of row k; w is the caller's mark array (chol.hpp:725,737)."""
    parent = np.ascontiguousarray(parent, dtype=np.int32)
    assert s.dtype == np.int32 and w.dtype == np.int32
    return _check(lib().sc_ereach(A.size(), _ptr(A.p), _ptr(A.i), _ptr(A.x) if x is not None else None, k,
                                  _ptr(parent), _ptr(s), _ptr(w), _ptr(x)), "ereach")


def compute_levels(parent) -> list:
    parent = np.ascontiguousarray(parent, dtype=np.int32)
    lev = np.zeros(len(parent), dtype=np.int32)
    nl = _check(lib().sc_compute_levels(len(parent), _ptr(parent), _ptr(lev)), "compute_levels")
    return [list(np.nonzero(lev == l)[0]) for l in range(nl)]


def compute_supernodes(S: "SChol"):
    """Returns (sn_id, supernodes) as src/chol.cpp:42-100."""
    n = S.size()
    sn_id = np.zeros(n, dtype=np.int32)
    sup = np.zeros(n + 1, dtype=np.int64)
    ns = _check(lib().sc_compute_supernodes(n, _ptr(np.ascontiguousarray(S.parent, dtype=np.int32)),
                                            _ptr(S.p), _ptr(sn_id), _ptr(sup)), "compute_supernodes")
    return sn_id, sup[:ns + 1]


def atree(S: "SChol", sn_id, supernodes) -> np.ndarray:
    ns = len(supernodes) - 1
    sp = np.zeros(ns, dtype=np.int32)
    _check(lib().sc_atree(S.size(), _ptr(S.p), _ptr(S.i), _ptr(np.ascontiguousarray(sn_id, dtype=np.int32)),
                          _ptr(np.ascontiguousarray(supernodes, dtype=np.int64)), ns, _ptr(sp)), "atree")
    return sp


def permute_symmetric(A: csc_matrix, perm: np.ndarray) -> csc_matrix:
    """P A P^T as upper CSC (perm[new] = old); entries below the diagonal of A are
    ignored as the reference does, duplicates are summed."""
    n = A.size()
    ip = np.empty(n, dtype=np.int64)
    ip[np.asarray(perm, dtype=np.int64)] = np.arange(n)
    col = np.repeat(np.arange(n, dtype=np.int64), np.diff(A.p))
    keep = A.i <= col
    a, b = ip[A.i[keep]], ip[col[keep]]
    return triplet_to_csc_matrix(np.minimum(a, b).astype(np.int32), np.maximum(a, b).astype(np.int32),
                                 A.x[keep], n)


def csc_to_dense(A: csc_matrix) -> np.ndarray:
    """chol.hpp:1448-1479 (returns a 2-D array; the reference returns column-major flat)."""
    D = np.zeros((A.rows(), A.cols()))
    cols = np.repeat(np.arange(A.cols()), np.diff(A.p).astype(np.int64))
    D[A.i, cols] = A.x
    if A.S != sym.none:
        D[cols, A.i] = A.x
    return D


# --------------------------------------------------------------------------
# analysis / numeric handles
# --------------------------------------------------------------------------
def default_options(**kw) -> Options:
    o = Options()
    lib().sc_default_options(C.byref(o))
    for k, v in kw.items():
        if k in ("nrelax", "zrelax"):
            for t, vv in enumerate(v):
                getattr(o, k)[t] = vv
        else:
            setattr(o, k, v)
    return o


class Symbolic:
    """Host symbolic analysis (schol + supernodal plan)."""

    def __init__(self, A: csc_matrix, options: Optional[Options] = None, **kw):
        self.A = A
        self.opt = options if options is not None else default_options(**kw)
        h = C.c_void_p()
        _check(lib().sc_analyze(A.size(), _ptr(A.p), _ptr(A.i), C.byref(self.opt), C.byref(h)), "analyze")
        self.h = h
        self.n = A.size()

    def stats(self) -> dict:
        st = SymbolicStats()
        _check(lib().sc_symbolic_get_stats(self.h, C.byref(st)), "stats")
        return st.as_dict()

    @property
    def nnz_L(self) -> int:
        return int(lib().sc_nnz_L(self.h))

    @property
    def flops(self) -> float:
        return float(lib().sc_flops(self.h))

    def pattern(self):
        Lp = np.zeros(self.n + 1, dtype=np.int64)
        Li = np.zeros(max(self.nnz_L, 1), dtype=np.int32)
        _check(lib().sc_symbolic_pattern(self.h, _ptr(Lp), _ptr(Li)), "pattern")
        return Lp, Li[: self.nnz_L]

    def perm(self) -> np.ndarray:
        """Ordering in effect, perm[new] = old (identity unless ordering=SC_ORDER_ND)."""
        p = np.zeros(max(self.n, 1), dtype=np.int32)
        _check(lib().sc_symbolic_perm(self.h, _ptr(p)), "perm")
        return p[: self.n]

    def etree(self):
        parent = np.zeros(self.n, dtype=np.int32)
        post = np.zeros(self.n, dtype=np.int32)
        _check(lib().sc_symbolic_etree(self.h, _ptr(parent), _ptr(post)), "etree")
        return parent, post

    def supernodes(self):
        """dict(start, m, w, parent, level) of the device supernode partition (postorder numbering)."""
        ns = self.stats()["n_supernodes"]
        st = np.zeros(ns + 1, dtype=np.int32)
        m = np.zeros(max(ns, 1), dtype=np.int32)
        par = np.zeros(max(ns, 1), dtype=np.int32)
        lev = np.zeros(max(ns, 1), dtype=np.int32)
        _check(lib().sc_symbolic_supernodes(self.h, _ptr(st), _ptr(m), _ptr(par), _ptr(lev)), "supernodes")
        return dict(start=st, m=m[:ns], w=np.diff(st), parent=par[:ns], level=lev[:ns])

    def owner_map(self, nranks: int):
        ns = self.stats()["n_supernodes"]
        own = np.zeros(max(ns, 1), dtype=np.int32)
        work = np.zeros(nranks, dtype=np.float64)
        _check(lib().sc_dist_owner_map(self.h, nranks, _ptr(own), _ptr(work)), "owner_map")
        return own[:ns], work

    def dist_plan_info(self, nranks: int) -> dict:
        """Multi-GPU plan summary: rank-group size per supernode, CB ranks of split fronts,
        slab ranks of distributed panels, comm steps and total messages."""
        ns = self.stats()["n_supernodes"]
        g = np.zeros(max(ns, 1), dtype=np.int32)
        cbr = np.zeros(max(ns, 1), dtype=np.int32)
        slr = np.zeros(max(ns, 1), dtype=np.int32)
        nst = C.c_int64()
        nmsg = _check(lib().sc_dist_plan_info(self.h, nranks, _ptr(g), _ptr(cbr), _ptr(slr), C.byref(nst)),
                      "dist_plan_info")
        return dict(gsize=g[:ns], split_cb_ranks=cbr[:ns], slab_ranks=slr[:ns], n_steps=nst.value, n_msgs=nmsg)

    def memory_plan(self, nranks: int = 1) -> dict:
        """Device memory plan without a device: per rank the panel arena (L), the
        interval-planned work arena (contribution blocks) and its lower bound, bytes."""
        pb, wb, lb = (np.zeros(nranks, dtype=np.int64) for _ in range(3))
        _check(lib().sc_memory_plan(self.h, nranks, _ptr(pb), _ptr(wb), _ptr(lb)), "memory_plan")
        return dict(panel=pb, work=wb, work_lower_bound=lb)

    def dist_steps(self, nranks: int) -> dict:
        """The plan's comm steps in order: kind (0 INIT, 1 SLAB, 2 DELIVER), level, front,
        slab / column group k and slab piece p."""
        n = _check(lib().sc_dist_steps(self.h, nranks, None, None, None, None, None, 0), "dist_steps")
        k, l, f, sk, sp = (np.zeros(max(n, 1), dtype=np.int32) for _ in range(5))
        _check(lib().sc_dist_steps(self.h, nranks, _ptr(k), _ptr(l), _ptr(f), _ptr(sk), _ptr(sp), n), "dist_steps")
        return dict(kind=k[:n], level=l[:n], front=f[:n], k=sk[:n], p=sp[:n])

    def dist_schedule(self, nranks: int, rank: int):
        """This rank's messages in posting order: (comm step, peer, bytes, is_send)."""
        cnt = _check(lib().sc_dist_schedule(self.h, nranks, rank, None, None, None, None, 0), "dist_schedule")
        lev = np.zeros(max(cnt, 1), dtype=np.int32)
        peer = np.zeros(max(cnt, 1), dtype=np.int32)
        nb = np.zeros(max(cnt, 1), dtype=np.int64)
        snd = np.zeros(max(cnt, 1), dtype=np.int32)
        _check(lib().sc_dist_schedule(self.h, nranks, rank, _ptr(lev), _ptr(peer), _ptr(nb), _ptr(snd), cnt),
               "dist_schedule")
        return lev[:cnt], peer[:cnt], nb[:cnt], snd[:cnt]

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            _lib.sc_free_symbolic(h)
            self.h = None


class Numeric:
    """Device factorization handle (pools + level schedule on one HIP device)."""

    def __init__(self, symb: Symbolic, device: int = -1, rank: int = 0, nranks: int = 1,
                 uid: Optional[bytes] = None, virtual: bool = False, transport=None, rccl_self: bool = False):
        """nranks > 1 with ``uid`` (from :func:`dist_unique_id` on rank 0): this process is
        ``rank`` of a subtree-partitioned multi-GPU factorization over RCCL.  ``virtual=True``
        runs all ``nranks`` ranks in this one process, each with its own memory; every
        message of the plan moves between them (device copies, or with ``rccl_self=True``
        RCCL send/receive to self on a 1-rank communicator).  ``transport`` (e.g.
        :class:`GlooHostTransport`): the multi-process protocol with every transfer staged
        through host memory instead of RCCL (tests; ranks may share a GPU)."""
        self.symb = symb
        self.rank, self.nranks = rank, nranks
        self.transport = transport
        h = C.c_void_p()
        if transport == "dry":
            _check(lib().sc_numeric_create_dist_dry(symb.h, device, rank, nranks, C.byref(h)),
                   "numeric_create_dist_dry")
        elif transport is not None:
            _check(lib().sc_numeric_create_dist_host(symb.h, device, rank, nranks, C.cast(transport.fn, C.c_void_p),
                                                     None, C.byref(h)), "numeric_create_dist_host")
        elif virtual:
            _check(lib().sc_numeric_create_dist_emulated(symb.h, device, nranks, 1 if rccl_self else 0, C.byref(h)),
                   "numeric_create_dist_emulated")
        elif nranks > 1:
            assert uid is not None and len(uid) == 128
            idbuf = C.create_string_buffer(uid, 128)
            _check(lib().sc_numeric_create_dist(symb.h, device, rank, nranks, idbuf, C.byref(h)),
                   "numeric_create_dist")
        else:
            _check(lib().sc_numeric_create(symb.h, device, C.byref(h)), "numeric_create")
        self.h = h

    def factor(self, Ax: np.ndarray) -> int:
        Ax = np.ascontiguousarray(Ax, dtype=np.float64)
        return _check(lib().sc_factor(self.h, _ptr(Ax)), "factor")

    def factor_device(self, d_Ax_ptr: int, sync: bool = True) -> int:
        return _check(lib().sc_factor_device(self.h, C.c_void_p(d_Ax_ptr), 1 if sync else 0), "factor_device")

    def status(self) -> int:
        return _check(lib().sc_numeric_status(self.h), "status")

    def set_profile(self, on=True):
        """True/1: HIP events around every launch (eager); 2: timestamp kernels around the
        CB SYRK launches only (compatible with hipGraph replay); False/0: off."""
        _check(lib().sc_numeric_set_profile(self.h, int(on)), "set_profile")

    def timing(self) -> np.ndarray:
        t = np.zeros(8)
        _check(lib().sc_numeric_timing(self.h, _ptr(t), 8), "timing")
        return t

    def level_times(self) -> np.ndarray:
        nl = self.symb.stats()["n_levels"]
        t = np.zeros(max(nl, 1))
        _check(lib().sc_numeric_level_times(self.h, _ptr(t), nl), "level_times")
        return t[:nl]

    def launch_trace(self) -> dict:
        n = _check(lib().sc_numeric_launch_trace(self.h, None, None, None, None, None, 0), "launch_trace")
        k, l, st = (np.zeros(max(n, 1), dtype=np.int32) for _ in range(3))
        ms, fl = np.zeros(max(n, 1)), np.zeros(max(n, 1))
        _check(lib().sc_numeric_launch_trace(self.h, _ptr(k), _ptr(l), _ptr(st), _ptr(ms), _ptr(fl), n), "trace")
        return dict(kind=k[:n], level=l[:n], stream=st[:n], ms=ms[:n], flops=fl[:n])

    def syrk_stats(self, wmin: int = 256):
        fl, ms, nl = C.c_double(), C.c_double(), C.c_int64()
        _check(lib().sc_numeric_syrk_stats(self.h, wmin, C.byref(fl), C.byref(ms), C.byref(nl)), "syrk_stats")
        return fl.value, ms.value, nl.value

    def launch_times(self) -> dict:
        """Per launch of the last profiled factorization: start / end ms (from the first
        main-stream launch), kind, comm step index (-1 if not a comm launch)."""
        n = _check(lib().sc_numeric_launch_times(self.h, None, None, None, None, None, 0), "launch_times")
        t0, t1 = np.zeros(max(n, 1)), np.zeros(max(n, 1))
        k, st, sm = (np.zeros(max(n, 1), dtype=np.int32) for _ in range(3))
        _check(lib().sc_numeric_launch_times(self.h, _ptr(t0), _ptr(t1), _ptr(k), _ptr(st), _ptr(sm), n),
               "launch_times")
        return dict(t0=t0[:n], t1=t1[:n], kind=k[:n], step=st[:n], stream=sm[:n])

    def syrk_bytes(self, wmin: int = 256) -> float:
        """Algorithmic HBM bytes of the launches syrk_stats(wmin) selects (C ABI
        sc_numeric_syrk_bytes)."""
        b = C.c_double()
        _check(lib().sc_numeric_syrk_bytes(self.h, wmin, C.byref(b)), "syrk_bytes")
        return b.value

    def memory(self) -> dict:
        """Device memory held, bytes: total, panel arenas, work arenas, work lower bound."""
        v = np.zeros(4, dtype=np.int64)
        _check(lib().sc_numeric_memory(self.h, _ptr(v), 4), "memory")
        return dict(total=int(v[0]), panel=int(v[1]), work=int(v[2]), work_lower_bound=int(v[3]))

    @property
    def stream(self) -> int:
        return lib().sc_numeric_stream(self.h) or 0

    def export(self) -> tuple:
        n = self.symb.n
        nz = self.symb.nnz_L
        Lp = np.zeros(n + 1, dtype=np.int64)
        Li = np.zeros(max(nz, 1), dtype=np.int32)
        Lx = np.zeros(max(nz, 1), dtype=np.float64)
        st = _check(lib().sc_export_L(self.h, _ptr(Lp), _ptr(Li), _ptr(Lx)), "export_L")
        return st, csc_matrix(n, n, Lp, Li[:nz], Lx[:nz], sym.none)

    def export_cols(self, j0: int, j1: int) -> tuple:
        """Columns [j0, j1) of L from the panels: (cp, ri, rx), column j's rows
        ri[cp[j-j0]:cp[j-j0+1]] (its front's rows from j down, relaxed zeros included)."""
        cp = np.zeros(j1 - j0 + 1, dtype=np.int64)
        tot = _check(lib().sc_export_L_cols(self.h, j0, j1, _ptr(cp), None, None), "export_cols")
        ri = np.zeros(max(tot, 1), dtype=np.int32)
        rx = np.zeros(max(tot, 1), dtype=np.float64)
        _check(lib().sc_export_L_cols(self.h, j0, j1, _ptr(cp), _ptr(ri), _ptr(rx)), "export_cols")
        return cp, ri[:tot], rx[:tot]

    def solve(self, b: np.ndarray) -> np.ndarray:
        """x = A^{-1} b on the GPU (host vectors in / out)."""
        b = np.ascontiguousarray(b, dtype=np.float64)
        x = np.zeros_like(b)
        st = _check(lib().sc_solve_host(self.h, _ptr(b), _ptr(x)), "solve")
        if st > 0:
            raise LibraryError(f"solve: A is not positive definite (column {st})")
        return x

    def solve_device(self, d_b_ptr: int, d_x_ptr: int) -> int:
        """x = A^{-1} b with device vectors (may alias)."""
        st = _check(lib().sc_solve_device(self.h, C.c_void_p(d_b_ptr), C.c_void_p(d_x_ptr)), "solve_device")
        if st > 0:
            raise LibraryError(f"solve_device: A is not positive definite (column {st})")
        return st

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            _lib.sc_free_numeric(h)
            self.h = None


_XPORT_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int64)


class GlooHostTransport:
    """Host-staged transport for :class:`Numeric` over ``torch.distributed`` (gloo):
    every comm step's buffers go device -> host -> gloo isend/irecv -> host -> device.
    For tests and debugging of the multi-process protocol without RCCL (several
    processes may then share one GPU); not a performance path."""

    def __init__(self, group=None):
        import torch.distributed as tdist

        self._dist = tdist
        self._group = group
        self._pending = []
        self.error = None
        self.fn = _XPORT_FN(self._callback)  # kept alive with the transport

    def _callback(self, ctx, op, peer, buf, nbytes):
        try:
            if op == 2:
                for w in self._pending:
                    w.wait()
                self._pending = []
                return 0
            import torch

            t = torch.frombuffer((C.c_char * nbytes).from_address(buf), dtype=torch.uint8)
            if op == 0:
                self._pending.append(self._dist.isend(t, int(peer), group=self._group))
            else:
                self._pending.append(self._dist.irecv(t, int(peer), group=self._group))
            return 0
        except Exception as e:  # reported through the library's status
            self.error = repr(e)
            return 1


def dist_unique_id() -> bytes:
    """RCCL unique id (128 bytes) for sc_numeric_create_dist; create on rank 0, broadcast."""
    buf = C.create_string_buffer(128)
    _check(lib().sc_dist_unique_id(buf), "dist_unique_id")
    return buf.raw


# --------------------------------------------------------------------------
# drop-in entry points
# --------------------------------------------------------------------------
def schol(A: csc_matrix, **kw) -> SChol:
    """Symbolic factorization (chol.hpp:873-946)."""
    s = Symbolic(A, **kw)
    Lp, Li = s.pattern()
    parent, _ = s.etree()
    return SChol(Lp, Li, parent)


def chol(A: csc_matrix, S=None, device: int = -1, **kw) -> Expected:
    """Numeric Cholesky on the GPU (chol.hpp:749-863; README's chol(A, S) form too).

    ``S`` may be a :class:`Symbolic` from a previous analysis of the same pattern.
    Returns an :class:`Expected` holding L (CSC, lower, reference layout) or the
    reference's error string.
    """
    symb = S if isinstance(S, Symbolic) else Symbolic(A, **kw)
    num = Numeric(symb, device)
    st = num.factor(A.x)
    if st > 0:
        return Expected(None, "A is not positive definite.", st)
    _, L = num.export()
    return Expected(L, None, 0)


def chol_sn(A: csc_matrix, **kw) -> Expected:
    """The reference's supernodal entry point (chol.hpp:1407); same GPU path as chol()."""
    return chol(A, **kw)
