"""TEST INFRASTRUCTURE ONLY -- parity checker, not product code.

ctypes front-end of ``oracle/refchol.c``, the CPU restatement of the reference's
simplicial ``chol()`` (evanwporter/SparseCholesky include/chol.hpp:749-863) and
its symbolic helpers.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module.

Parity pinning: see DESIGN.md "Oracle" -- the reference is unbuildable here
(needs stand-in headers), so the oracle is pinned by the reference's own known
answers and by reference outputs recorded in SURVEY.md, committed in
tests/golden/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle_refchol.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P, I64 = C.c_void_p, C.c_int64
        L.oracle_etree.argtypes = [I64, P, P, P]
        L.oracle_post_order.argtypes = [I64, P, P]
        L.oracle_col_count.argtypes = [I64, P, P, P, P, P]
        L.oracle_ereach.argtypes = [I64, P, P, P, I64, P, P, P, P]
        L.oracle_ereach.restype = I64
        L.oracle_symbolic.argtypes = [I64, P, P, P, P, P, P, C.POINTER(C.c_double)]
        L.oracle_symbolic.restype = I64
        L.oracle_chol.argtypes = [I64, P, P, P, P, P, P, P, C.c_int]
        L.oracle_chol.restype = I64
        L.oracle_schol.argtypes = [I64, P, P, P, P, P]
        L.oracle_time_chol.argtypes = [I64, P, P, P, C.c_int, C.c_int, C.POINTER(C.c_double)]
        L.oracle_time_chol.restype = I64
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _csc(A):
    Ap = np.ascontiguousarray(A.p, dtype=np.int64)
    Ai = np.ascontiguousarray(A.i, dtype=np.int32)
    Ax = np.ascontiguousarray(A.x, dtype=np.float64) if getattr(A, "x", None) is not None else None
    return Ap, Ai, Ax


def etree(A):
    Ap, Ai, _ = _csc(A)
    n = len(Ap) - 1
    parent = np.zeros(n, dtype=np.int32)
    lib().oracle_etree(n, _p(Ap), _p(Ai), _p(parent))
    return parent


def post_order(parent):
    parent = np.ascontiguousarray(parent, dtype=np.int32)
    post = np.zeros(len(parent), dtype=np.int32)
    lib().oracle_post_order(len(parent), _p(parent), _p(post))
    return post


def ereach(A, k, parent, s, w, with_x=False):
    Ap, Ai, Ax = _csc(A)
    n = len(Ap) - 1
    parent = np.ascontiguousarray(parent, dtype=np.int32)
    x = np.zeros(n) if with_x else None
    top = lib().oracle_ereach(n, _p(Ap), _p(Ai), _p(Ax) if with_x else None, k, _p(parent), _p(s), _p(w), _p(x))
    return top, x


def symbolic(A):
    """Returns dict(parent, post, colcount, Lp, nnz_L, flops, depth)."""
    Ap, Ai, _ = _csc(A)
    n = len(Ap) - 1
    parent = np.zeros(n, dtype=np.int32)
    post = np.zeros(n, dtype=np.int32)
    cc = np.zeros(n, dtype=np.int64)
    Lp = np.zeros(n + 1, dtype=np.int64)
    fl = C.c_double(0.0)
    nz = lib().oracle_symbolic(n, _p(Ap), _p(Ai), _p(parent), _p(post), _p(cc), _p(Lp), C.byref(fl))
    return dict(parent=parent, post=post, colcount=cc, Lp=Lp, nnz_L=int(nz), flops=fl.value,
                depth=etree_depth(parent))


def etree_depth(parent):
    """Number of depth levels of the etree forest (compute_levels, src/chol.cpp:7-40)."""
    parent = np.asarray(parent)
    n = len(parent)
    depth = np.full(n, -1, dtype=np.int64)
    for j in range(n):
        if depth[j] != -1:
            continue
        path = []
        v = j
        while v != -1 and depth[v] == -1:
            path.append(v)
            v = parent[v]
        base = 0 if v == -1 else depth[v] + 1
        for u in reversed(path):
            depth[u] = base
            base += 1
    return int(depth.max() + 1) if n else 0


def chol(A, faithful_workspace=False):
    """Up-looking chol() restatement.  Returns (status, Lp, Li, Lx).

    status = 0 on success, k+1 for the first non-positive pivot of row k
    ("A is not positive definite.", chol.hpp:849-850).
    """
    Ap, Ai, Ax = _csc(A)
    n = len(Ap) - 1
    sy = symbolic(A)
    Lp = sy["Lp"]
    nz = sy["nnz_L"]
    Li = np.zeros(max(nz, 1), dtype=np.int32)
    Lx = np.zeros(max(nz, 1), dtype=np.float64)
    st = lib().oracle_chol(n, _p(Ap), _p(Ai), _p(Ax), _p(sy["parent"]), _p(Lp), _p(Li), _p(Lx),
                           1 if faithful_workspace else 0)
    return int(st), Lp, Li[:nz], Lx[:nz]


def time_chol(A, reps=5, faithful_workspace=True):
    """Best-of-`reps` seconds of the whole reference chol() call (symbolic + numeric),
    timed in C.  Returns (status, seconds)."""
    Ap, Ai, Ax = _csc(A)
    n = len(Ap) - 1
    best = C.c_double()
    st = lib().oracle_time_chol(n, _p(Ap), _p(Ai), _p(Ax), reps, 1 if faithful_workspace else 0, C.byref(best))
    return int(st), best.value


def schol(A):
    Ap, Ai, _ = _csc(A)
    n = len(Ap) - 1
    sy = symbolic(A)
    Li = np.zeros(max(sy["nnz_L"], 1), dtype=np.int32)
    lib().oracle_schol(n, _p(Ap), _p(Ai), _p(sy["parent"]), _p(sy["Lp"]), _p(Li))
    return sy["Lp"], Li[: sy["nnz_L"]], sy["parent"]
