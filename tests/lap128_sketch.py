"""Compact parity sketch of a 128^3 Laplacian factor (TEST INFRASTRUCTURE).

The whole 128^3 factor L (n = 2,097,152, nnz(L) = 2.83e9, 34 GB) cannot be a
fixture, so the oracle's L (oracle/refchol.c, reference chol.hpp:749-863) is
reduced once, by tests/golden/make_lap128_sketch.py, to quantities that are
linear or quadratic in L and that any L can be reduced to the same way:

  * ``chunk_sumsq[c]``  = ||L(:, c*65536 : (c+1)*65536)||_F^2 for all 32 chunks;
  * ``group_sumsq[g]``  = ||L(:, J0 + g*1024 : J0 + (g+1)*1024)||_F^2 over
    J = [n - 262144, n) (every top-3-level separator and the root; ~97% of F);
  * ``Y[s]``            = L(:, J)^T r_s for 4 seeded Gaussian vectors r_s;
  * ``B[c, t]``         = u_t^T L(:, chunk c) v_t for 16 seeded Gaussian pairs.

For a Gaussian r, E ||X^T r||^2 = ||X||_F^2, so ||Y_G - Y_O|| estimates
||G - O||_F over J (4 samples), and (B_G - B_O)[c, :] estimates it per chunk
(16 samples) over the whole factor.  Column sums are formed per column in
entry order (scipy's CSR mat-vecs), so both sides round the same way.

Both the generator (oracle side) and the -m gpu test (GPU factor exported
through the C ABI, ``Numeric.export_cols``) use ``Accumulator``.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

K = 128
N = K ** 3
CHUNK = 65536
NCHUNK = N // CHUNK
J0 = N - 262144
GROUP = 1024
NGROUP = (N - J0) // GROUP
NY = 4
NB = 16
SEED = 20260518


def random_vectors():
    rng = np.random.default_rng(SEED)
    R = rng.standard_normal((N, NY + NB))  # r_s (columns 0..3) and u_t (4..19), row-major
    V = rng.standard_normal((NB, N))       # v_t
    return R, V


class Accumulator:
    """Feed column blocks [c0, c1) of L in increasing order (any block sizes)."""

    def __init__(self):
        self.R, self.V = random_vectors()
        self.chunk_sumsq = np.zeros(NCHUNK)
        self.group_sumsq = np.zeros(NGROUP)
        self.Y = np.zeros((NY, N - J0))
        self.B = np.zeros((NCHUNK, NB))
        self.next_col = 0
        self.nnz = 0

    def add(self, c0: int, c1: int, colptr: np.ndarray, ri: np.ndarray, rx: np.ndarray):
        assert c0 == self.next_col and c1 > c0
        colptr = np.asarray(colptr, dtype=np.int64)
        lp = (colptr - colptr[0]).astype(np.int32)
        assert len(lp) == c1 - c0 + 1 and int(lp[-1]) == len(rx) == len(ri)
        M = sp.csc_matrix((rx, np.asarray(ri, dtype=np.int32), lp), shape=(N, c1 - c0))
        S = np.asarray(M.T @ self.R)  # (c1 - c0) x 20, per column in entry order
        colsq = np.add.reduceat(rx * rx, lp[:-1]) if len(rx) else np.zeros(c1 - c0)
        cols = np.arange(c0, c1)
        np.add.at(self.chunk_sumsq, cols // CHUNK, colsq)
        inj = cols >= J0
        if inj.any():
            jj = cols[inj] - J0
            np.add.at(self.group_sumsq, jj // GROUP, colsq[inj])
            self.Y[:, jj] = S[inj, :NY].T
        prod = S[:, NY:] * self.V[:, c0:c1].T  # (c1 - c0) x 16
        for c in np.unique(cols // CHUNK):
            sel = (cols // CHUNK) == c
            self.B[c] += prod[sel].sum(axis=0)
        self.next_col = c1
        self.nnz += len(rx)

    def result(self) -> dict:
        assert self.next_col == N
        return dict(chunk_sumsq=self.chunk_sumsq, group_sumsq=self.group_sumsq, Y=self.Y, B=self.B,
                    nnz=np.int64(self.nnz))


def column_blocks(Lp: np.ndarray, max_entries: int = 100_000_000):
    """Column ranges [c0, c1) of at most ~max_entries entries, cut at chunk boundaries."""
    c0 = 0
    while c0 < N:
        cend = min(N, (c0 // CHUNK + 1) * CHUNK)
        target = Lp[c0] + max_entries
        c1 = int(np.searchsorted(Lp, target, side="right")) - 1
        c1 = max(c0 + 1, min(c1, cend))
        yield c0, c1
        c0 = c1


def input_digest(A) -> str:
    import hashlib
    h = hashlib.sha256()
    for a in (np.asarray(A.p, np.int64), np.asarray(A.i, np.int32), np.asarray(A.x, np.float64)):
        h.update(a.tobytes())
    return h.hexdigest()[:32]


def compare(got: dict, ref: dict) -> dict:
    """Error estimates of the GPU factor G against the oracle O (relative to O)."""
    cs_g, cs_o = np.sqrt(got["chunk_sumsq"]), np.sqrt(ref["chunk_sumsq"])
    gs_g, gs_o = np.sqrt(got["group_sumsq"]), np.sqrt(ref["group_sumsq"])
    dY = got["Y"] - ref["Y"]
    sketch_J = np.sqrt((dY * dY).sum() / (ref["Y"] * ref["Y"]).sum())
    dB = got["B"] - ref["B"]
    per_chunk = np.sqrt((dB * dB).mean(axis=1)) / cs_o
    return dict(chunk_norm_rel=float(np.max(np.abs(cs_g - cs_o) / cs_o)),
                group_norm_rel=float(np.max(np.abs(gs_g - gs_o) / gs_o)),
                sketch_J_rel_fro=float(sketch_J),
                sketch_chunk_rel_fro_max=float(per_chunk.max()),
                # the GPU export keeps the relaxed supernodes' explicit zeros (never equal)
                entries=(int(got["nnz"]), int(ref["nnz"])))
