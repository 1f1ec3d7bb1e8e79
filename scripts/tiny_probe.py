#!/usr/bin/env python3
"""Repeated bcsstk01 factorizations (for a kernel trace of the tiny launch): 200 eager
factorizations through one handle, then a solve whose backward error checks the factor
(the package may be a variant build).  Usage: tiny_probe.py [package dir]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else ROOT)
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

A = sc.load_matrix_market_to_csc(os.path.join(ROOT, "tests/golden/bcsstk01.mtx"))
num = sc.Numeric(sc.Symbolic(A, use_graph=0))
for _ in range(200):
    assert num.factor(A.x) == 0
n = A.size()
U = sp.csc_matrix((A.x, A.i, A.p), shape=(n, n))
U = sp.triu(U)
Af = U + sp.triu(U, 1).T
b = np.random.default_rng(3).standard_normal(n)
x = num.solve(b)
be = np.abs(Af @ x - b).max() / (abs(Af).sum(axis=1).max() * np.abs(x).max() + np.abs(b).max())
print(f"tiny probe ok {sc.__file__} backward error {be:.2e}")
assert be < 1e-13 or os.environ.get("TINY_NOCHECK")  # probe 1 factors nothing
