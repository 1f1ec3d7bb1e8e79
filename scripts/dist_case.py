#!/usr/bin/env python3
"""One emulated multi-rank factorization against the same package's single-GPU factor
(bisecting a partitioned-plan parity failure across builds).
  dist_case.py PKGDIR K NRANKS [key=value ...]   (options also applied to the single-GPU run)"""
import os
import sys

sys.path.insert(0, os.path.abspath(sys.argv[1]))
import numpy as np  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

k, nranks = int(sys.argv[2]), int(sys.argv[3])
opts = {}
for kv in sys.argv[4:]:
    a, b = kv.split("=")
    opts[a] = int(b)
A = sc.laplacian3d(k)
base = dict(panel_nb_outer=128, dist_cbb=64, small_front_max=32)
base.update(opts)
s = sc.Symbolic(A, **base)
one = sc.Numeric(s)
assert one.factor(A.x) == 0
_, L0 = one.export()
v = sc.Numeric(s, nranks=nranks, virtual=True)
for _ in range(2):
    assert v.factor(A.x) == 0
_, L1 = v.export()
err = float(np.linalg.norm(L1.x - L0.x) / np.linalg.norm(L0.x))
print(f"{sys.argv[1]} k={k} n={nranks} {opts}: rel diff vs single GPU {err:.3e}", flush=True)
