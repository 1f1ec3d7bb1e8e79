#!/usr/bin/env python3
"""bcsstk01 tiny-dense launches back to back (no host wait between them) next to the
synchronised ones, for a kernel trace: does the kernel's duration depend on the GPU
being kept busy (clock state) rather than on its instructions?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

A = sc.load_matrix_market_to_csc(os.path.join(ROOT, "tests/golden/bcsstk01.mtx"))
num = sc.Numeric(sc.Symbolic(A, use_graph=0))
d = torch.from_numpy(A.x).to("cuda:0")
for _ in range(100):  # synchronised: one factorization at a time
    assert num.factor_device(d.data_ptr(), sync=True) == 0
torch.cuda.synchronize()
for _ in range(400):  # back to back
    num.factor_device(d.data_ptr(), sync=False)
torch.cuda.synchronize()
assert num.factor_device(d.data_ptr(), sync=True) == 0
print("tiny b2b ok")
