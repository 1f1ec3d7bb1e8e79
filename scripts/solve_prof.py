#!/usr/bin/env python3
"""Factor lap k^3 and run the GPU solve a few times (for rocprofv3 kernel stats)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
A = sc.laplacian3d(k)
s = sc.Symbolic(A)
num = sc.Numeric(s, device=0)
d_Ax = torch.from_numpy(A.x).to("cuda:0")
assert num.factor_device(d_Ax.data_ptr(), sync=True) == 0
d_b = torch.ones(A.size(), dtype=torch.float64, device="cuda:0")
d_x = torch.empty_like(d_b)
for i in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    num.solve_device(d_b.data_ptr(), d_x.data_ptr())
    print(f"solve {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
