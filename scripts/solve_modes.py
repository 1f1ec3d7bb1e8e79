"""128^3 solve time, graph replay vs direct launches (sc_debug_solve_eager)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
A = sc.laplacian3d(k)
num = sc.Numeric(sc.Symbolic(A, use_graph=1))
d = torch.from_numpy(A.x).to("cuda:0")
assert num.factor_device(d.data_ptr(), sync=True) == 0
b = torch.ones(A.size(), dtype=torch.float64, device="cuda:0")
x = torch.empty_like(b)
torch.cuda.synchronize()
for eager in (0, 1, 0):
    sc.lib().sc_debug_solve_eager(num.h, eager)
    num.solve_device(b.data_ptr(), x.data_ptr())
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        num.solve_device(b.data_ptr(), x.data_ptr())
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"k={k} eager={eager}: best {min(ts):.2f} ms", flush=True)
