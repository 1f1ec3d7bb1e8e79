"""Kernel trace of the small configs (run under rocprofv3 --kernel-trace): a few
eager factorizations of bcsstk01 and 1138_bus."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

for name in sys.argv[1:] or ["1138_bus"]:
    A = sc.load_matrix_market_to_csc(os.path.join(ROOT, "tests", "golden", name + ".mtx"))
    num = sc.Numeric(sc.Symbolic(A, use_graph=0))
    d = torch.tensor(A.x, device="cuda:0", dtype=torch.float64)
    for _ in range(5):
        assert num.factor_device(d.data_ptr(), sync=True) == 0
    torch.cuda.synchronize()
