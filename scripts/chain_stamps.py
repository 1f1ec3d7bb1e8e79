"""Phase breakdown of the chain launch (runs of single small-front levels) of a small
config: shader-clock stamps per chained front (sc_debug_chain_stamps), eager."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "1138_bus"
A = sc.load_matrix_market_to_csc(os.path.join(ROOT, "tests", "golden", name + ".mtx"))
num = sc.Numeric(sc.Symbolic(A, use_graph=0))
L = sc.lib()
cnt = L.sc_debug_chain_stamps(num.h, 1, None, 0)
d = torch.tensor(A.x, device="cuda:0", dtype=torch.float64)
for _ in range(3):
    assert num.factor_device(d.data_ptr(), sync=True) == 0
st = np.zeros(cnt, dtype=np.uint64)
L.sc_debug_chain_stamps(num.h, 0, st.ctypes.data, cnt)
st = st.reshape(-1, 8).astype(np.int64)
ph = np.diff(st[:, :5], axis=1)  # load, assemble next, steps, panel+cb
tot = st[-1, 4] - st[0, 0]
print(f"{name}: {len(st)} chained fronts, {tot} clocks total, {tot / len(st):.0f} per front")
for k, nm in enumerate(["load", "asm next", "steps", "panel+cb"]):
    print(f"  {nm:9s} mean {ph[:, k].mean():8.0f}  max {ph[:, k].max():8d}")
gaps = st[1:, 0] - st[:-1, 4]
print(f"  between fronts mean {gaps.mean():.0f}")
