"""Top-level panel chain of the 128^3 factorization: per-kind launch durations
(eager, HIP events) with and without lookahead.  Usage: rootsteps.py [k] [opts-json]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import sparsecholesky_amd as sc  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
extra = json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}
A = sc.laplacian3d(k)
names = ["small", "asm", "potrf", "trsm", "panel", "cb", "comm", "rec", "wait"]
for la in (0, 1):
    S = sc.Symbolic(A, lookahead=la, **extra)
    num = sc.Numeric(S, device=0)
    dx = torch.from_numpy(A.x).cuda()
    num.factor_device(dx.data_ptr())
    num.set_profile(1)
    num.factor_device(dx.data_ptr())
    t = num.level_times()
    tr = num.launch_trace()
    print(f"lookahead={la}: total {t.sum():.1f} ms")
    for L in range(len(t) - 3, len(t)):
        parts = []
        for kk in range(6):
            for s in (0, 1):
                sel = (tr["level"] == L) & (tr["kind"] == kk) & (tr["stream"] == s)
                if sel.any():
                    ms = tr["ms"][sel]
                    fl = tr["flops"][sel].sum()
                    parts.append(f"{names[kk]}/s{s} n={sel.sum()} sum={ms.sum():.2f} "
                                 f"avg={1e3 * ms.mean():.1f}us med={1e3 * np.median(ms):.1f}us "
                                 f"{fl / max(ms.sum(), 1e-9) / 1e9:.1f}TF/s")
        print(f"  level {L} ({t[L]:.1f} ms): " + "; ".join(parts))
    del num
