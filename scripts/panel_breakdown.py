"""Panel-update (and CB) SYRK launches of a profiled 128^3 factorization, bucketed by
per-launch flops: where the panel-update time goes (stream 0 = chain, 1 = lookahead)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import sparsecholesky_amd as sc

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
A = sc.laplacian3d(k)
S = sc.Symbolic(A)
num = sc.Numeric(S, device=0)
dx = torch.from_numpy(A.x).cuda()
num.factor_device(dx.data_ptr())
num.set_profile(True)
num.factor_device(dx.data_ptr())
tr = num.launch_trace()
for kind, name in ((4, "panel"), (5, "cb"), (2, "potrf"), (3, "trsm")):
    for st in (0, 1):
        sel = (tr["kind"] == kind) & (tr["stream"] == st)
        if not sel.any():
            continue
        fl, ms = tr["flops"][sel], tr["ms"][sel]
        print(f"{name} stream {st}: launches {sel.sum()}, {ms.sum():.1f} ms, {fl.sum()/1e12:.3f} TF, "
              f"{fl.sum()/(ms.sum()*1e-3)/1e12 if ms.sum() > 0 else 0:.1f} TF/s")
        if kind in (4, 5):
            edges = [0, 1e8, 1e9, 1e10, 1e11, 1e12, 1e14]
            for a, b in zip(edges[:-1], edges[1:]):
                s2 = (fl >= a) & (fl < b)
                if s2.any():
                    print(f"   flops [{a:.0e},{b:.0e}): n={s2.sum():5d} {ms[s2].sum():8.1f} ms {fl[s2].sum()/(ms[s2].sum()*1e-3)/1e12:6.1f} TF/s"
                          f"  avg {ms[s2].mean()*1e3:8.1f} us")
