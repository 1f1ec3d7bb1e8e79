"""Per-level time vs executed flops of the 128^3 factorization (profiled run)."""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import sparsecholesky_amd as sc

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
extra = json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}
A = sc.laplacian3d(k)
S = sc.Symbolic(A, **extra)
d = S.supernodes()
m = d["m"].astype(float); w = d["w"].astype(float); lev = d["level"]
f = w * m * m - m * w * (w - 1) + (w - 1) * w * (2 * w - 1) / 6.0
num = sc.Numeric(S, device=0)
dx = torch.from_numpy(A.x).cuda()
num.factor_device(dx.data_ptr())
num.set_profile(True)
num.factor_device(dx.data_ptr())
t = num.level_times()
tot = t.sum()
print(f"total level time {tot:.1f} ms, phases {num.timing().round(1).tolist()}")
for L in range(len(t)):
    sel = lev == L
    fl = f[sel].sum()
    big = np.sort(w[sel])[::-1][:3].astype(int).tolist()
    print(f"level {L:2d}: fronts {sel.sum():7d}  maxw {big}  maxm {int(m[sel].max()):6d}  exec {fl/1e12:7.3f} TF  time {t[L]:8.2f} ms  rate {fl/(t[L]*1e-3)/1e12 if t[L]>0 else 0:6.2f} TF/s")

tr = num.launch_trace()
names = ["small", "asm", "potrf", "trsm", "panel", "cb", "comm"]
print("per level kernel ms (stream0 | stream1):")
for L in range(len(t)):
    row = []
    for kk in range(6):
        sel0 = (tr["level"] == L) & (tr["kind"] == kk) & (tr["stream"] == 0)
        sel1 = (tr["level"] == L) & (tr["kind"] == kk) & (tr["stream"] == 1)
        a, b = tr["ms"][sel0].sum(), tr["ms"][sel1].sum()
        if a > 0 or b > 0:
            nlaunch = int(sel0.sum() + sel1.sum())
            row.append(f"{names[kk]} {a:.1f}" + (f"|{b:.1f}" if b > 0 else "") + f" (n={nlaunch})")
    print(f"  level {L:2d}: " + ", ".join(row))
