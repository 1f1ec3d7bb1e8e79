"""Panel-update launches of one eager 128^3 factorization (HIP events per launch):
per level and stream, launches, flops, summed ms and TF/s; plus the per-level wall
time (main stream) and chain kernels.  Eager timing serialises nothing: the events
bracket each launch on its own stream."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[2:]}  # e.g. lookahead=0
A = sc.laplacian3d(k)
num = sc.Numeric(sc.Symbolic(A, use_graph=0, **opts))
d = torch.from_numpy(A.x).to("cuda:0")
num.set_profile(1)
for _ in range(2):
    assert num.factor_device(d.data_ptr(), sync=True) == 0
t = num.launch_trace()
lt = num.level_times()
names = {0: "small", 1: "asm", 2: "potrf", 3: "trsm", 4: "panel", 5: "cb", 6: "comm"}
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for kind, lev, st, ms, fl in zip(t["kind"], t["level"], t["stream"], t["ms"], t["flops"]):
    key = (int(lev), names.get(int(kind), str(kind)), int(st))
    a = agg[key]
    a[0] += 1
    a[1] += ms
    a[2] += fl
for lev in range(len(lt)):
    rows = [(key, v) for key, v in agg.items() if key[0] == lev]
    if not rows:
        continue
    print(f"level {lev}: wall {lt[lev]:.2f} ms")
    for key, (n, ms, fl) in sorted(rows, key=lambda kv: -kv[1][1]):
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 and fl > 0 else 0.0
        print(f"   {key[1]:6s} strm {key[2]}  launches {n:5d}  {ms:8.2f} ms  {fl:.3e} fl  {tf:6.1f} TF/s")
