"""Large-front assembly at 128^3: per level, the eager assembly launch time, its
algorithmic bytes (each front entry written once, each child CB entry read once;
packed lower triangles) and the rate, for a few tile/column kernel thresholds
(asm_tile_min_m); plus the graph-replayed factor time of each (best of 5)."""
import collections
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
thresholds = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [8192]
A = sc.laplacian3d(k)
d = torch.from_numpy(A.x).to("cuda:0")
sn = sc.Symbolic(A).supernodes()
m, w, par, lev = sn["m"].astype(np.float64), sn["w"], sn["parent"], sn["level"]
mb = m - w
small_max = 128  # capi.cpp default small_front_max
gb = collections.defaultdict(float)
for s in range(len(m)):
    if m[s] > small_max:
        gb[int(lev[s])] += m[s] * (m[s] + 1) / 2 * 8
for s in range(len(m)):
    p = par[s]
    if p >= 0 and m[p] > small_max:
        gb[int(lev[p])] += mb[s] * (mb[s] + 1) / 2 * 8
for thr in thresholds:
    sym = sc.Symbolic(A, use_graph=0, asm_tile_min_m=thr)
    num = sc.Numeric(sym)
    num.set_profile(1)
    for _ in range(2):
        assert num.factor_device(d.data_ptr(), sync=True) == 0
    t = num.launch_trace()
    agg = collections.defaultdict(float)
    for kind, lev, ms in zip(t["kind"], t["level"], t["ms"]):
        if int(kind) == 1:
            agg[int(lev)] += float(ms)
    del num
    num = sc.Numeric(sc.Symbolic(A, asm_tile_min_m=thr))
    best = ctypes.c_double(0)
    sc.lib().sc_debug_time_factor(num.h, ctypes.c_void_p(d.data_ptr()), 5, ctypes.byref(best))
    print(f"asm_tile_min_m {thr}: factor {best.value:.2f} ms, assembly {sum(agg.values()):.2f} ms "
          f"({sum(gb.values()) / 1e9:.1f} GB)", flush=True)
    for lv in sorted(agg):
        print(f"   level {lv:2d}  asm {agg[lv]:7.3f} ms  {gb[lv] / 1e9:6.2f} GB  "
              f"{gb[lv] / (agg[lv] * 1e-3) / 1e12:5.2f} TB/s", flush=True)
    del num
