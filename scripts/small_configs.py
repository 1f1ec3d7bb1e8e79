#!/usr/bin/env python3
"""GPU factorization time of the small configs (Python-level: ctypes call + torch sync
included; *_c: timed in C, launch to status read-back) (BASELINE configs[1..2]: bcsstk01, 1138_bus;
plus lap 16^3 / 32^3), eager and hipGraph replay, next to the oracle restatement of the
reference chol() on one host core.  Prints one JSON line per matrix."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
import sparsecholesky_amd as sc  # noqa: E402

if os.environ.get("SC_LIB"):  # A/B: another build of the library
    sc.LIB_PATH = os.environ["SC_LIB"]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best * 1e3


cases = [("bcsstk01", sc.load_matrix_market_to_csc(os.path.join(ROOT, "tests/golden/bcsstk01.mtx"))),
         ("1138_bus", sc.load_matrix_market_to_csc(os.path.join(ROOT, "tests/golden/1138_bus.mtx"))),
         ("lap16_nd", sc.laplacian3d(16)), ("lap32_nd", sc.laplacian3d(32))]
for name, A in cases:
    out = {"matrix": name, "n": A.size()}
    for graph in (0, 1):
        s = sc.Symbolic(A, use_graph=graph)
        num = sc.Numeric(s, device=0)
        d = torch.from_numpy(A.x).to("cuda:0")
        ms = timeit(lambda: num.factor_device(d.data_ptr(), sync=True), 20)
        out["gpu_ms_graph" if graph else "gpu_ms_eager"] = round(ms, 3)
        best = ctypes.c_double()
        sc.lib().sc_debug_time_factor(num.h, ctypes.c_void_p(d.data_ptr()), 50, ctypes.byref(best))
        out["gpu_ms_c_graph" if graph else "gpu_ms_c_eager"] = round(best.value, 4)
        out["levels"] = s.stats()["n_levels"]
        out["flops"] = s.flops
    t = []
    for _ in range(5):
        t0 = time.perf_counter()
        st, *_ = oracle.chol(A, faithful_workspace=True)
        t.append((time.perf_counter() - t0) * 1e3)
    out["cpu_ref_restatement_ms_1core"] = round(min(t), 3)
    st, sec = oracle.time_chol(A, reps=20, faithful_workspace=True)
    out["cpu_ref_restatement_ms_1core_c"] = round(sec * 1e3, 4)
    st, Lp, Li, Lx = oracle.chol(A)
    r = sc.chol(A)
    out["rel_fro_vs_oracle"] = float(np.linalg.norm(r.value().x - Lx) / np.linalg.norm(Lx))
    print(json.dumps(out), flush=True)
