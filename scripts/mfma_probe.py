"""Measured fp64 MFMA peak (register-only probe, independent accumulator chains) and
the SYRK kernel on random operands.  --probe-only: just the probe (counter pass)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparsecholesky_amd as sc  # noqa: E402

L = sc.lib()
t = C.c_double()
for nacc in ((8,) if "--probe-only" in sys.argv else (4, 8, 16)):
    L.sc_debug_bench(0, 1024, 20000, 3, nacc, C.byref(t))
    print("mfma peak probe nacc", nacc, round(t.value, 2), "TF/s", flush=True)
if "--probe-only" not in sys.argv:
    for M, K in ((16384, 8192), (16384, 2048), (8192, 1024)):
        L.sc_debug_bench(1, M, K, 3, 128, C.byref(t))
        print("syrk128", M, K, round(t.value, 2), "TF/s", flush=True)
