import ctypes as C, sys
sys.path.insert(0, "/root/repo")
import sparsecholesky_amd as sc
L = sc.lib()
t = C.c_double()
for nacc in (4, 8, 16):
    L.sc_debug_bench(0, 1024, 20000, 3, nacc, C.byref(t)); print("mfma peak probe nacc", nacc, round(t.value, 2), "TF/s")
for M, K in ((16384, 8192), (16384, 2048), (8192, 1024)):
    L.sc_debug_bench(1, M, K, 3, 128, C.byref(t)); print("syrk128", M, K, round(t.value, 2), "TF/s")
