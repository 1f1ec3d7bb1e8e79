"""BK A/B for the CB SYRK kernel on random data (sc_debug_bench which = 1 / 6 / 7:
BK = 16 (default) / 8 / 32), 128x128 tiles, M x M lower triangle, K deep."""
import ctypes as C
import sys

sys.path.insert(0, "/root/repo")
import sparsecholesky_amd as sc  # noqa: E402

L = sc.lib()
t = C.c_double()
for M, K in ((16384, 4096), (16384, 1024), (8192, 2048), (4096, 1024)):
    row = []
    for which, bk in ((1, 16), (6, 8), (7, 32)):
        L.sc_debug_bench(which, M, K, 5, 128, C.byref(t))
        row.append(f"BK{bk} {t.value:6.2f}")
    print(f"syrk128 M={M} K={K}: " + "  ".join(row) + " TF/s", flush=True)
