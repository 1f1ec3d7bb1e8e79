"""General-product kernel (gemm_mfma_kernel, TAG 2) against the SYRK kernel on the
panel shapes (M rows x 1024 columns, K = 1024): plain store, in-place subtract,
triangular B (the tall solve's K trim), and the TAG 0 SYRK on the same trapezoid.

  python scripts/gemm_probe.py > gpurun_out/gemm_probe.jsonl
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparsecholesky_amd as sc  # noqa: E402


def main():
    for M in (12288, 20480):
        for K in (512, 1024):
            for arg, what in [(0, "store"), (1, "subtract_in_place"), (2, "store_ktri"), (4, "syrk_trapezoid")]:
                out = C.c_double()
                rc = sc.lib().sc_debug_bench(7, M, K, 5, arg, C.byref(out))
                print(json.dumps(dict(M=M, N=K, K=K, kind=what, rc=rc, tflops=round(out.value, 2))), flush=True)
                if rc != 0:
                    raise SystemExit(rc)


if __name__ == "__main__":
    main()
