"""SYRK tile instances on random data (sc_debug_bench which=1): the 8-wave 128 x 128
tile (arg 128, the default CB instance), the 4-wave 128 x 128 tile (arg 129: 64 x 64
per wave) and the 64 x 64 tile (arg 64); TFLOP/s of M x M triangles, K deep.

  python scripts/tile_probe.py > gpurun_out/tile_probe.jsonl
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparsecholesky_amd as sc  # noqa: E402


def main():
    L = sc.lib()
    for M, K in ((16384, 4096), (16384, 1024), (8192, 8192), (4096, 2048)):
        for rep in range(2):
            for arg in (128, 129, 64):
                t = C.c_double()
                rc = L.sc_debug_bench(1, M, K, 3, arg, C.byref(t))
                print(json.dumps(dict(M=M, K=K, tile=arg, rep=rep, rc=rc, tflops=round(t.value, 2))), flush=True)


if __name__ == "__main__":
    main()
