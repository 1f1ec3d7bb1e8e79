"""Kernel microbenchmarks on the GPU box: fp64 MFMA ceiling and the SYRK kernel (random data)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparsecholesky_amd as sc  # noqa: E402


def run(which, M, K, reps, arg):
    t = C.c_double()
    rc = sc.lib().sc_debug_bench(which, M, K, reps, arg, C.byref(t))
    return round(t.value, 2) if rc == 0 else f"rc={rc}"


def panel():
    """POTRF of one 64 x 64 block and the fused POTRF + TRSM of an M x 64 panel, us per launch."""
    out = {}
    for M in (2048, 16448):
        out[f"M={M} potrf us"] = run(2, M, 1, 50, 0)
        out[f"M={M} potrf+trsm us"] = run(3, M, 1, 50, 0)
    for k, v in out.items():
        print(f"{k:45s} {v}")
    print(json.dumps(out))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "panel":
        return panel()
    out = {}
    for blocks in (1024, 2048):
        out[f"peak blocks={blocks} nacc=8"] = run(0, blocks, 20000, 3, 8)
    for M, K in ((4096, 256), (4096, 1024), (8192, 2048), (16384, 4096), (16384, 8192)):
        for tile in (64, 128, 1128):
            out[f"syrk M={M} K={K} tile={tile}"] = run(1, M, K, 3, tile)
    for k, v in out.items():
        print(f"{k:45s} {v}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
