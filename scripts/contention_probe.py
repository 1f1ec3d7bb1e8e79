"""Dispatch-contention probe (sc_debug_contention): how long a chain of small
critical-path launches (fused POTRF + TRSM, 4 or 64 workgroups each) takes while a
big panel-update SYRK fills the GPU from another stream, and whether CU-masking the
big launch's stream (eager or graph-replayed) gives the chain its slots back.

  python scripts/contention_probe.py > gpurun_out/contention.jsonl
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparsecholesky_amd as sc  # noqa: E402


def probe(M, K, rows, nchain, mode, stride):
    out = (C.c_double * 8)()
    rc = sc.lib().sc_debug_contention(M, K, rows, nchain, mode, stride, out)
    return rc, list(out)


def main():
    M, K, nchain = 12288, 1024, 32
    cases = [(0, 0), (1, 32), (1, 16), (1, 8), (2, 0), (3, 32), (3, 8), (4, 0), (6, 0), (7, 32), (7, 8)]
    for rows in (1024, 4096, 16384):
        for mode, stride in cases:
            rc, o = probe(M, K, rows, nchain, mode, stride)
            rec = dict(M=M, K=K, chain_rows=rows, nchain=nchain, mode=mode, mask_stride=stride, rc=rc,
                       chain_alone_ms=round(o[0], 3), hog_alone_ms=round(o[1], 3), chain_under_hog_ms=round(o[2], 3),
                       hog_under_chain_ms=round(o[3], 3), both_ms=round(o[4], 3), hog_cus=int(o[5]))
            print(json.dumps(rec), flush=True)
            if rc != 0:
                raise SystemExit(f"probe failed rc={rc}")


if __name__ == "__main__":
    main()
