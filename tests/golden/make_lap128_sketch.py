"""Generates tests/golden/lap128_sketch.npz (committed): the oracle's 128^3 factor, sketched.

Runs the oracle (oracle/refchol.c ``oracle_chol``, the restatement of the reference's
up-looking chol(), include/chol.hpp:749-863; hoisted O(n) workspace, 1 thread) once on
the 128^3 7-point Laplacian in SURVEY Appendix B's geometric ND order (the bench
workload, BASELINE configs[3]), then reduces L with tests/lap128_sketch.py:
per-chunk Frobenius norms, per-1024-column norms over the last 262,144 columns,
Gaussian sketches L(:, J)^T r_s there, and bilinear sketches u^T L(:, chunk) v per
chunk.  tests/test_gpu_parity.py::test_lap128_oracle_sketch compares the GPU
factor's sketch with it.

Needs ~35 GB of RAM (nnz(L) = 2.83e9: int32 rows + fp64 values) and hours of one core.
Run (build container, in the background):
    python -u tests/golden/make_lap128_sketch.py > tests/golden/make_lap128_sketch.log 2>&1
"""
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import oracle  # noqa: E402
import sparsecholesky_amd as sc  # noqa: E402  (input generator only: sc_laplacian3d)
import lap128_sketch as ls  # noqa: E402


def main():
    global ls
    t0 = time.time()
    A = sc.laplacian3d(ls.K)
    digest = ls.input_digest(A)
    print(f"A: n {A.size()}, nnz(upper) {len(A.i)}, digest {digest}", flush=True)
    sy = oracle.symbolic(A)
    print(f"symbolic: nnz(L) {sy['nnz_L']}, F {sy['flops']:.6e}, {time.time() - t0:.1f} s", flush=True)

    done = C.c_int64.in_dll(oracle.lib(), "oracle_chol_rows_done")
    stop = threading.Event()

    def monitor():
        t1 = time.time()
        while not stop.wait(300):
            k = done.value
            print(f"  oracle rows {k} / {ls.N} ({100.0 * k / ls.N:.2f}%), {time.time() - t1:.0f} s", flush=True)

    th = threading.Thread(target=monitor, daemon=True)
    th.start()
    t1 = time.time()
    st, Lp, Li, Lx = oracle.chol(A)
    t_chol = time.time() - t1
    stop.set()
    print(f"oracle chol: status {st}, {t_chol:.0f} s, {sy['flops'] / t_chol / 1e9:.2f} GF/s", flush=True)
    assert st == 0

    # L took hours: if the reduction fails, keep it in memory and retry the reduction
    # (re-importing tests/lap128_sketch.py) whenever tests/golden/.retry_sketch appears.
    retry = os.path.join(HERE, ".retry_sketch")
    while True:
        try:
            acc = ls.Accumulator()
            for c0, c1 in ls.column_blocks(Lp):
                p0, p1 = int(Lp[c0]), int(Lp[c1])
                acc.add(c0, c1, Lp[c0:c1 + 1], Li[p0:p1], Lx[p0:p1])
            res = acc.result()
            break
        except Exception:
            import importlib
            import traceback
            traceback.print_exc()
            print(f"reduction failed; touch {retry} to retry", flush=True)
            while not os.path.exists(retry):
                time.sleep(30)
            os.remove(retry)
            ls = importlib.reload(ls)
    meta = dict(digest=digest, nnz_L=int(sy["nnz_L"]), flops=float(sy["flops"]), oracle_seconds=t_chol,
                oracle_status=int(st), seed=ls.SEED, fro=float(np.sqrt(res["chunk_sumsq"].sum())))
    out = os.path.join(HERE, "lap128_sketch.npz")
    np.savez(out, meta=np.array(json.dumps(meta)), **res)
    print(f"wrote {out} ({os.path.getsize(out) / 1e6:.1f} MB): {json.dumps(meta)}", flush=True)
    print(f"total {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
