"""Where a persistent slab chain (panel_psk) spends its time: one eager factorization
with the kernel's debug stamps on (sc_debug_psk_stamps), summarised per launch (one
slab of one level): dispatch spread of the workgroups, the diagonal-block chain (owner
of step j: L11 ready -> owner of step j + 1: L11 ready), and per workgroup the time in
waits, TRSM and inner updates.

  python scripts/psk_stamps.py [k] [key=value ...]     (e.g. 128 lookahead=0)
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sparsecholesky_amd as sc  # noqa: E402

NS = 1 + 3 * 16


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[2:]}
    opts.setdefault("panel_psk", 1)
    A = sc.laplacian3d(k)
    num = sc.Numeric(sc.Symbolic(A, use_graph=0, **opts))
    d = torch.from_numpy(A.x).to("cuda:0")
    assert num.factor_device(d.data_ptr(), sync=True) == 0
    L = sc.lib()
    nwg = L.sc_debug_psk_stamps(num.h, 1, None, None, 0)
    assert num.factor_device(d.data_ptr(), sync=True) == 0
    info = np.zeros(8 * nwg, dtype=np.int32)
    st = np.zeros(NS * nwg, dtype=np.uint64)
    L.sc_debug_psk_stamps(num.h, 0, info.ctypes.data_as(C.c_void_p), st.ctypes.data_as(C.c_void_p), NS * nwg)
    info = info.reshape(nwg, 8)
    st = st.reshape(nwg, NS).astype(np.int64)
    out = []
    for seq in np.unique(info[:, 0]):
        sel = np.flatnonzero(info[:, 0] == seq)
        I, T = info[sel], st[sel]
        t0 = T[:, 0].min()
        us = lambda x: (x - t0) * 0.01  # 100 MHz ticks -> us
        TR = int(I[0, 7])
        fronts = np.unique(I[:, 2])
        rec = dict(launch=int(seq), level=int(I[0, 1]), fronts=len(fronts), wgs=len(sel),
                   slab=[int(I[0, 4]), int(I[0, 5])], rows_per_wg=TR)
        last = np.where(T > 0, T, 0).max()
        rec["span_us"] = round(float((last - t0) * 0.01), 1)
        rec["start_spread_us"] = round(float(us(T[:, 0].max())), 1)
        # the chain of the first front: owner of step j = row block 64 j / TR
        f0 = fronts[0]
        nsteps = (int(I[0, 5]) - int(I[0, 4])) // 64
        l11 = []
        for j in range(min(nsteps, 16)):
            rb = 64 * j // TR
            w = np.flatnonzero((I[:, 2] == f0) & (I[:, 3] == rb))
            if len(w):
                l11.append(float(us(T[w[0], 1 + 3 * j])))
        rec["chain_l11_ready_us"] = [round(x, 1) for x in l11]
        rec["chain_step_us"] = round(float(np.mean(np.diff(l11))), 1) if len(l11) > 1 else None
        # per workgroup phases over the steps it ran (stamps > 0)
        waits, trsm, upd = [], [], []
        for row in T:
            prev = row[0]
            for j in range(16):
                a, b, c = row[1 + 3 * j], row[2 + 3 * j], row[3 + 3 * j]
                if a == 0:
                    break
                waits.append(a - prev)
                if b:
                    trsm.append(b - a)
                if c and b:
                    upd.append(c - b)
                prev = c if c else (b if b else a)
        rec["avg_wait_us"] = round(float(np.mean(waits)) * 0.01, 2) if waits else None
        rec["avg_trsm_us"] = round(float(np.mean(trsm)) * 0.01, 2) if trsm else None
        rec["avg_update_us"] = round(float(np.mean(upd)) * 0.01, 2) if upd else None
        busy = [(r[r > 0].max() - r[0]) * 0.01 for r in T]
        rec["wg_life_us_mean_max"] = [round(float(np.mean(busy)), 1), round(float(np.max(busy)), 1)]
        out.append(rec)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
