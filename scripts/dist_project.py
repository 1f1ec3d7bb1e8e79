#!/usr/bin/env python3
"""Per-rank timing projection of the N-GPU plan on one GPU.

Each rank's part of the plan (its subtree fronts, split-front panels and CB blocks,
packing / unpacking of every comm step) runs alone on the device with the transfers
dropped (sc_numeric_create_dist_dry).  max over ranks is a lower bound of the N-GPU
step time (it leaves out transfer time and waiting on peers).

Communication term (host-only, from the plan's message list, sc_dist_schedule): per
comm step a rank's exchange with each peer runs on that pair's own xGMI link, so the
step takes max over peers of max(bytes sent, bytes received) / link_GBs plus a
per-message latency.  comm_ms = the sum over the rank's steps, i.e. every transfer
serialised behind the rank's compute (nothing overlapped): rank_ms + comm_ms is an
upper-bound projection, rank_ms alone the lower bound.

  python scripts/dist_project.py [--k 128] [--n 2,4,8] [--opt key=value ...]
  python scripts/dist_project.py --comm-only      (no GPU: the communication term alone)
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def comm_model(symb, n, link_gbs, msg_us):
    """Per rank: bytes sent / received and the serialised transfer time of its comm steps."""
    import numpy as np

    out = {"comm_ms": [], "sent_GB": [], "recv_GB": [], "steps": []}
    for r in range(n):
        step, peer, nb, snd = symb.dist_schedule(n, r)
        t = 0.0
        nsteps = 0
        for st in np.unique(step):
            sel = step == st
            link = {}
            for p, b, s in zip(peer[sel], nb[sel], snd[sel]):
                a = link.setdefault(int(p), [0, 0])
                a[0 if s else 1] += int(b)
            t += max(max(a) for a in link.values()) / (link_gbs * 1e9) * 1e3 + sel.sum() * msg_us * 1e-3
            nsteps += 1
        out["comm_ms"].append(round(t, 2))
        out["sent_GB"].append(round(float(nb[snd == 1].sum()) / 1e9, 3))
        out["recv_GB"].append(round(float(nb[snd == 0].sum()) / 1e9, 3))
        out["steps"].append(nsteps)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--n", default="2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--link-gbs", type=float, default=50.0,
                    help="achievable GB/s per direction of one xGMI link (spec 153 per link)")
    ap.add_argument("--msg-us", type=float, default=10.0, help="per-message latency, us")
    ap.add_argument("--comm-only", action="store_true")
    args = ap.parse_args()
    import sparsecholesky_amd as sc

    if args.comm_only:
        kw = {}
        for kv in args.opt:
            key, val = kv.split("=", 1)
            kw[key] = int(val)
        symb = sc.Symbolic(sc.laplacian3d(args.k), **kw)
        for n in [int(x) for x in args.n.split(",")]:
            cm = comm_model(symb, n, args.link_gbs, args.msg_us)
            print(json.dumps({"k": args.k, "n": n, "opts": kw, "link_GBs": args.link_gbs, **cm}), flush=True)
        return
    import torch

    kw = {}
    for kv in args.opt:
        key, val = kv.split("=", 1)
        kw[key] = int(val)
    A = sc.laplacian3d(args.k)
    symb = sc.Symbolic(A, **kw)
    F = symb.stats()["flops"]
    d_Ax = torch.from_numpy(A.x).to("cuda:0")
    for n in [int(x) for x in args.n.split(",")]:
        info = symb.dist_plan_info(n)
        _, work = symb.owner_map(n)
        per = []
        for r in range(n):
            num = sc.Numeric(symb, device=0, rank=r, nranks=n, transport="dry")
            num.factor_device(d_Ax.data_ptr(), sync=True)
            best = None
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                num.factor_device(d_Ax.data_ptr(), sync=False)
                num.status()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) * 1e3
                best = dt if best is None else min(best, dt)
            per.append(round(best, 2))
            del num
            gc.collect()
            print(f"  n={n} rank {r}: {best:.1f} ms", flush=True)
        mx = max(per)
        cm = comm_model(symb, n, args.link_gbs, args.msg_us)
        with_comm = [round(a + b, 2) for a, b in zip(per, cm["comm_ms"])]
        print(json.dumps({"k": args.k, "n": n, "opts": kw, "rank_ms": per, "max_rank_ms": mx,
                          "projected_gflops_upper": round(F / (mx * 1e-3) / 1e9, 1),
                          "rank_ms_with_comm_serial": with_comm, "max_rank_ms_with_comm_serial": max(with_comm),
                          "projected_gflops_with_comm_serial": round(F / (max(with_comm) * 1e-3) / 1e9, 1),
                          "link_GBs": args.link_gbs, **cm,
                          "work_share": [round(float(x) / float(work.sum()), 3) for x in work],
                          "comm_steps": info["n_steps"], "messages": info["n_msgs"]}), flush=True)


if __name__ == "__main__":
    main()
