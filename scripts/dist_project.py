#!/usr/bin/env python3
"""Per-rank timing projection of the N-GPU plan on one GPU.

Each rank's part of the plan (its subtree fronts, split-front panels and CB blocks,
packing / unpacking of every comm step) runs alone on the device with the transfers
dropped (sc_numeric_create_dist_dry).  max over ranks is a lower bound of the N-GPU
step time (it leaves out transfer time and waiting on peers).

  python scripts/dist_project.py [--k 128] [--n 2,4,8] [--opt key=value ...]
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--n", default="2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--opt", action="append", default=[])
    args = ap.parse_args()
    import torch
    import sparsecholesky_amd as sc

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
        print(json.dumps({"k": args.k, "n": n, "opts": kw, "rank_ms": per, "max_rank_ms": mx,
                          "projected_gflops_upper": round(F / (mx * 1e-3) / 1e9, 1),
                          "work_share": [round(float(x) / float(work.sum()), 3) for x in work],
                          "comm_steps": info["n_steps"], "messages": info["n_msgs"]}), flush=True)


if __name__ == "__main__":
    main()
