#!/usr/bin/env python3
"""Rank `rank`'s part of an n-GPU factorization alone on this GPU (dry transport: comm
steps pack and unpack, nothing moves), for kernel traces and counter passes of one
rank's schedule.

  python3 scripts/dry_rank.py [--k 128] [--n 8] [--rank 0] [--steps 3] [--opt key=value ...]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    import torch

    import sparsecholesky_amd as sc

    kw = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.opt}
    A = sc.laplacian3d(a.k)
    s = sc.Symbolic(A, **kw)
    num = sc.Numeric(s, device=0, rank=a.rank, nranks=a.n, transport="dry")
    d = torch.from_numpy(A.x).to("cuda:0")
    for i in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        num.factor_device(d.data_ptr(), sync=False)
        num.status()
        torch.cuda.synchronize()
        print(f"k={a.k} n={a.n} rank {a.rank} step {i}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
