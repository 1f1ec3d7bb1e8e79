#!/usr/bin/env python3
"""Numeric-factorization benchmark (BASELINE.json metric: fp64 GFLOP/s + wall time).

Workload: synthetic 3D 7-point Laplacian, k^3 grid (default k=128, BASELINE
configs[3]), deterministic geometric nested-dissection order.
A "step" is one complete numeric factorization (assembly, POTRF/TRSM, SYRK,
extend-add of every front) with A's values already resident in HBM.
GFLOP/s = F / step time, F = sum_j colcount[j]^2 (algorithmic).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--k 128]

N > 1 is launched by torch.distributed.run (one rank per GPU): the assembly
tree is partitioned by subtrees over the ranks; contribution blocks move over
RCCL only at subtree-merge fronts.
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X fp64 matrix (dense) spec, SURVEY.md Appendix C
HBM_PEAK_GBS = 8000.0


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(k=32, reps=2):
    """Reference chol() restatement (oracle, 1 thread, the reference's per-row O(n)
    workspace kept) on a bounded sample of the same workload family."""
    import oracle
    import sparsecholesky_amd as sc

    A = sc.laplacian3d(k)
    sy = oracle.symbolic(A)
    oracle.chol(sc.laplacian3d(8), faithful_workspace=True)  # load/warm
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        st, *_ = oracle.chol(A, faithful_workspace=True)
        dt = time.perf_counter() - t0
        assert st == 0
        best = dt if best is None else min(best, dt)
    return {
        "value": round(sy["flops"] / best / 1e9, 4),
        "unit": "GFLOP/s",
        "cores": 1,
        "kind": "port",
        "sample": f"lap3d {k}^3 ND (n={k**3}, F={sy['flops']:.4e}), oracle/refchol.c restatement of "
                  f"reference chol(), faithful per-row workspace, best of {reps}: {best:.3f} s; "
                  f"host: {cpu_model()}, nproc={os.cpu_count()}",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-k", type=int, default=32)
    ap.add_argument("--graph", type=int, default=0)
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()

    import torch
    import sparsecholesky_amd as sc

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 or world > 1:
        raise SystemExit("multi-GPU bench not available in this build")
    torch.cuda.set_device(local_rank)
    dev = local_rank

    t0 = time.perf_counter()
    A = sc.laplacian3d(args.k)
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    symb = sc.Symbolic(A, use_graph=args.graph)
    t_an = time.perf_counter() - t0
    st = symb.stats()
    F = st["flops"]
    t0 = time.perf_counter()
    num = sc.Numeric(symb, device=dev)
    t_alloc = time.perf_counter() - t0
    d_Ax = torch.from_numpy(A.x).to(f"cuda:{dev}")
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        rc = num.factor_device(d_Ax.data_ptr(), sync=True)
        assert rc == 0, f"factorization failed: {rc}"

    num.set_profile(not args.graph)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        num.factor_device(d_Ax.data_ptr(), sync=False)
    rc = num.status()  # synchronizes the library stream
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert rc == 0
    ms_step = dt * 1e3 / args.steps
    gflops = F / (ms_step * 1e-3) / 1e9

    roof = None
    phases = None
    if not args.graph:
        phases = num.timing().tolist()
        fl, ms, nl = num.syrk_stats(256)
        if ms > 0 and nl > 0:
            ach = fl / (ms * 1e-3) / 1e12
            roof = {
                "bound": "mfma", "achieved": round(ach, 3), "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / FP64_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                "kernel": "syrk_mfma_kernel (CB update, fronts w>=256)",
                "flops_per_step": fl, "kernel_ms_per_step": round(ms, 3), "launches_per_step": nl,
            }

    out = {
        "metric": "numeric-factorization fp64 GFLOP/s (F=sum colcount^2)",
        "value": round(gflops, 2),
        "unit": "GFLOP/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (3D 7-point Laplacian, geometric ND order, exact integer values)",
        "config": {
            "workload": f"lap3d_{args.k}_nd",
            "n": st["n"], "nnz_A_upper": st["nnz_A"], "nnz_L": st["nnz_L"], "flops": F,
            "supernodes": st["n_supernodes"], "levels": st["n_levels"], "max_front": st["max_front_m"],
            "flops_executed": st["flops_executed"], "parallelism": "single GPU",
        },
        "roofline": roof,
        "timing_s": {"generate": round(t_gen, 3), "analyze": round(t_an, 3), "numeric_create": round(t_alloc, 3)},
        "phase_ms": phases,
    }
    if not args.no_cpu_baseline and rank == 0:
        out["cpu_baseline"] = cpu_baseline(args.cpu_k)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
