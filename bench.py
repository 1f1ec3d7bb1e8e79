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
import re
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


# The dominant kernel: the CB SYRK on 128 x 128 tiles with the trickle epilogue.  Its
# kernel-trace name carries one template argument per kernel parameter, and their
# number grew over the rounds (<128, 2, 4, 1>, <128, 2, 4, 1, 0>, <128, 2, 4, 1, 0, 0>):
# the profile lookups match the instance on its leading arguments, whatever follows.
DOMINANT_KERNEL = "syrk_mfma_kernel<128,2,4,1,0,0>"
_DOMINANT_RE = re.compile(r"syrk_mfma_kernel<128, 2, 4, 1(, 0)*>")


def _dominant_entry(table):
    """The entry of a per-kernel table (kernel name -> stats) that is the dominant
    kernel instance, or None."""
    for name, v in table.items():
        if _DOMINANT_RE.search(name):
            return name, v
    return None


def _latest_profile(fname):
    """The newest committed profiles/rNN/<fname> (rounds in descending order)."""
    pdir = os.path.join(ROOT, "profiles")
    try:
        rounds = sorted((d for d in os.listdir(pdir) if re.fullmatch(r"r\d\d", d)), reverse=True)
    except OSError:
        return None
    for d in rounds:
        p = os.path.join(pdir, d, fname)
        if os.path.exists(p):
            return p
    return None


def cb_syrk_traffic(p=None):
    """HBM bytes per dominant-kernel launch from the newest committed PMC profile (or
    the summary `p`; scripts/gpu.sh pmc: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes,
    FETCH_SIZE doubled per the gfx950 note); (None, None) when the profile is absent."""
    p = p or _latest_profile("pmc_summary.json")
    if p is None:
        return None, None
    try:
        with open(p) as f:
            hit = _dominant_entry(json.load(f)["kernels"])
    except (OSError, KeyError, ValueError):
        return None, None
    if hit is None:
        return None, None
    name, cb = hit
    b = cb["fetch_bytes_per_launch"] + cb["write_bytes_per_launch"]
    rel = os.path.relpath(p, ROOT)
    return round(b), (f"bytes per {DOMINANT_KERNEL} launch (FETCH_SIZE x2 + WRITE_SIZE), {rel} "
                      f"[{name.split('(')[0]}]; L2-miss bytes incl. Infinity-Cache hits")


def cb_syrk_mfma_counters(p=None):
    """MFMA utilisation and clock of the dominant kernel from the newest committed
    counter pass (or the summary `p`; scripts/gpu.sh mfma: SQ_VALU_MFMA_BUSY_CYCLES /
    (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) on an eager bench step); None when absent."""
    p = p or _latest_profile("mfma_util.json")
    if p is None:
        return None
    try:
        with open(p) as f:
            hit = _dominant_entry(json.load(f)["step_kernels"])
    except (OSError, KeyError, ValueError):
        return None
    if hit is None:
        return None
    _, v = hit
    return {"mfma_busy_frac": v["raw_mfma_ratio"], "clock_GHz": v["clock_GHz"],
            "source": f"{os.path.relpath(p, ROOT)} (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE)"}


def backward_error(A, x, b):
    """Normwise backward error of x for the symmetric A held as upper CSC."""
    import scipy.sparse as sp

    U = sp.csc_matrix((A.x, A.i, A.p), shape=(A.n_cols, A.n_cols))
    d = U.diagonal()
    Ax = U @ x + U.T @ x - d * x
    r = np.abs(Ax - b).max()
    anorm = np.abs(U).sum(axis=0).A1 + np.abs(U).sum(axis=1).A1 - np.abs(d)
    return float(r / (anorm.max() * np.abs(x).max() + np.abs(b).max()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-solve", action="store_true")
    ap.add_argument("--cpu-k", type=int, default=32)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--relax-wmax", type=int, default=None)
    ap.add_argument("--nbo", type=int, default=None, help="panel outer block (rank-k update width)")
    ap.add_argument("--lookahead", type=int, default=None)
    ap.add_argument("--inner-order", type=int, default=None)
    ap.add_argument("--opt", action="append", default=[],
                    help="extra sc_options field, key=value (lists comma-separated), e.g. nrelax=4,16,48")
    ap.add_argument("--tile", type=int, default=None, help="SYRK tile: 0 auto, 64, 128")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--transport", choices=["rccl", "host", "dry"], default="rccl",
                    help="N > 1 data path: rccl (default, one GPU per rank); host: every transfer staged "
                         "through host memory over gloo (rehearsal with several ranks on one GPU); dry: "
                         "comm steps move nothing (per-rank compute only, the factor is not validated)")
    args = ap.parse_args()

    import torch
    import sparsecholesky_amd as sc

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.gpus > 1 and world == 1:
        raise SystemExit("multi-GPU runs are launched with torch.distributed.run (one rank per GPU)")
    # rccl: one GPU per rank; host / dry rehearsals may put several ranks on one GPU
    dev = local_rank if args.transport == "rccl" else local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist

        # CPU group: carries only the RCCL unique id, barriers and the max-time
        # reduction; the data path (contribution blocks) is RCCL inside the library.
        dist.init_process_group("gloo")

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    t0 = time.perf_counter()
    A = sc.laplacian3d(args.k)
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    kw = {"use_graph": args.graph if world == 1 else 0}
    if args.relax_wmax is not None:
        kw["relax_wmax"] = args.relax_wmax
    if args.nbo is not None:
        kw["panel_nb_outer"] = args.nbo
    if args.lookahead is not None:
        kw["lookahead"] = args.lookahead
    if args.inner_order is not None:
        kw["inner_order"] = args.inner_order
    if args.tile is not None:
        kw["syrk_tile"] = args.tile
    for kv in args.opt:
        key, val = kv.split("=", 1)
        vals = [float(x) if "." in x else int(x) for x in val.split(",")]
        kw[key] = vals if len(vals) > 1 else vals[0]
    symb = sc.Symbolic(A, **kw)
    t_an = time.perf_counter() - t0
    st = symb.stats()
    F = st["flops"]
    t0 = time.perf_counter()
    work_share = None
    if world > 1:
        if args.transport == "rccl":
            uid = [sc.dist_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            num = sc.Numeric(symb, device=dev, rank=rank, nranks=world, uid=uid[0])
        else:
            num = sc.Numeric(symb, device=dev, rank=rank, nranks=world,
                             transport=sc.GlooHostTransport() if args.transport == "host" else "dry")
        _, wr = symb.owner_map(world)
        work_share = [round(float(x) / float(wr.sum()), 4) for x in wr]
    else:
        num = sc.Numeric(symb, device=dev)
    t_alloc = time.perf_counter() - t0
    d_Ax = torch.from_numpy(A.x).to(f"cuda:{dev}")
    torch.cuda.synchronize()

    # Roofline timing inside the timed region: under hipGraph replay, 1-thread
    # s_memrealtime stamp kernels bracket each CB SYRK launch (HIP cannot time
    # events captured in a graph); eager runs use HIP events around every launch.
    # Enabled before the warmup so the graph captured there is the one timed.
    num.set_profile(2 if args.graph else 1)
    for _ in range(max(args.warmup, 1 if args.graph else 0)):
        rc = num.factor_device(d_Ax.data_ptr(), sync=True)
        # dry transport: received blocks hold stale values, a pivot may fail (not a factor)
        assert rc == 0 or args.transport == "dry", f"factorization failed: {rc}"

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        num.factor_device(d_Ax.data_ptr(), sync=False)
    rc = num.status()  # synchronizes the library stream
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    barrier()
    assert rc == 0 or args.transport == "dry", f"factorization failed: {rc}"
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_step = dt * 1e3 / args.steps
    gflops = F / (ms_step * 1e-3) / 1e9

    roof = None
    phases = None
    if not args.graph:
        phases = [round(x, 3) for x in num.timing().tolist()]
    # dominant kernel = the CB SYRK instance on 128 x 128 tiles with the trickle epilogue
    # (the dispatches the rocprofv3 kernel trace lists as syrk_mfma_kernel<128, 2, 4, 1, 0>;
    # <128, 2, 4, 1> before the epilogue template parameter)
    fl, ms, nl = num.syrk_stats(-2)
    gfl, gms, gnl = num.syrk_stats(256)
    if ms > 0 and nl > 0:
        ach = fl / (ms * 1e-3) / 1e12
        traffic, tnote = cb_syrk_traffic()
        alg = num.syrk_bytes(-2) / nl  # algorithmic bytes per launch of the same launches
        roof = {
            "bound": "mfma", "achieved": round(ach, 3), "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / FP64_MFMA_PEAK_TFLOPS, 4), "traffic": traffic, "traffic_note": tnote,
            "algorithmic_bytes_per_launch": round(alg),
            "traffic_ratio": round(traffic / alg, 3) if traffic and alg > 0 else None,
            "traffic_ratio_note": "counter bytes / algorithmic bytes (operand rows once + C written once + "
                                  "gathered children's CB entries once), per launch",
            "kernel": f"{DOMINANT_KERNEL} (CB update)" + (" on rank 0" if world > 1 else ""),
            "flops_per_step": fl, "kernel_ms_per_step": round(ms, 3), "launches_per_step": nl,
            "avg_launch_ms": round(ms / nl, 3),
        }
        if gms > 0:
            roof["gate_w256_tflops"] = round(gfl / (gms * 1e-3) / 1e12, 3)
        roof["counters"] = cb_syrk_mfma_counters()
    pfl, pms, pnl = num.syrk_stats(-1) if not args.graph else (0.0, -1.0, 0)
    cfl, cms, cnl = num.syrk_stats(0)
    if roof is not None and pms > 0 and cms > 0:
        roof["other_syrk"] = {"panel_update_tflops": round(pfl / (pms * 1e-3) / 1e12, 2),
                              "panel_update_ms": round(pms, 2), "panel_update_flops": pfl,
                              "cb_all_tflops": round(cfl / (cms * 1e-3) / 1e12, 2)}

    mem = num.memory()  # before the solve allocates its buffers (and, multi-rank, the gathered factor)
    # Validation of the factor just timed (outside the timed region): x = A^-1 b by
    # the GPU triangular solves with that factor (multi-rank handles gather
    # the factor collectively first), then the normwise backward error on the host,
    # ||A x - b||_inf / (||A||_inf ||x||_inf + ||b||_inf), with A from the upper CSC.
    # A wrong factor cannot pass: the bound is 1e-12 (measured 6.9e-16 at 128^3).
    solve = None
    berr = None
    skip = "skipped: dry transport (no data moved, factor not valid)"
    validate = args.transport != "dry"
    if world > 1 and validate:
        # the multi-rank solve gathers the whole factor on every rank: when rehearsal
        # ranks share one GPU, check (collectively, so all ranks take the same branch)
        # that every sharer's copy fits, else skip the check instead of failing mid-gather
        tot = torch.tensor([float(mem["panel"])], dtype=torch.float64)
        dist.all_reduce(tot)
        ndev = max(torch.cuda.device_count(), 1)
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        sharers = 1 if args.transport == "rccl" else sum(1 for r in range(lw) if r % ndev == dev)
        barrier()
        free, _ = torch.cuda.mem_get_info(dev)
        need = sharers * (tot.item() + 16.0 * st["n"] + 2e9)
        ok = torch.tensor([1 if free >= need else 0], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not ok.item():
            skip = (f"skipped: {sharers} ranks share one GPU and the solve gathers the whole factor "
                    f"({tot.item() / 1e9:.1f} GB) on each (parity of this plan: tests/test_gpu_parity.py)")
            validate = False
    if validate:
        d_b = torch.ones(st["n"], dtype=torch.float64, device=f"cuda:{dev}")
        d_x = torch.empty_like(d_b)
        torch.cuda.synchronize()  # d_b complete before the library stream reads it
        num.solve_device(d_b.data_ptr(), d_x.data_ptr())
        x = d_x.cpu().numpy()
        berr = backward_error(A, x, np.ones(st["n"]))
        if not berr < 1e-12:
            raise SystemExit(f"validation failed: backward error {berr:.3e} of the timed factor")
    if world == 1 and not args.no_solve:
        # solve timing: forward + backward sweep, each reads L once (8 * panel entries
        # bytes, relaxed zeros included)
        reps = 3
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            num.solve_device(d_b.data_ptr(), d_x.data_ptr())
        torch.cuda.synchronize()
        sms = (time.perf_counter() - t0) * 1e3 / reps
        lbytes = 2.0 * 8.0 * st["panel_entries"]
        solve = {"ms": round(sms, 3), "L_read_GBs": round(lbytes / (sms * 1e-3) / 1e9, 1),
                 "note": "x = A^-1 b, device vectors, forward + backward sweep; GB/s = 2 x 8 B x panel entries / time"}
    out = {
        "metric": "numeric-factorization fp64 GFLOP/s (F=sum colcount^2)",
        "value": round(gflops, 2),
        "unit": "GFLOP/s",
        "n_gpus": world,
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
            "flops_executed": st["flops_executed"],
            "parallelism": "single GPU" if world == 1 else
            f"subtree partition over {world} GPUs, RCCL p2p of contribution blocks at merge fronts"
            if args.transport == "rccl" else
            f"subtree partition over {world} ranks on {torch.cuda.device_count()} GPU(s), transport "
            f"{args.transport} (rehearsal of the N-GPU protocol; not an N-GPU measurement)",
            "work_share_per_rank": work_share,
            "options": {"relax_wmax": symb.opt.relax_wmax, "panel_nb_outer": symb.opt.panel_nb_outer,
                        "small_front_max": symb.opt.small_front_max, "use_graph": symb.opt.use_graph,
                        "lookahead": symb.opt.lookahead, "syrk_tile": symb.opt.syrk_tile,
                        "inner_order": symb.opt.inner_order,
                        **({"dist_asm": symb.opt.dist_asm, "dist_pieces": symb.opt.dist_pieces} if world > 1 else {}),
                        **{k: v for k, v in kw.items() if k not in ("use_graph",)}},
        },
        "roofline": roof,
        "timing_s": {"generate": round(t_gen, 3), "analyze": round(t_an, 3), "numeric_create": round(t_alloc, 3)},
        "phase_ms": phases,
        "validation": {"backward_error": float(f"{berr:.3e}") if berr is not None else None, "bound": 1e-12,
                       "check": "GPU solve with the timed factor, ||Ax-b||/(||A|| ||x||+||b||), inf-norms"
                       if berr is not None else skip},
        "transport": args.transport if world > 1 else None,
        "device_memory_GB": {"total": round(mem["total"] / 1e9, 2), "panels_L": round(mem["panel"] / 1e9, 2),
                             "work_arena_CB": round(mem["work"] / 1e9, 2),
                             "note": "rank 0 of the handle, factorization only (solve buffers excluded)"},
        "solve": solve,
    }
    if not args.no_cpu_baseline and rank == 0 and world == 1:
        out["cpu_baseline"] = cpu_baseline(args.cpu_k)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
