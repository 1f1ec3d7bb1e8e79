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
serialised behind the rank's compute (nothing overlapped): rank_ms + comm_ms is the
"serialised-comm estimate" -- NOT an upper bound: it leaves out the time a rank waits
for another rank's compute.

Critical-path estimate (--timeline, one extra eager profiled factorization per rank):
each rank's dry timeline gives, per comm step, the time its comm stream posts the step
(sends: when the data is computed) and the time its main stream needs the step (the
start of its next main-stream launch).  A discrete-event replay over the plan's global
step order then moves every message over its link (link_GBs per direction, msg_us each,
one transfer at a time per directed link), starts a step on a rank no earlier than the
rank's previous step (one in-order comm stream), and delays a receiving rank's compute
from the need point until its data has arrived -- so waiting on other ranks' compute
and on the links is on the critical path, while transfers that overlap compute are
not.  Assumed, not measured: link_GBs (default 50 GB/s per direction of one xGMI
link; 153 GB/s spec) and msg_us.

  python scripts/dist_project.py [--k 128] [--n 2,4,8] [--opt key=value ...] [--timeline] [--graph]
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


KINDS = {0: "INIT", 1: "SLAB", 2: "DELIVER"}


def comm_by_kind(symb, n, link_gbs, msg_us):
    """GB sent per comm-step kind, and per kind the largest per-rank serialised link time
    (the comm_model sum restricted to that kind's steps)."""
    import numpy as np

    st = symb.dist_steps(n)
    gb = {k: 0.0 for k in KINDS.values()}
    ms = {k: [] for k in KINDS.values()}
    for r in range(n):
        step, peer, nb, snd = symb.dist_schedule(n, r)
        t = {k: 0.0 for k in KINDS.values()}
        for a in np.unique(step):
            sel = step == a
            kind = KINDS.get(int(st["kind"][a]), str(int(st["kind"][a])))
            link = {}
            for p, b, s in zip(peer[sel], nb[sel], snd[sel]):
                x = link.setdefault(int(p), [0, 0])
                x[0 if s else 1] += int(b)
                if s:
                    gb[kind] = gb.get(kind, 0.0) + int(b) / 1e9
            t[kind] = t.get(kind, 0.0) + max(max(x) for x in link.values()) / (link_gbs * 1e9) * 1e3 + \
                sel.sum() * msg_us * 1e-3
        for k, v in t.items():
            ms.setdefault(k, []).append(v)
    return ({k: round(v, 2) for k, v in gb.items()},
            {k: round(max(v), 1) if v else 0.0 for k, v in ms.items()})


def rank_timeline(num):
    """From one eager profiled factorization of a dry handle: (total ms, post[step],
    need[step], main-stream launches [(t0, t1, kind)]) -- the step's comm-stream start,
    and the start of the first main-stream launch after it in schedule order (the point
    the main stream waits for the step)."""
    tl = num.launch_times()
    t0, t1, kind, step, strm = tl["t0"], tl["t1"], tl["kind"], tl["step"], tl["stream"]
    total = float(max(t1.max(), 0.0)) if len(t1) else 0.0
    post, need = {}, {}
    for i in range(len(t0)):
        if kind[i] != 6:
            continue
        st = int(step[i])
        post[st] = float(t0[i])
        nxt = next((float(t0[j]) for j in range(i + 1, len(t0)) if strm[j] == 0), total)
        need[st] = max(nxt, float(t1[i]))
    main = [(float(a), float(b), int(k)) for a, b, k, q in zip(t0, t1, kind, strm) if q == 0 and k != 6]
    return total, post, need, main


def critical_path(symb, n, timelines, link_gbs, msg_us, explain=False):
    """Discrete-event replay of the plan's comm steps over the ranks' dry timelines (see
    the module docstring).  Returns per-rank finish times (ms); with explain=True also
    the critical path as a chain of segments (see explain_chain)."""
    sends = {}  # step -> [(src, dst, bytes)] in plan order
    for r in range(n):
        step, peer, nb, snd = symb.dist_schedule(n, r)
        for st, p, b, s in zip(step, peer, nb, snd):
            if s:
                sends.setdefault(int(st), []).append((r, int(p), int(b)))
    delay = [0.0] * n      # accumulated wait of each rank's main stream
    comm_free = [0.0] * n  # each rank's comm stream
    link_free = {}
    # per rank, the waits that raised its delay, in order: the step, its need point (in
    # the rank's own dry timeline), the delay after it, and the message that arrived last
    # (source rank, its post point, how many of the source's own waits preceded it, what
    # bounded the transfer's start, the transfer time)
    events = [[] for _ in range(n)]
    for st in sorted(sends):
        msgs = sends[st]
        parts = sorted({m[0] for m in msgs} | {m[1] for m in msgs})
        start = {}
        for r in parts:
            post = timelines[r][1]
            start[r] = max(post.get(st, 0.0) + delay[r], comm_free[r])
        done = dict(start)
        last = {}
        for src, dst, b in msgs:
            lf = link_free.get((src, dst), 0.0)
            t0 = max(start[src], start[dst], lf)
            xfer = b / (link_gbs * 1e9) * 1e3 + msg_us * 1e-3
            t = t0 + xfer
            link_free[(src, dst)] = t
            done[src] = max(done[src], t)
            done[dst] = max(done[dst], t)
            if t > last.get(dst, (-1.0,))[0]:
                bound = "src" if t0 == start[src] else ("link" if t0 == lf else "dst")
                last[dst] = (t, src, bound, xfer, len(events[src]))
        for r in parts:
            comm_free[r] = done[r]
            if r in last:  # a receiver waits at its need point
                nd = timelines[r][2].get(st, 0.0)
                nw = done[r] - nd
                if nw > delay[r]:
                    t, src, bound, xfer, nsrc = last[r]
                    events[r].append(dict(step=st, need=nd, delay=nw, prev=delay[r], src=src,
                                          src_post=timelines[src][1].get(st, 0.0), src_events=nsrc, bound=bound,
                                          xfer=xfer))
                    delay[r] = nw
    finish = [round(max(timelines[r][0] + delay[r], comm_free[r]), 2) for r in range(n)]
    if not explain:
        return finish
    return finish, explain_chain(symb, n, timelines, events, finish)


KIND_NAMES = {0: "small", 1: "asm", 2: "potrf", 3: "trsm", 4: "panel", 5: "cb", 6: "comm"}


def explain_chain(symb, n, timelines, events, finish):
    """Backtrack the critical path from the rank that finishes last.  Each element: a
    compute segment on one rank (its dry timeline between two points, with the main-
    stream kernel time in it by launch kind) and the hand-off that preceded it (step id,
    kind, level, front, slab / group k, piece p; wait ms = from the source's post point,
    delayed as the source ran, to the data's arrival: transfer plus link / comm-stream
    queueing, `bound` says which limited the start).  The chain continues on the source
    rank at its post point, so finish = sum(compute) + sum(wait) when the last rank ends
    on its own compute."""
    steps = symb.dist_steps(n)
    r = max(range(n), key=lambda q: finish[q])
    t_end = timelines[r][0]
    nev = len(events[r])  # the replay applies a rank's latest delay to everything after it
    chain = []

    def by_kind(rank, a, b):
        out = {}
        for t0, t1, k in timelines[rank][3]:
            lo, hi = max(t0, a), min(t1, b)
            if hi > lo:
                nm = KIND_NAMES.get(k, str(k))
                out[nm] = out.get(nm, 0.0) + hi - lo
        return {k: round(v, 3) for k, v in out.items()}

    guard = 0
    while guard < 100000:
        guard += 1
        if nev == 0:
            chain.append(dict(rank=r, compute_ms=round(t_end, 3), compute_by_kind=by_kind(r, 0.0, t_end),
                              wait_ms=0.0))
            break
        e = events[r][nev - 1]  # the wait that set the delay this point of the rank runs behind
        st = e["step"]
        src, ns = e["src"], e["src_events"]
        src_at = e["src_post"] + (events[src][ns - 1]["delay"] if ns > 0 else 0.0)
        chain.append(dict(rank=r, compute_ms=round(t_end - e["need"], 3), compute_by_kind=by_kind(r, e["need"], t_end),
                          step=st, step_kind={0: "INIT", 1: "SLAB", 2: "DELIVER"}.get(int(steps["kind"][st])),
                          level=int(steps["level"][st]), front=int(steps["front"][st]), k=int(steps["k"][st]),
                          p=int(steps["p"][st]), wait_ms=round(e["need"] + e["delay"] - src_at, 3), src=src,
                          bound=e["bound"], transfer_ms=round(e["xfer"], 3)))
        r, t_end, nev = src, e["src_post"], ns
    chain.reverse()
    tot = {"compute_ms": round(sum(c["compute_ms"] for c in chain), 3),
           "wait_ms": round(sum(c["wait_ms"] for c in chain), 3)}
    by_step_kind, by_launch = {}, {}
    for c in chain:
        if "step_kind" in c:
            by_step_kind[c["step_kind"]] = round(by_step_kind.get(c["step_kind"], 0.0) + c["wait_ms"], 3)
        for k, v in c["compute_by_kind"].items():
            by_launch[k] = round(by_launch.get(k, 0.0) + v, 3)
    return dict(chain=chain, totals=tot, wait_by_step_kind=by_step_kind, compute_by_launch_kind=by_launch,
                finish_ms=max(finish))


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
    ap.add_argument("--timeline", action="store_true",
                    help="also the critical-path estimate (one eager profiled factorization per rank)")
    ap.add_argument("--graph", action="store_true",
                    help="also time every rank's dry schedule replayed as one hipGraph (eager vs graph gap)")
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
            gbk, msk = comm_by_kind(symb, n, args.link_gbs, args.msg_us)
            print(json.dumps({"k": args.k, "n": n, "opts": kw, "link_GBs": args.link_gbs, **cm,
                              "sent_GB_by_kind": gbk, "serial_link_ms_max_rank_by_kind": msk}), flush=True)
        return
    import torch

    kw = {}
    for kv in args.opt:
        key, val = kv.split("=", 1)
        kw[key] = int(val)
    A = sc.laplacian3d(args.k)
    symb = sc.Symbolic(A, **kw)
    symb_g = sc.Symbolic(A, use_graph=1, **kw) if args.graph else None
    F = symb.stats()["flops"]
    d_Ax = torch.from_numpy(A.x).to("cuda:0")

    def timed(num):
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
        return round(best, 2)

    for n in [int(x) for x in args.n.split(",")]:
        info = symb.dist_plan_info(n)
        _, work = symb.owner_map(n)
        per, per_g, tls = [], [], []
        for r in range(n):
            num = sc.Numeric(symb, device=0, rank=r, nranks=n, transport="dry")
            best = timed(num)
            per.append(best)
            if args.timeline:
                num.set_profile(1)
                num.factor_device(d_Ax.data_ptr(), sync=True)
                tot, post, need, main = rank_timeline(num)
                f = best / tot if tot > 0 else 1.0  # the event-bracketed run is slower: rescale
                tls.append((best, {k: v * f for k, v in post.items()}, {k: v * f for k, v in need.items()},
                            [(a * f, b * f, k) for a, b, k in main]))
            del num
            gc.collect()
            msg = f"  n={n} rank {r}: {best:.1f} ms"
            if symb_g is not None:
                num = sc.Numeric(symb_g, device=0, rank=r, nranks=n, transport="dry")
                per_g.append(timed(num))
                del num
                gc.collect()
                msg += f" (graph {per_g[-1]:.1f} ms)"
            print(msg, flush=True)
        mx = max(per)
        cm = comm_model(symb, n, args.link_gbs, args.msg_us)
        with_comm = [round(a + b, 2) for a, b in zip(per, cm["comm_ms"])]
        rec = {"k": args.k, "n": n, "opts": kw, "rank_ms": per, "max_rank_ms": mx,
               "projected_gflops_no_comm": round(F / (mx * 1e-3) / 1e9, 1),
               "rank_ms_with_comm_serial": with_comm, "max_rank_ms_with_comm_serial": max(with_comm),
               "projected_gflops_with_comm_serial": round(F / (max(with_comm) * 1e-3) / 1e9, 1),
               "link_GBs": args.link_gbs, "msg_us": args.msg_us, **cm,
               "work_share": [round(float(x) / float(work.sum()), 3) for x in work],
               "comm_steps": info["n_steps"], "messages": info["n_msgs"]}
        if per_g:
            rec["rank_ms_graph"] = per_g
            rec["max_rank_ms_graph"] = max(per_g)
        if tls:
            for gbs in sorted({args.link_gbs, 100.0}):
                cp, why = critical_path(symb, n, tls, gbs, args.msg_us, explain=True)
                rec[f"critical_path_ms_{int(gbs)}GBs"] = cp
                rec[f"critical_path_explained_{int(gbs)}GBs"] = why
                rec[f"max_critical_path_ms_{int(gbs)}GBs"] = max(cp)
                rec[f"projected_gflops_critical_path_{int(gbs)}GBs"] = round(F / (max(cp) * 1e-3) / 1e9, 1)
            rec["timeline_total_ms"] = [round(t[0], 2) for t in tls]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
