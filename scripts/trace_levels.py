#!/usr/bin/env python3
"""Timeline of the top levels of one factorization from a rocprofv3 kernel trace
(graph replay or eager): per level the lookahead-stream panel updates (start, end,
duration), the 64-column chain of every slab (span, summed TRSM time) and the CB
SYRK; the last factorization before the first solve in the trace is used.

  python scripts/trace_levels.py gpurun_out/prof [levels=3]

(Replaces the round-2 root_chain / chain_timeline / phase_occupancy one-offs.)"""
import csv
import glob
import sys


def short(n):
    for k, v in (("trsm_panel_g", "TRSM"), ("trsm_partial", "TRSMp"), ("potrf", "POTRF"),
                 ("syrk_mfma_kernel<128, 2, 4, 1, 0>", "CB"), ("syrk_mfma_kernel<128, 2, 4, 1, 1>", "CBe"),
                 ("syrk_mfma_kernel<64, 2, 2, 1", "CB64"), ("syrk_mfma_kernel<128, 2, 4, 0, 0>", "LA"),
                 ("syrk_mfma_kernel<128, 2, 4, 0, 1>", "UPD128"), ("syrk_mfma_kernel<64, 2, 2, 0, 1>", "UPD64"),
                 ("panel_tall", "TALL"), ("solve_inv", "INV"), ("assemble", "ASM"), ("stamp", "stamp"),
                 ("solve_fwd", "solve"), ("solve_gemv", "solve"), ("solve_diag", "solve"), ("front_small", "small")):
        if k in n:
            return v
    return n[:24]


def main():
    path = sys.argv[1]
    nlev = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    f = glob.glob(path + "/**/*kernel_trace.csv", recursive=True) if not path.endswith(".csv") else [path]
    rows = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f[0]))]
    rows.sort(key=lambda x: x[1])
    solves = [i for i, r in enumerate(rows) if r[0] == "solve"]
    fact = rows[:solves[0]] if solves else rows
    cb = [i for i, r in enumerate(fact) if r[0] == "CB"]
    # segment after the last CB launch is the root; before it, one segment per level
    bounds = [(cb[-1] + 1, len(fact), "root")]
    for q in range(1, nlev):
        if len(cb) > q:
            bounds.append((cb[-q - 1] + 1, cb[-q], f"root-{q}"))
    for a, b, name in bounds:
        seg = fact[a:b]
        if not seg:
            continue
        t0 = seg[0][1]
        chain_end = max(r[2] for r in seg if r[0] in ("TRSM", "TRSMp", "POTRF", "LA", "UPD128", "UPD64", "ASM", "TALL"))
        la = [r for r in seg if r[0] == "LA"]
        tr = [r for r in seg if r[0] == "TRSM"]
        print(f"{name}: panel phase {(chain_end - t0) / 1e6:.2f} ms, lookahead launches {len(la)} "
              f"({sum(r[2] - r[1] for r in la) / 1e6:.2f} ms), TRSM launches {len(tr)} "
              f"({sum(r[2] - r[1] for r in tr) / 1e6:.2f} ms)")
        for r in la:
            print(f"   LA {(r[1] - t0) / 1e6:7.2f} - {(r[2] - t0) / 1e6:7.2f}  ({(r[2] - r[1]) / 1e6:.2f})")
        for k in range(0, len(tr), 16):
            g = tr[k:k + 16]
            print(f"   slab {k // 16:2d} chain {(g[0][1] - t0) / 1e6:7.2f} - {(g[-1][2] - t0) / 1e6:7.2f} "
                  f"span {(g[-1][2] - g[0][1]) / 1e6:5.2f}  TRSM {sum(x[2] - x[1] for x in g) / 1e6:5.2f}")
        if b < len(fact) and fact[b][0] == "CB":
            print(f"   CB {(fact[b][1] - t0) / 1e6:7.2f} - {(fact[b][2] - t0) / 1e6:7.2f}")


if __name__ == "__main__":
    main()
