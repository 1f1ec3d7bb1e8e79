"""Analyze a rocprofv3 kernel trace of eager 128^3 factorizations: over the last
48 ms (the root front) per-kernel durations, GPU busy time, and the idle gap
between a POTRF and the TRSM that follows it on the chain."""
import collections
import csv
import sys

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "front_small" in r["Kernel_Name"]]
first_of_last = starts[-4] if len(starts) >= 4 else 0  # 4 small-front launches per level 0
run = rows[first_of_last:]
t0 = int(run[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in run)
print(f"last run: {len(run)} dispatches, {(t1 - t0) / 1e6:.1f} ms")


def short(n):
    for k in ("potrf", "trsm_partial", "trsm", "syrk_mfma_kernel<128, 2, 4, 1", "syrk_mfma_kernel<128, 2, 4, 0",
              "syrk_mfma_kernel<64", "assemble", "front_small", "stamp"):
        if k in n:
            return k
    return n[:30]


for win in (48e6, 181e6):
    tail = [r for r in run if int(r["End_Timestamp"]) > t1 - win]
    ivs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in tail)
    busy = 0
    cs, ce = ivs[0]
    for s, e in ivs[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"last {win / 1e6:.0f} ms: {len(tail)} dispatches, GPU busy (any kernel) {busy / 1e6:.1f} ms")
    dur = collections.defaultdict(list)
    for r in tail:
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:34s} n={len(v):5d} sum {sum(v) / 1e3:7.2f} ms avg {sum(v) / len(v):8.1f} us")
    g1, g2 = [], []
    for i, r in enumerate(tail):
        if short(r["Kernel_Name"]) == "potrf":
            for q in tail[i + 1:i + 8]:
                if short(q["Kernel_Name"]) == "trsm":
                    g1.append((int(q["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3)
                    break
        if short(r["Kernel_Name"]) == "trsm":
            for q in tail[i + 1:i + 8]:
                if short(q["Kernel_Name"]) in ("syrk_mfma_kernel<64", "syrk_mfma_kernel<128, 2, 4, 0", "potrf"):
                    g2.append((int(q["Start_Timestamp"]) - int(r["End_Timestamp"])) / 1e3)
                    break
    if g1:
        print(f"  potrf end -> trsm start: n={len(g1)} avg {sum(g1) / len(g1):.1f} us, min {min(g1):.1f}")
    if g2:
        print(f"  trsm end -> next chain kernel: n={len(g2)} avg {sum(g2) / len(g2):.1f} us, min {min(g2):.1f}")
