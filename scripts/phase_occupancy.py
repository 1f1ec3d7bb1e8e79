"""From a rocprofv3 kernel trace of one eager 128^3 factorization: over time windows
(the root front, the level-17 pivot phase), how long the GPU ran (a) a big panel
update (syrk<128,...,0>), (b) only chain kernels (POTRF / TRSM / 64-tile updates),
(c) a CB SYRK, (d) nothing."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "front_small" in r["Kernel_Name"]]
run = rows[starts[-4]:]
t1 = max(int(r["End_Timestamp"]) for r in run)


def cls(n):
    if "syrk_mfma_kernel<128, 2, 4, 0" in n:
        return "big_update"
    if "syrk_mfma_kernel<128, 2, 4, 1" in n or "syrk_mfma_kernel<64, 2, 2, 1" in n:
        return "cb"
    if "potrf" in n or "trsm" in n or "syrk_mfma_kernel<64, 2, 2, 0" in n:
        return "chain"
    return "other"


ev = []
for r in run:
    c = cls(r["Kernel_Name"])
    ev.append((int(r["Start_Timestamp"]), 1, c))
    ev.append((int(r["End_Timestamp"]), -1, c))
ev.sort()


def window(a, b, label):
    act = {"big_update": 0, "cb": 0, "chain": 0, "other": 0}
    acc = {"big_update": 0.0, "cb": 0.0, "only_chain": 0.0, "other": 0.0, "idle": 0.0}
    last = a
    for t, d, c in ev:
        if t > a and last < b:
            lo, hi = max(last, a), min(t, b)
            if hi > lo:
                if act["cb"]:
                    acc["cb"] += hi - lo
                elif act["big_update"]:
                    acc["big_update"] += hi - lo
                elif act["chain"]:
                    acc["only_chain"] += hi - lo
                elif act["other"]:
                    acc["other"] += hi - lo
                else:
                    acc["idle"] += hi - lo
        act[c] += d
        last = t
    tot = (b - a) / 1e6
    print(f"{label}: {tot:.1f} ms: " + ", ".join(f"{k} {v / 1e6:.1f}" for k, v in acc.items()))


window(t1 - 48.5e6, t1, "root (last 48.5 ms)")
window(t1 - 181e6, t1 - 48.5e6, "level 17 (133 ms before)")
window(t1 - 261e6, t1 - 181e6, "level 16 (80 ms before)")
