"""Per-kernel MFMA utilisation and clock from rocprofv3 --pmc counter CSVs
(scripts/gpu.sh mfma).  GRBM_GUI_ACTIVE is summed over the 8 XCDs
(MI355X_MICROARCH.md, DVFS note): clock = GRBM / 8 / duration.  Raw MFMA ratio =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM / 8 * 1024 SIMDs); utilisation = raw ratio of the
kernel / raw ratio of the register-only probe (which issues nothing but MFMAs).

For short dispatches GRBM_GUI_ACTIVE also counts cycles outside the dispatch's own
kernel-trace window, so GRBM / 8 / duration can exceed the part's 2.4 GHz maximum
(2.8-3.7 GHz for the 30-80 us panel kernels).  Such a clock is not
reported: clock_GHz is null there, and the busy fraction is the time-based one,
SQ_VALU_MFMA_BUSY_CYCLES / (duration x 2.4 GHz x 1024 SIMDs) -- a lower bound (the
clock is at most 2.4 GHz).  busy_basis names which one a row uses."""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Dispatch_Id"]
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[k] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for k, c in per.items():
        name, ns = meta[k]
        a = agg[name]
        a["launches"] += 1
        a["ns"] += ns
        for cn, v in c.items():
            a[cn] += v
    return agg


F_MAX_GHZ = 2.4  # MI355X peak engine clock (MI355X_MICROARCH.md)


def ratio(a):
    g = a.get("GRBM_GUI_ACTIVE", 0.0)
    return a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(g / 8.0 * 1024.0, 1.0)


def busy(a):
    """(busy fraction, clock GHz or None, basis): counter-clock based when that clock is
    physical (<= 2.4 GHz + 1 %), else time-based at the 2.4 GHz maximum."""
    clk = a["GRBM_GUI_ACTIVE"] / 8.0 / a["ns"] if a["ns"] > 0 else 0.0
    if 0.0 < clk <= F_MAX_GHZ * 1.01:
        return ratio(a), round(clk, 3), "GRBM_GUI_ACTIVE"
    tb = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(a["ns"] * F_MAX_GHZ * 1024.0, 1.0)
    return tb, None, "kernel-trace duration x 2.4 GHz"


def main():
    probe = load(sys.argv[1])
    step = load(sys.argv[2])
    pk = max(probe, key=lambda n: probe[n]["ns"])
    pr, pclk, _ = busy(probe[pk])
    out = {"note": __doc__.replace("\n", " "),
           "probe": {"kernel": pk[:80], "raw_mfma_ratio": round(pr, 4), "clock_GHz": pclk},
           "step_kernels": {}}
    tot = sum(a["ns"] for a in step.values())
    for name, a in sorted(step.items(), key=lambda kv: -kv[1]["ns"]):
        if a["ns"] < 0.005 * tot:
            continue
        b, clk, basis = busy(a)
        out["step_kernels"][name[:90]] = {
            "launches": int(a["launches"]), "ms": round(a["ns"] / 1e6, 3),
            "clock_GHz": clk, "busy_basis": basis,
            "mfma_util": round(b / pr, 4) if pr > 0 else None,
            "raw_mfma_ratio": round(b, 4),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
