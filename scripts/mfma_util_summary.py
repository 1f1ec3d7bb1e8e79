"""Per-kernel MFMA utilisation and clock from rocprofv3 --pmc counter CSVs
(scripts/gpu_mfma_util.sh).  GRBM_GUI_ACTIVE is summed over the 8 XCDs
(MI355X_MICROARCH.md, DVFS note): clock = GRBM / 8 / duration.  Raw MFMA ratio =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM / 8 * 1024 SIMDs); utilisation = raw ratio of the
kernel / raw ratio of the register-only probe (which issues nothing but MFMAs)."""
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


def ratio(a):
    g = a.get("GRBM_GUI_ACTIVE", 0.0)
    return a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(g / 8.0 * 1024.0, 1.0)


def main():
    probe = load(sys.argv[1])
    step = load(sys.argv[2])
    pk = max(probe, key=lambda n: probe[n]["ns"])
    pr = ratio(probe[pk])
    out = {"note": __doc__.replace("\n", " "),
           "probe": {"kernel": pk[:80], "raw_mfma_ratio": round(pr, 4),
                     "clock_GHz": round(probe[pk]["GRBM_GUI_ACTIVE"] / 8.0 / probe[pk]["ns"], 3)},
           "step_kernels": {}}
    tot = sum(a["ns"] for a in step.values())
    for name, a in sorted(step.items(), key=lambda kv: -kv[1]["ns"]):
        if a["ns"] < 0.005 * tot:
            continue
        out["step_kernels"][name[:90]] = {
            "launches": int(a["launches"]), "ms": round(a["ns"] / 1e6, 3),
            "clock_GHz": round(a["GRBM_GUI_ACTIVE"] / 8.0 / a["ns"], 3),
            "mfma_util": round(ratio(a) / pr, 4) if pr > 0 else None,
            "raw_mfma_ratio": round(ratio(a), 4),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
