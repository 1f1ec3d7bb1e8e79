"""Summarize rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs (scripts/gpu_pmc.sh)
into per-launch HBM bytes of the CB SYRK kernel (syrk_mfma_kernel<*, 1>).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is reported in KB and
tallies 128-B read requests as 64 B on gfx950, so it is doubled; WRITE_SIZE (KB)
is taken as is.  Our loads are 8 B per lane (coalesced 512-B column runs), a width
the guide calls uncalibrated: the absolute value is indicative, ratios are exact."""
import csv
import glob
import json
import os
import sys


def read(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "")
            disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
            per.setdefault(name, {})
            per[name][disp] = per[name].get(disp, 0.0) + float(r["Counter_Value"])
    return per


def main():
    fetch = read(sys.argv[1], "FETCH_SIZE")
    write = read(sys.argv[2], "WRITE_SIZE")
    out = {"note": "bytes per launch; FETCH_SIZE x2 (gfx950 128-B requests tallied as 64 B), KB -> B",
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, {})
        w = write.get(name, {})
        nf, nw = max(len(f), 1), max(len(w), 1)
        out["kernels"][name[:90]] = {
            "launches": max(len(f), len(w)),
            "fetch_bytes_per_launch": 2.0 * 1024.0 * sum(f.values()) / nf,
            "write_bytes_per_launch": 1024.0 * sum(w.values()) / nw,
        }
    cb = [v for k, v in out["kernels"].items() if (k.startswith("void sc::syrk_mfma_kernel<128, 2, 4, 1>") or
                                                    k.startswith("void sc::syrk_mfma_kernel<128, 2, 4, 1, 0>"))]
    if cb:
        out["cb_syrk_128"] = cb[0]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
