"""Root-front chain timing from a rocprofv3 kernel trace (graph or eager): over the
last `win` ms of the trace, per POTRF dispatch the next TRSM and the next panel
update (syrk ..., 0) that starts after that TRSM ends; prints mean durations and
gaps, i.e. the critical-path cost of one 64-column step."""
import csv
import glob
import statistics
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
win = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 45e6
rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", ""))
        for r in csv.DictReader(open(f))]
rows.sort(key=lambda x: x[1])
t1 = max(r[2] for r in rows if "potrf" in r[0])
rows = [r for r in rows if r[2] > t1 - win and r[1] < t1 and "solve" not in r[0] and "permute" not in r[0]]
pot = [r for r in rows if "potrf" in r[0]]
trs = [r for r in rows if "trsm_panel" in r[0]]
upd = [r for r in rows if "syrk_mfma_kernel" in r[0] and r[0].rstrip().endswith(", 0>(sc::GemmTask const*, HIP_vector_type<int, 2u> const*)") or ("syrk_mfma_kernel" in r[0] and ", 0>" in r[0])]
stats = {"potrf": [], "gap_pt": [], "trsm": [], "gap_tu": [], "upd": [], "gap_up": []}
for i, p in enumerate(pot[:-1]):
    t = next((x for x in trs if x[1] >= p[2]), None)
    if t is None:
        continue
    u = next((x for x in upd if x[1] >= t[2]), None)
    nxt = pot[i + 1]
    stats["potrf"].append((p[2] - p[1]) / 1e3)
    stats["gap_pt"].append((t[1] - p[2]) / 1e3)
    stats["trsm"].append((t[2] - t[1]) / 1e3)
    if u is not None and u[1] < nxt[1]:
        stats["gap_tu"].append((u[1] - t[2]) / 1e3)
        stats["upd"].append((u[2] - u[1]) / 1e3)
        stats["gap_up"].append((nxt[1] - u[2]) / 1e3)
print(f"window {win / 1e6:.0f} ms: {len(pot)} POTRF, {len(trs)} TRSM, {len(upd)} panel updates")
for k, v in stats.items():
    if v:
        print(f"  {k:7s} mean {statistics.mean(v):7.1f} us  median {statistics.median(v):7.1f} us  n {len(v)}")
step = [(pot[i + 1][1] - pot[i][1]) / 1e3 for i in range(len(pot) - 1)]
print(f"  POTRF-to-POTRF mean {statistics.mean(step):.1f} us, median {statistics.median(step):.1f} us")
