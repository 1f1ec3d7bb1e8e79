"""Per-launch durations of the last factorization in a small_trace.py kernel trace."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "front_small" in r["Kernel_Name"] or "sc::" in r["Kernel_Name"]]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 7
last = rows[-n:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  grid {r.get('Grid_Size', r.get('Workgroup_Size_X', '')):>7s}  {r['Kernel_Name'][:60]}")
print("wall", (int(last[-1]["End_Timestamp"]) - t0) / 1e3, "us")
