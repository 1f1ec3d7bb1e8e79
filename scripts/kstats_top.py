"""Top kernels of a rocprofv3 --stats directory (kernel_stats.csv): name, calls, avg us, total ms.

  python scripts/kstats_top.py DIR [N]
"""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
f = sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True))[-1]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:n]:
    print(f"{r['Calls']:>8} {float(r['AverageNs']) / 1e3:10.2f} us {float(r['TotalDurationNs']) / 1e6:10.2f} ms  {r['Name'][:110]}")
