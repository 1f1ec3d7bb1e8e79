# MFMA utilisation and effective clock of the SYRK kernel (microbench dispatches):
# SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * SIMDs), clock = GRBM_GUI_ACTIVE / duration.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -f csv \
  -d gpurun_out/pmc_mfma -o mf -- python3 scripts/ubench.py > gpurun_out/pmc_mfma.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/pmc_mfma/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
d = collections.defaultdict(dict)
meta = {}
for r in rows:
    k = r["Dispatch_Id"]
    d[k][r["Counter_Name"]] = d[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    meta[k] = (r["Kernel_Name"][:48], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Grid_Size"])
for k in sorted(d, key=int):
    name, ns, grid = meta[k]
    c = d[k]
    g = c.get("GRBM_GUI_ACTIVE", 0)
    if ns < 200000:
        continue
    util = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(g * 1024, 1)
    print(f"{name:48s} grid={grid:>9s} {ns/1e6:8.3f} ms  clock {g/ns:5.2f} GHz  mfma_util {util:5.1f}%  sq_busy {c.get('SQ_BUSY_CYCLES',0):.3g}")
PY
