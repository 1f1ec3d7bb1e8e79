# A/B of the comm-stream priority on one rank's projected time (8 ranks, ranks 0 and 7),
# then the PMC HBM-traffic passes of the CB SYRK.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for pv in 0 1 2; do
  SC_COMM_PRIO=$pv timeout -k 10 300 python -u scripts/dist_project.py --n 8 > gpurun_out/prio_$pv.log 2>&1 || exit $?
  echo "prio $pv"; grep '^{' gpurun_out/prio_$pv.log
done
bash scripts/gpu_pmc.sh
