# Per-level eager breakdown (scripts/panel_breakdown.py) of variant packages.
#   scripts/gpu_breakdown_ab.sh VARIANT [VARIANT ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 300 python3 gpurun_var/$v/scripts/panel_breakdown.py 128 > gpurun_out/breakdown_$v.txt 2>&1 || exit $?
  echo "breakdown $v done"
done
