# per-level eager breakdowns for option sets: scripts/gpu_bd.sh NAME@k=v@k=v ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%@*}; opts=""
  [ "$spec" != "$name" ] && opts=$(echo "${spec#*@}" | tr '@' ' ')
  timeout -k 10 300 python3 scripts/panel_breakdown.py 128 $opts > gpurun_out/bd_$name.txt 2>&1 || { tail -5 gpurun_out/bd_$name.txt; exit 1; }
  echo "breakdown $name done"
done
