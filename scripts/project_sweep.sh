# N = 8 projection (dry ranks + critical-path replay) for several option sets, one log each:
#   bash scripts/project_sweep.sh NAME@k=v@k=v ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  v=${spec%%@*}
  opts=()
  if [ "$spec" != "$v" ]; then
    IFS='@' read -ra kv <<< "${spec#*@}"
    for o in "${kv[@]}"; do opts+=(--opt "$o"); done
  fi
  timeout -k 10 600 python -u scripts/dist_project.py --n 8 --reps 1 --timeline "${opts[@]}" > gpurun_out/proj_$v.log 2>&1 || { tail -5 gpurun_out/proj_$v.log; exit 1; }
  echo "== $spec"; grep -E '^\{' gpurun_out/proj_$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    keys=[k for k in d if 'critical' in k or 'dry' in k or 'max' in k]
    print({k:(d[k] if not isinstance(d[k],dict) else {kk:vv for kk,vv in d[k].items() if not isinstance(vv,(list,dict))}) for k in keys})
"
done
