# N-GPU projections of option sets on the one GPU: scripts/gpu_proj.sh NAME@k=v@k=v ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%@*}; opts=()
  if [ "$spec" != "$name" ]; then
    IFS='@' read -ra kv <<< "${spec#*@}"
    for o in "${kv[@]}"; do opts+=(--opt "$o"); done
  fi
  timeout -k 10 560 python3 -u scripts/dist_project.py --n 8 --timeline "${opts[@]}" > gpurun_out/proj_$name.log 2>&1 || { tail -5 gpurun_out/proj_$name.log; exit 1; }
  python3 -c "
import json,sys
d=[json.loads(l) for l in open('gpurun_out/proj_$name.log') if l.startswith('{')][-1]
print('$name', 'dry max', d['max_rank_ms'], 'cp50', d.get('max_critical_path_ms_50GBs'), 'cp100', d.get('max_critical_path_ms_100GBs'), 'wait', d.get('critical_path_explained_50GBs',{}).get('totals'))"
done
