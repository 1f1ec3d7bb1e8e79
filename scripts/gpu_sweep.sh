# Parameter sweep of the 128^3 bench (no CPU baseline).  Usage: bash scripts/gpu_sweep.sh "<args1>" "<args2>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --k 128 --steps 2 --warmup 1 --no-cpu-baseline $a > gpurun_out/sweep_$i.log 2>&1
  rc=$?
  echo "[$a] rc=$rc $(grep '^{' gpurun_out/sweep_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"] if d["roofline"] else None, [round(x,1) for x in d["phase_ms"]])' 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/sweep_$i.log; exit $rc; fi
done
