# Parameter sweep of the bench (no CPU baseline).  Usage: bash scripts/gpu_sweep.sh "<args1>" "<args2>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $a > gpurun_out/sweep_$i.log 2>&1
  rc=$?
  echo "[$a] rc=$rc $(grep '^{' gpurun_out/sweep_$i.log | python3 scripts/summarize.py 2>&1)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/sweep_$i.log; exit $rc; fi
done
