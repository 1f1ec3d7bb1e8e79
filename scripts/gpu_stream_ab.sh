# A/B: does an idle extra stream (and its priority) slow the single-GPU factorization?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_none.log 2>&1 || exit $?
echo none; grep '^{' gpurun_out/ab_none.log | python3 scripts/summarize.py
for pv in 0 1 2; do
  SC_EXTRA_STREAM=1 SC_COMM_PRIO=$pv timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_$pv.log 2>&1 || exit $?
  echo "extra prio $pv"; grep '^{' gpurun_out/ab_$pv.log | python3 scripts/summarize.py
done
