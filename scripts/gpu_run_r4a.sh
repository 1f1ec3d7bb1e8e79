export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python scripts/contention_probe.py > gpurun_out/contention.jsonl 2> gpurun_out/contention.err || { echo probe failed; tail gpurun_out/contention.err; exit 1; }
echo probe done
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rP --timeout 400 --timeout-method thread -p no:cacheprovider -k "tall or tiny or dense or readme or panel_schedule or reference_matrices" > gpurun_out/pytest_tall.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pytest_tall.log; [ $rc -eq 0 ] || exit $rc
for o in 0 2 0 2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --opt panel_tall=$o > gpurun_out/ab_tall$o.log 2>&1 || { tail -5 gpurun_out/ab_tall$o.log; exit 1; }
  echo "tall=$o $(grep '^{' gpurun_out/ab_tall$o.log | tail -1 | python3 scripts/summarize.py)"
done
timeout -k 10 300 python scripts/panel_breakdown.py 128 panel_tall=2 > gpurun_out/breakdown_tall2.txt 2>&1 || exit 1
echo breakdown done
