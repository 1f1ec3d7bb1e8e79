set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "solve" -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_solve.log 2>&1
rc=$?; echo "pytest solve rc=$rc"; tail -15 gpurun_out/pytest_solve.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['solve'])"
exit $rc
