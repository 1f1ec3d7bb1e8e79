# Fused forward solve: solve parity tests, then bench (solve ms) without the CPU baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "solve or lap128" -x -v -s --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_solve_fused.log 2>&1
rc=$?; echo "solve tests rc=$rc"; grep -E "lap128|passed|failed|FAIL" gpurun_out/pytest_solve_fused.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_solve_fused.json 2> gpurun_out/bench_solve_fused.err
rc=$?; echo "bench rc=$rc"
python -c "import json; d=json.load(open('gpurun_out/bench_solve_fused.json')); print(d['ms_per_step'], d['solve'])"
exit $rc
