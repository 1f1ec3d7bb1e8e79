# GPU parity suite + one default bench line (run through gpurun from the repo root).
#   scripts/gpu_suite.sh [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then SEL=(-k "$K"); else SEL=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "${SEL[@]}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json
exit $rc
