set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --k 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench64.log 2>&1
rc=$?; echo "bench64 rc=$rc"; tail -5 gpurun_out/bench64.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --k 128 --steps 2 --warmup 1 > gpurun_out/bench128.log 2>&1
rc=$?; echo "bench128 rc=$rc"; tail -5 gpurun_out/bench128.log
exit $rc
