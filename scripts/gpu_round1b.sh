# GPU run: parity tests, then a rocprofv3 kernel-trace profile of the 128^3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof128 -o k128 -- python3 bench.py --k 128 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench128_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/bench128_prof.log
find gpurun_out/prof128 -name "*stats*" | head
exit $rc
