# Multi-GPU protocol checks on one GPU: emulated partitions and multi-process host transport,
# then the single-GPU parity suite and a default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_parity.py -k "partition or multiprocess" -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo "pytest dist rc=$rc"; tail -15 gpurun_out/pytest_dist.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | python3 scripts/summarize.py
exit $rc
