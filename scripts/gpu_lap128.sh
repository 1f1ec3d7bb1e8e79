# 128^3 closed-block parity + full-size solve backward error (prints the numbers).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k lap128 -x -v -s --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_lap128.log 2>&1
rc=$?; echo "lap128 rc=$rc"; grep -E "lap128|passed|failed" gpurun_out/pytest_lap128.log
exit $rc
