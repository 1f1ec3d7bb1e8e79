# 128^3 closed-block parity + solve, SYRK BK probe, full GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k lap128 -x -v --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_lap128.log 2>&1
rc=$?; echo "lap128 rc=$rc"; tail -4 gpurun_out/pytest_lap128.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/syrk_bk_probe.py > gpurun_out/bk_probe.log 2>&1
rc2=$?; echo "bk rc=$rc2"; cat gpurun_out/bk_probe.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc3=$?; echo "suite rc=$rc3"; tail -4 gpurun_out/pytest_gpu.log
exit $rc3
