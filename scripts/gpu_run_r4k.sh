export TMPDIR=/tmp; mkdir -p gpurun_out
# short-K CB launch shapes (levels 4-9): lean instance for K <= 64, 64-tiles below K = 256
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "panel_schedule and (cb_lean_kmin or cb_small_kmax)" > gpurun_out/pytest_cbk.log 2>&1
rc=$?; echo pytest cbk rc=$rc; tail -2 gpurun_out/pytest_cbk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/gpu_ab.sh base cb_lean_kmin=0 cb_small_kmax=256 || exit 1
timeout -k 10 300 python3 scripts/panel_breakdown.py 128 > gpurun_out/breakdown_final.txt 2>&1 || exit 1
echo done
