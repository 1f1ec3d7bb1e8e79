export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "panel_schedule and la_streams" > gpurun_out/pytest_lst.log 2>&1
rc=$?; echo pytest lst rc=$rc; tail -2 gpurun_out/pytest_lst.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/gpu_ab.sh base la_streams=2 la_streams=4 || exit 1
echo done
