export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/dist_case.py . 20 2 > gpurun_out/dist_case.log 2>&1 || { cat gpurun_out/dist_case.log; exit 1; }
cat gpurun_out/dist_case.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dist_gpu.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider -k "partitioned or dist" > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo pytest dist rc=$rc; tail -3 gpurun_out/pytest_dist.log; exit $rc
