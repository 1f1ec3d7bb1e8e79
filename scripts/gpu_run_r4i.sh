export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/dist_case.py . 20 2 > gpurun_out/dist_case.log 2>&1 || { cat gpurun_out/dist_case.log; exit 1; }
cat gpurun_out/dist_case.log
# left-looking lookahead stream (lookahead = 3): parity, then A/B against the default
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "(panel_schedule and lookahead) or left_looking_lookahead" > gpurun_out/pytest_ll3.log 2>&1
rc=$?; echo pytest ll3 rc=$rc; tail -2 gpurun_out/pytest_ll3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash scripts/gpu_ab.sh base lookahead=3 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dist_gpu.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider -k "partitioned or dist" > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo pytest dist rc=$rc; tail -3 gpurun_out/pytest_dist.log; exit $rc
