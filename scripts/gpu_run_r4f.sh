export TMPDIR=/tmp; mkdir -p gpurun_out
# left-looking slab updates (lookahead = 2): parity, A/B against the default and no lookahead
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "(panel_schedule and (lookahead or cb_gather_min_w)) or left_looking" > gpurun_out/pytest_ll.log 2>&1
rc=$?; echo pytest ll rc=$rc; tail -2 gpurun_out/pytest_ll.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/gpu_ab.sh base lookahead=2 lookahead=0 cb_gather_min_w=64 || exit 1
# tiny dense: parity, small configs, kernel durations of the variants
timeout -k 10 500 bash scripts/gpu.sh tiny td_old td_p1 td_p2 td_lds || exit 1
echo done
