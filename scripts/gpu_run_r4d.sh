export TMPDIR=/tmp; mkdir -p gpurun_out
# panel modes 3/4 and per-slab CB updates: parity, then their A/B against the default
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "(panel_schedule and (tall or cb_slab)) or (lap48_full and (cb_by_slab or two_level or default))" > gpurun_out/pytest_tall3.log 2>&1
rc=$?; echo pytest tall rc=$rc; tail -2 gpurun_out/pytest_tall3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash scripts/gpu_ab.sh base panel_tall=3,la_grid=448 panel_tall=4,la_grid=448 cb_slab=1,la_grid=448 cb_slab=1 || exit 1
timeout -k 10 300 python3 scripts/panel_breakdown.py 128 > gpurun_out/breakdown.txt 2>&1 || exit 1
echo breakdown done
echo done
