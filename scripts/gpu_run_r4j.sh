export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "panel_schedule and la_split" > gpurun_out/pytest_las.log 2>&1
rc=$?; echo pytest las rc=$rc; tail -2 gpurun_out/pytest_las.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash scripts/gpu_ab.sh base la_split=2 la_split=4 || exit 1

timeout -k 10 400 python -u scripts/dist_project.py --k 128 --n 8 --reps 2 --timeline --opt dist_pieces=2 > gpurun_out/proj_p2.log 2>&1 || { tail -5 gpurun_out/proj_p2.log; exit 1; }
grep '^{' gpurun_out/proj_p2.log
echo done
