export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_probe.py > gpurun_out/gemm_probe.jsonl 2>&1 || { tail -3 gpurun_out/gemm_probe.jsonl; exit 1; }
echo gemm probe done
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "panel_schedule and tall" > gpurun_out/pytest_tall3.log 2>&1
rc=$?; echo pytest tall rc=$rc; tail -2 gpurun_out/pytest_tall3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash scripts/gpu_ab.sh base panel_tall=3,la_grid=448 panel_tall=4,la_grid=448 panel_tall=3 la_grid=448 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider -k "lap48_full or partitioned_defaults_lap64 or lap128_emulated8 or split_fronts_emulated" > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pytest_dist.log; exit $rc
