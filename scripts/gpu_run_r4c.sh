export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rP --timeout 600 --timeout-method thread -p no:cacheprovider -k "partitioned_defaults_lap64 or lap128_emulated8 or la_grid or split_fronts_emulated or bitwise_equal" > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pytest_dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/gemm_probe.py > gpurun_out/gemm_probe.jsonl 2>&1 || exit 1
echo gemm probe done
timeout -k 10 600 bash scripts/gpu_ab.sh base la_grid=448 la_grid=480 la_grid=384 || exit 1
