export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python scripts/contention_probe.py resident > gpurun_out/contention_resident.jsonl 2> gpurun_out/contention_resident.err || { echo probe failed; tail gpurun_out/contention_resident.err; exit 1; }
echo probe done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rP --timeout 600 --timeout-method thread -p no:cacheprovider -k "partitioned or lap128_emulated8" > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/pytest_dist.log; exit $rc
