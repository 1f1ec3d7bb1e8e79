set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "chain" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_chain.log 2>&1
rc=$?; echo "pytest chain rc=$rc"; tail -8 gpurun_out/pytest_chain.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/small_configs.py > gpurun_out/small_configs.jsonl 2> gpurun_out/small_configs.err || exit $?
cat gpurun_out/small_configs.jsonl
