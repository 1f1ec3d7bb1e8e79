set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "panel_schedule" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cbslab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_cbslab.log
[ $rc -eq 0 ] || exit $rc
for o in "" "--opt cb_slab=1" "--opt cb_slab=1 --nbo 512" "--opt cb_slab=1 --nbo 2048"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-solve $o > gpurun_out/cbslab.log 2>&1 || exit $?
  echo "opts [$o]"; grep '^{' gpurun_out/cbslab.log | python3 scripts/summarize.py
done
