set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "panel or lap48_full or solve or reference or tiny or not_positive or laplacian" > gpurun_out/pytest_pf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pf.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu.sh abopt pf1@panel_prefactor=1 pf0@panel_prefactor=0
