# round-6 GPU tasks (run through gpurun from the repo root)
#   scripts/gpu_r6.sh tests EXPR         pytest -m gpu -k EXPR
#   scripts/gpu_r6.sh ab SPEC...         interleaved option A/B (scripts/gpu.sh abopt)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
task=$1; shift
case "$task" in
  tests)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
      -k "$1" > gpurun_out/pytest_r6.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r6.log; exit $rc ;;
  testsab)
    expr=$1; shift
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
      -k "$expr" > gpurun_out/pytest_r6.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r6.log; [ $rc -eq 0 ] || exit $rc
    bash scripts/gpu.sh abopt "$@" ;;
  *) echo "unknown task"; exit 2 ;;
esac
