# Distributed panels: multi-rank protocol tests on one GPU (emulated + multi-process
# host transport), RCCL self send/recv emulation, then the per-rank 128^3 projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_parity.py -k "partition or multiprocess" -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo "pytest dist rc=$rc"; tail -22 gpurun_out/pytest_dist.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/rccl_emul.py 20 > gpurun_out/rccl_emul.log 2>&1
rc=$?; echo "rccl rc=$rc"; grep '^{' gpurun_out/rccl_emul.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/dist_project.py > gpurun_out/project.log 2>&1
rc=$?; echo "project rc=$rc"; grep '^{' gpurun_out/project.log
exit $rc
