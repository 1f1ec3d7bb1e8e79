# RCCL send/recv path on the one-GPU box: the emulated multi-rank plan with RCCL
# self transfers, under a kernel trace (RCCL kernels listed in the stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_rccl -o rccl -- \
  python3 scripts/rccl_emul.py 20 > gpurun_out/rccl_emul.log 2>&1
rc=$?; echo "rccl rc=$rc"; cat gpurun_out/rccl_emul.log | grep -v "^$" | tail -8
find gpurun_out/prof_rccl -name "*kernel_stats.csv" | head -3
exit $rc
