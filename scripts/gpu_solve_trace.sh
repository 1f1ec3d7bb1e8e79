# Solve timing (graph vs eager) and a kernel trace of the solve at 128^3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/solve_modes.py 128 2>&1 | grep -v amdgpu || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/solve_prof -o s -- python3 scripts/solve_modes.py 128 > gpurun_out/solve_prof.log 2>&1 || exit $?
find gpurun_out/solve_prof -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-4 | grep -i "solve\|permute"
