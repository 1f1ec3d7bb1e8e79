set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sprof -o solve -- python3 scripts/solve_prof.py 128 > gpurun_out/solve_prof.log 2>&1 || exit $?
cat gpurun_out/solve_prof.log | grep solve
head -20 gpurun_out/sprof/solve_kernel_stats.csv | cut -c1-150
