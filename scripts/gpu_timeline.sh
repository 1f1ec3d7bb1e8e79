# Kernel timeline of an eager 128^3 factorization (rocprofv3 kernel trace) -> chain analysis.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -f csv -d gpurun_out/tl -o tl -- python3 bench.py --graph 0 --steps 1 --warmup 1 --no-cpu-baseline --no-solve > gpurun_out/tl.log 2>&1 || exit $?
python3 scripts/chain_timeline.py gpurun_out/tl/tl_kernel_trace.csv
