# Round profile: rocprofv3 kernel stats of the default bench (graph replay) and the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_default.log | python3 scripts/summarize.py
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit $?
ls gpurun_out/prof
