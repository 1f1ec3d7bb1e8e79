# Single-GPU bench (after the comm-stream fix) and the per-rank N-GPU projections.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | python3 scripts/summarize.py
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/dist_project.py > gpurun_out/project.log 2>&1
rc=$?; echo "project rc=$rc"; grep '^{' gpurun_out/project.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/dist_project.py --opt dist_split=0 > gpurun_out/project_nosplit.log 2>&1
rc=$?; echo "project nosplit rc=$rc"; grep '^{' gpurun_out/project_nosplit.log
exit $rc
