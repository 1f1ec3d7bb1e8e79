set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for o in "--lookahead 1" "--lookahead 4" "--lookahead 5" "--lookahead 2" "--lookahead 1"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-solve $o > gpurun_out/la.log 2>&1 || exit $?
  echo "opts [$o]"; grep '^{' gpurun_out/la.log | python3 scripts/summarize.py
done
