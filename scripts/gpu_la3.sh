set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/la3.txt
run() {
  timeout -k 10 240 python bench.py --steps 2 --no-cpu-baseline --no-solve "$@" > gpurun_out/sw.log 2>&1 || return $?
  echo "$* :: $(grep '^{' gpurun_out/sw.log | python3 scripts/summarize.py)" | tee -a gpurun_out/la3.txt
}
run || exit $?
run --lookahead 3 || exit $?
run --lookahead 3 --panel-variant 3 || exit $?
run --lookahead 0 || exit $?
