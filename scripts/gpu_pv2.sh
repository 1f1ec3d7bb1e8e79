set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/pv2.txt
run() {
  timeout -k 10 240 python bench.py --steps 2 --no-cpu-baseline --no-solve "$@" > gpurun_out/sw.log 2>&1 || return $?
  echo "$* :: $(grep '^{' gpurun_out/sw.log | python3 scripts/summarize.py)" | tee -a gpurun_out/pv2.txt
}
run || exit $?
run --panel-variant 2 || exit $?
run --panel-variant 2 --lookahead 3 || exit $?
run --panel-variant 2 --nbo 512 || exit $?
run || exit $?
