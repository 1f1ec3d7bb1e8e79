# Default-parameter sweep at 128^3 (one bench line per setting).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/sweep2.txt
run() {
  timeout -k 10 240 python bench.py --steps 2 --no-cpu-baseline --no-solve "$@" > gpurun_out/sw.log 2>&1 || return $?
  echo "$* :: $(grep '^{' gpurun_out/sw.log | python3 scripts/summarize.py)" | tee -a gpurun_out/sweep2.txt
}
run || exit $?
run --nbo 768 || exit $?
run --nbo 1280 || exit $?
run --nbo 1536 || exit $?
run --opt small_front_max=96 || exit $?
run --opt small_front_max=64 || exit $?
run --opt asm_tile_min_m=4096 || exit $?
run --opt asm_tile_min_m=16384 || exit $?
run --opt nrelax=8,32,64 || exit $?
run --opt nrelax=4,16,32 || exit $?
run --opt zrelax=0.8,0.1,0.02 || exit $?
run --opt zrelax=0.8,0.2,0.08 || exit $?
run --relax-wmax 0 || exit $?
run --opt inner_order=0 || exit $?
run || exit $?
