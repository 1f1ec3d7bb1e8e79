# Kernel-trace stats of one graph-replayed bench step per variant (gpurun_var/NAME), for
# kernel-level A/B:  bash scripts/kstats_ab.sh NAME [NAME ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kst_$v -o k -- \
    python3 gpurun_var/$v/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-solve > gpurun_out/kst_$v.log 2>&1 || exit $?
  python3 scripts/kstats_top.py gpurun_out/kst_$v > gpurun_out/kst_$v.txt || exit $?
  echo "== $v"; cat gpurun_out/kst_$v.txt
done
