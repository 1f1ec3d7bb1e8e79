# A/B: extra-stream penalty in eager mode (multi-GPU ranks run eager) vs graph replay.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --graph 0 --no-cpu-baseline > gpurun_out/eager.log 2>&1 || exit $?
echo "eager"; grep '^{' gpurun_out/eager.log | python3 scripts/summarize.py
SC_EXTRA_STREAM=1 timeout -k 10 300 python bench.py --graph 0 --no-cpu-baseline > gpurun_out/eager_extra.log 2>&1 || exit $?
echo "eager extra"; grep '^{' gpurun_out/eager_extra.log | python3 scripts/summarize.py
