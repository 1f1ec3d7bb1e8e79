# A/B: hardware queues per process vs the extra-stream penalty.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/hwq8.log 2>&1 || exit $?
echo "hwq8"; grep '^{' gpurun_out/hwq8.log | python3 scripts/summarize.py
GPU_MAX_HW_QUEUES=8 SC_EXTRA_STREAM=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/hwq8_extra.log 2>&1 || exit $?
echo "hwq8 extra"; grep '^{' gpurun_out/hwq8_extra.log | python3 scripts/summarize.py
GPU_MAX_HW_QUEUES=16 SC_EXTRA_STREAM=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/hwq16_extra.log 2>&1 || exit $?
echo "hwq16 extra"; grep '^{' gpurun_out/hwq16_extra.log | python3 scripts/summarize.py
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u scripts/dist_project.py --n 8 > gpurun_out/hwq8_proj.log 2>&1 || exit $?
echo "hwq8 projection"; grep '^{' gpurun_out/hwq8_proj.log
