# MFMA utilisation and effective clock of every kernel of one eager 128^3 bench step,
# normalised by the register-only fp64 MFMA probe (100% MFMA by construction).
# Counters: SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE (one pass each
# program, kernel trace only); summary -> gpurun_out/mfma_util.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -k 10 300 python3 scripts/mfma_probe.py > gpurun_out/mfma_probe.log 2>&1 || exit $?
cat gpurun_out/mfma_probe.log
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -f csv -d gpurun_out/pmc_probe -o pr -- \
  python3 scripts/mfma_probe.py --probe-only > gpurun_out/pmc_probe.log 2>&1 || exit $?
timeout -s KILL 600 rocprofv3 --pmc $C --kernel-trace -f csv -d gpurun_out/pmc_step -o st -- \
  python3 bench.py --graph 0 --steps 1 --warmup 0 --no-cpu-baseline --no-solve > gpurun_out/pmc_step.log 2>&1 || exit $?
python3 scripts/mfma_util_summary.py gpurun_out/pmc_probe gpurun_out/pmc_step > gpurun_out/mfma_util.json || exit $?
cat gpurun_out/mfma_util.json
