# HBM traffic of the CB SYRK (roofline.traffic): FETCH_SIZE and WRITE_SIZE in two
# separate rocprofv3 --pmc passes (they do not fit one pass on gfx950), kernel trace
# only, on an eager (non-graph) bench step so every dispatch is attributed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -f csv -d gpurun_out/pmc_$c -o pmc -- \
    python3 bench.py --graph 0 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1 || exit $?
done
python3 scripts/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > gpurun_out/pmc_summary.json
cat gpurun_out/pmc_summary.json
