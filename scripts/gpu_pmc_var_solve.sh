# FETCH_SIZE / WRITE_SIZE passes (one eager step) of library variants: scripts/gpu_pmc_var.sh NAME ...
#   -> gpurun_out/pmcs_NAME.json (scripts/pmc_summary.py); one summary line for the CB SYRK each
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -f csv -d gpurun_out/pmcs_${v}_$c -o pmc -- \
      python3 gpurun_var/$v/bench.py --graph 0 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcs_${v}_$c.log 2>&1 || exit 1
  done
  python3 scripts/pmc_summary.py gpurun_out/pmcs_${v}_FETCH_SIZE gpurun_out/pmcs_${v}_WRITE_SIZE > gpurun_out/pmcs_$v.json || exit 1
  python3 -c "
import json
d = json.load(open('gpurun_out/pmcs_$v.json'))['kernels']
for k, x in d.items():
    if 'syrk_mfma_kernel<128, 2, 4, 1, 0' in k: print('$v', k[:48], x['launches'], round(x['fetch_bytes_per_launch'] / 1e9, 3), round(x['write_bytes_per_launch'] / 1e9, 3))"
done
