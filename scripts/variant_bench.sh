# A/B bench of the variant packages built by build_variants.sh (interleaved, twice each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    timeout -k 10 300 python3 gpurun_var/$v/bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/var_$v.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/var_$v.log') if l.startswith('{')][-1]); print('$v', d['ms_per_step'], d['roofline']['achieved'], d['validation']['backward_error'])"
  done
done
