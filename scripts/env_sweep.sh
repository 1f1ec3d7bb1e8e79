# Bench ms per factorization for values of one environment knob: env_sweep.sh VAR v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  env "$var=$v" timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sweep_$v.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sweep_$v.log') if l.startswith('{')][-1]); print('$var=$v', d['ms_per_step'], d['validation']['backward_error'])"
done
