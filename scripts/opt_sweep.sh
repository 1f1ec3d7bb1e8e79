# Bench ms per factorization for option sets: opt_sweep.sh "xlevel=0" "xlevel=1 panel_nb_outer=512" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for set in "$@"; do
  args=""
  for kv in $set; do args="$args --opt $kv"; done
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline $args > gpurun_out/osweep_$i.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/osweep_$i.log') if l.startswith('{')][-1]); print('$set', d['ms_per_step'], d['validation']['backward_error'])"
  i=$((i+1))
done
