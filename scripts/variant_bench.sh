# A/B bench of variant packages built by build_variants.sh (interleaved, twice each).
#   variant_bench.sh NAME[@key=val[@key=val...]] ...   (key=val: sc_options passed with --opt)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for spec in "$@"; do
    v=${spec%%@*}
    opts=()
    if [ "$spec" != "$v" ]; then
      IFS='@' read -ra kv <<< "${spec#*@}"
      for o in "${kv[@]}"; do opts+=(--opt "$o"); done
    fi
    tag=$(echo "$spec" | tr '@=,' '___')
    timeout -k 10 300 python3 gpurun_var/$v/bench.py --steps 5 --warmup 2 --no-cpu-baseline "${opts[@]}" > gpurun_out/var_$tag.log 2>&1 || { tail -5 gpurun_out/var_$tag.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/var_$tag.log') if l.startswith('{')][-1]); print('$spec', d['ms_per_step'], d['roofline']['achieved'], d['validation']['backward_error'])"
  done
done
