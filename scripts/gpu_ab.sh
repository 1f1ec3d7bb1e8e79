# Interleaved A/B of sc_options variants on the in-tree build (two rounds):
#   bash scripts/gpu_ab.sh "opt=val[,opt=val...]" ...   ("base" = defaults)
# prints "<variant> ms GF/s cb_TF/s backward_error" per run; logs in gpurun_out/ab_*.log
export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do
  for spec in "$@"; do
    opts=()
    if [ "$spec" != "base" ]; then IFS=',' read -ra kv <<< "$spec"; for o in "${kv[@]}"; do opts+=(--opt "$o"); done; fi
    tag=$(echo "$spec" | tr '=,' '__')
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-solve "${opts[@]}" > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_$tag.log') if l.startswith('{')][-1]); print('$spec', d['ms_per_step'], d['value'], d['roofline']['achieved'], d['validation']['backward_error'])"
  done
done
