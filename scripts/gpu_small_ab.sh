# Interleaved small-config timings of library variants (gpurun_var/NAME/.../libsparsecholesky_amd.so):
#   bash scripts/gpu_small_ab.sh NAME ...   -> gpurun_out/small_NAME_REP.jsonl, one summary line each
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    SC_LIB=$PWD/gpurun_var/$v/sparsecholesky_amd/libsparsecholesky_amd.so timeout -k 10 300 python3 scripts/small_configs.py \
      > gpurun_out/small_${v}_$rep.jsonl 2> gpurun_out/small_${v}_$rep.err || { tail -5 gpurun_out/small_${v}_$rep.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/small_${v}_$rep.jsonl'):
    d = json.loads(l); print('$v', d['matrix'], d['gpu_ms_c_eager'], d['gpu_ms_c_graph'], d['levels'], '%.2e' % d['rel_fro_vs_oracle'])"
  done
done
