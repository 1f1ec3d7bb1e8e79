export TMPDIR=/tmp; mkdir -p gpurun_out
# 64-tile gather: first segment batch prefetched under the K loop (in-tree build = lib_pf)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "lap48_full or lap64_full or cb_lean_kmin or cb_small_kmax or cb_gather" > gpurun_out/pytest_pf.log 2>&1
rc=$?; echo pytest pf rc=$rc; tail -2 gpurun_out/pytest_pf.log; [ $rc -eq 0 ] || exit $rc
L=sparsecholesky_amd
for rep in 1 2; do
  for v in base pf pfnl; do
    cp $L/lib_$v.so $L/libsparsecholesky_amd.so
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-solve > gpurun_out/ab_g_$v.log 2>&1 || { tail -5 gpurun_out/ab_g_$v.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_g_$v.log') if l.startswith('{')][-1]); print('$v', d['ms_per_step'], d['roofline']['achieved'], d['validation']['backward_error'])"
  done
done
cp $L/lib_pf.so $L/libsparsecholesky_amd.so
timeout -k 10 300 python3 scripts/panel_breakdown.py 128 > gpurun_out/breakdown_pf.txt 2>&1 || exit 1
cp $L/lib_base.so $L/libsparsecholesky_amd.so
timeout -k 10 300 python3 scripts/panel_breakdown.py 128 > gpurun_out/breakdown_base.txt 2>&1 || exit 1
echo done
