export TMPDIR=/tmp; mkdir -p gpurun_out
# 128-tile gather: relative indices staged in LDS (in-tree build = lib_stage)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "lap48_full or lap64_full" > gpurun_out/pytest_stage.log 2>&1
rc=$?; echo pytest stage rc=$rc; tail -2 gpurun_out/pytest_stage.log; [ $rc -eq 0 ] || exit $rc
L=sparsecholesky_amd
for rep in 1 2; do
  for v in base stage stage_q2 stage_occ3; do
    cp $L/lib_$v.so $L/libsparsecholesky_amd.so
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-solve > gpurun_out/ab_g_$v.log 2>&1 || { tail -5 gpurun_out/ab_g_$v.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab_g_$v.log') if l.startswith('{')][-1]); print('$v', d['ms_per_step'], d['roofline']['achieved'], d['validation']['backward_error'])"
  done
done
cp $L/lib_stage.so $L/libsparsecholesky_amd.so
timeout -k 10 300 python3 scripts/panel_breakdown.py 128 > gpurun_out/breakdown_stage.txt 2>&1 || exit 1
cp $L/lib_base.so $L/libsparsecholesky_amd.so
timeout -k 10 300 python3 scripts/panel_breakdown.py 128 > gpurun_out/breakdown_base.txt 2>&1 || exit 1
echo done
