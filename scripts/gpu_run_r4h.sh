export TMPDIR=/tmp; mkdir -p gpurun_out
# bisect the 20^3 two-rank partitioned parity failure
for p in gpurun_var/at_6011b72 gpurun_var/at_1c28b07 gpurun_var/at_043c6f8 .; do
  timeout -k 10 120 python3 scripts/dist_case.py $p 20 2 >> gpurun_out/dist_case.log 2>&1 || { tail -3 gpurun_out/dist_case.log; exit 1; }
done
timeout -k 10 120 python3 scripts/dist_case.py . 20 2 dist_pieces=1 >> gpurun_out/dist_case.log 2>&1 || exit 1
timeout -k 10 120 python3 scripts/dist_case.py . 20 2 dist_asm=0 >> gpurun_out/dist_case.log 2>&1 || exit 1
timeout -k 10 120 python3 scripts/dist_case.py . 20 4 >> gpurun_out/dist_case.log 2>&1 || exit 1
cat gpurun_out/dist_case.log
# four-stage LDS-DMA K loop against the same build without
timeout -k 10 500 bash scripts/gpu.sh ab def glds2 || exit 1
echo done
