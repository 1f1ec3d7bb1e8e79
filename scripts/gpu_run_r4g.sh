export TMPDIR=/tmp; mkdir -p gpurun_out
# CB / panel SYRK K loop with LDS-DMA operand stages (SC_GLDS) against the same build without
timeout -k 10 700 bash scripts/gpu.sh ab def glds glds2 || exit 1
# tiny dense: factor-twice probe and the LDS-resident variant
timeout -k 10 400 bash scripts/gpu.sh tiny td_p2 td_lds || exit 1
# distributed plan parity (slab pieces included)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider -k "partitioned" > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo pytest dist rc=$rc; tail -3 gpurun_out/pytest_dist.log; [ $rc -eq 0 ] || exit $rc
echo done
