export TMPDIR=/tmp; mkdir -p gpurun_out
# distributed plan parity (slab pieces included)
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider -k "partitioned" > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo pytest dist rc=$rc; tail -3 gpurun_out/pytest_dist.log; [ $rc -eq 0 ] || exit $rc
# 8-rank critical-path projection, whole-slab vs pieced hand-over, eager vs graph
timeout -k 10 300 python -u scripts/dist_project.py --k 128 --n 8 --reps 2 --timeline --graph --opt dist_pieces=1 > gpurun_out/proj_p1.log 2>&1 || { tail -5 gpurun_out/proj_p1.log; exit 1; }
timeout -k 10 300 python -u scripts/dist_project.py --k 128 --n 8 --reps 2 --timeline --graph > gpurun_out/proj_p4.log 2>&1 || { tail -5 gpurun_out/proj_p4.log; exit 1; }
echo done
