export TMPDIR=/tmp; mkdir -p gpurun_out
# 8-rank critical-path projection, whole-slab vs pieced hand-over, eager vs graph
timeout -k 10 400 python -u scripts/dist_project.py --k 128 --n 8 --reps 2 --timeline --graph --opt dist_pieces=1 > gpurun_out/proj_p1.log 2>&1 || { tail -5 gpurun_out/proj_p1.log; exit 1; }
timeout -k 10 400 python -u scripts/dist_project.py --k 128 --n 8 --reps 2 --timeline --graph > gpurun_out/proj_p4.log 2>&1 || { tail -5 gpurun_out/proj_p4.log; exit 1; }
echo done
