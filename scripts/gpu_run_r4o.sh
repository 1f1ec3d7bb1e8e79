export TMPDIR=/tmp; mkdir -p gpurun_out
# resident lookahead grids in the default panel mode
timeout -k 10 700 bash scripts/gpu_ab.sh base la_grid=448 la_grid=496 la_grid=384 || exit 1
echo done
