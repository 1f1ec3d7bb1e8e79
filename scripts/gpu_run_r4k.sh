export TMPDIR=/tmp; mkdir -p gpurun_out
# the whole GPU suite and one default bench line (the round-end driver runs the same)
timeout -k 10 1100 bash scripts/gpu.sh suite
