export TMPDIR=/tmp; mkdir -p gpurun_out
# bench.py's N > 1 branch on the one GPU with the round-4 defaults (distributed assembly, slab
# pieces): host-staged transport (real multi-process protocol) and dry
timeout -k 10 900 bash scripts/gpu.sh rehearse 64 2 4
