export TMPDIR=/tmp; mkdir -p gpurun_out
# round-4 evidence: bench + kernel stats, HBM traffic counters, MFMA utilisation
timeout -k 10 500 bash scripts/gpu.sh profile || exit 1
timeout -k 10 400 bash scripts/gpu.sh pmc || exit 1
timeout -k 10 300 bash scripts/gpu.sh mfma || exit 1
echo done
