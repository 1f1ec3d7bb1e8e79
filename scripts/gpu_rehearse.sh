# bench.py's N>1 branch on the one GPU of the box: torch.distributed.run with the
# host-staged transport (GlooHostTransport) and the dry transport, several ranks per GPU.
#   scripts/gpu_rehearse.sh [k] [ranks...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
K=${1:-48}; shift || true
RANKS=${@:-2 4}
for n in $RANKS; do
  for tr in host dry; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 3 --warmup 1 --k $K --transport $tr \
      > gpurun_out/rehearse_k${K}_n${n}_${tr}.log 2>&1 || { echo "rehearsal n=$n $tr failed"; tail -20 gpurun_out/rehearse_k${K}_n${n}_${tr}.log; exit 1; }
    grep '^{' gpurun_out/rehearse_k${K}_n${n}_${tr}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, '$tr', d['n_gpus'], d['ms_per_step'], d['value'], d['validation']['backward_error'], d['config']['work_share_per_rank'])"
  done
done
