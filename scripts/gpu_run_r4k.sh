export TMPDIR=/tmp; mkdir -p gpurun_out
# N=8 projection sweep of plan options around the round-4 defaults
for o in dist_slab_block=1 dist_slab_block=3 dist_pieces=3 dist_cbb=2048 dist_cbb=512; do
  timeout -k 10 300 python -u scripts/dist_project.py --k 128 --n 8 --reps 2 --timeline --opt $o > gpurun_out/proj_$o.log 2>&1 || { tail -5 gpurun_out/proj_$o.log; exit 1; }
  grep '^{' gpurun_out/proj_$o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$o', d['max_rank_ms'], d['max_rank_ms_with_comm_serial'], d['max_critical_path_ms_50GBs'], d['max_critical_path_ms_100GBs'])"
done
echo done
