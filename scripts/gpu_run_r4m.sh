export TMPDIR=/tmp; mkdir -p gpurun_out
# N=8 projection of the current build for 1, 2 and 4 slab pieces (the dist_pieces default)
for p in 1 2 4; do
  timeout -k 10 300 python -u scripts/dist_project.py --k 128 --n 8 --reps 2 --timeline --opt dist_pieces=$p > gpurun_out/proj_cur_p$p.log 2>&1 || { tail -5 gpurun_out/proj_cur_p$p.log; exit 1; }
  grep '^{' gpurun_out/proj_cur_p$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($p, d['max_rank_ms'], d['max_rank_ms_with_comm_serial'], d['max_critical_path_ms_50GBs'], d['max_critical_path_ms_100GBs'])"
done
echo done
