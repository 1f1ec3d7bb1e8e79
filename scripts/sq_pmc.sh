cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -f csv -d gpurun_out/sqpmc -o sq -- python3 bench.py --graph 0 --steps 1 --warmup 0 --no-cpu-baseline --no-solve > gpurun_out/sqpmc.log 2>&1
