# GPU-box tasks (run through gpurun from the repo root; every step has its own time
# limit and the first failure ends the call).
#   scripts/gpu.sh suite [pytest -k expr]   parity suite (-m gpu) + one default bench line
#   scripts/gpu.sh profile                  bench line + rocprofv3 kernel stats of the bench
#   scripts/gpu.sh pmc                      FETCH_SIZE / WRITE_SIZE passes -> pmc_summary.json
#   scripts/gpu.sh mfma                     MFMA-busy / clock counters -> mfma_util.json
#   scripts/gpu.sh breakdown [variant ...]  per-level eager breakdown (in-tree, or gpurun_var/<variant>)
#   scripts/gpu.sh ab SPEC ...              interleaved A/B bench of variants (build_variants.sh);
#                                           SPEC = NAME[@key=val[@key=val...]] (sc_options via --opt)
#   scripts/gpu.sh abopt SPEC ...           interleaved A/B bench of option sets on the in-tree build;
#                                           SPEC = NAME[@key=val[@key=val...]]
#   scripts/gpu.sh rehearse [k] [ranks...]  bench.py's N>1 branch on this one GPU (host / dry transport)
#   scripts/gpu.sh project [--opt k=v ...]  per-rank dry projection of the N-GPU plan + comm term
#   scripts/gpu.sh rccl                     emulated ranks over real RCCL send/recv to self, kernel trace
#   scripts/gpu.sh small                    small-config timings (bcsstk01, 1138_bus, lap 16^3 / 32^3)
#   scripts/gpu.sh solve                    solve parity tests + solve kernel trace at 128^3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
task=$1; shift || true
bench_line() {  # $1 = log file; prints the summary of its JSON line
  grep '^{' "$1" | tail -1 | python3 scripts/summarize.py
}
case "$task" in
  suite)
    if [ -n "$1" ]; then SEL=(-k "$1"); else SEL=(); fi
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
      -p no:cacheprovider "${SEL[@]}" > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
    [ $rc -ne 0 ] && exit $rc
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
    rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json
    exit $rc ;;
  profile)
    timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
    bench_line gpurun_out/bench_default.log
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o bench -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit $?
    ls gpurun_out/prof ;;
  pmc)
    # FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950: one pass each, kernel
    # trace only, on an eager step so every dispatch is attributed
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -f csv -d gpurun_out/pmc_$c -o pmc -- \
        python3 bench.py --graph 0 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1 || exit $?
    done
    python3 scripts/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > gpurun_out/pmc_summary.json || exit $?
    cat gpurun_out/pmc_summary.json ;;
  mfma)
    C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
    timeout -k 10 300 python3 scripts/mfma_probe.py > gpurun_out/mfma_probe.log 2>&1 || exit $?
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -f csv -d gpurun_out/pmc_probe -o pr -- \
      python3 scripts/mfma_probe.py --probe-only > gpurun_out/pmc_probe.log 2>&1 || exit $?
    timeout -s KILL 600 rocprofv3 --pmc $C --kernel-trace -f csv -d gpurun_out/pmc_step -o st -- \
      python3 bench.py --graph 0 --steps 1 --warmup 0 --no-cpu-baseline --no-solve > gpurun_out/pmc_step.log 2>&1 || exit $?
    python3 scripts/mfma_util_summary.py gpurun_out/pmc_probe gpurun_out/pmc_step > gpurun_out/mfma_util.json || exit $?
    cat gpurun_out/mfma_util.json ;;
  breakdown)
    if [ $# -eq 0 ]; then
      timeout -k 10 300 python3 scripts/panel_breakdown.py 128 > gpurun_out/breakdown.txt 2>&1 || exit $?
    fi
    for v in "$@"; do
      timeout -k 10 300 python3 gpurun_var/$v/scripts/panel_breakdown.py 128 > gpurun_out/breakdown_$v.txt 2>&1 || exit $?
      echo "breakdown $v done"
    done ;;
  ab)
    for rep in 1 2; do
      for spec in "$@"; do
        v=${spec%%@*}
        opts=()
        if [ "$spec" != "$v" ]; then
          IFS='@' read -ra kv <<< "${spec#*@}"
          for o in "${kv[@]}"; do opts+=(--opt "$o"); done
        fi
        tag=$(echo "$spec" | tr '@=,' '___')
        timeout -k 10 300 python3 gpurun_var/$v/bench.py --steps 5 --warmup 2 --no-cpu-baseline "${opts[@]}" \
          > gpurun_out/var_$tag.log 2>&1 || { tail -5 gpurun_out/var_$tag.log; exit 1; }
        python3 -c "import json; d=json.loads([l for l in open('gpurun_out/var_$tag.log') if l.startswith('{')][-1]); print('$spec', d['ms_per_step'], d['roofline']['achieved'], d['validation']['backward_error'])"
      done
    done ;;
  abopt)
    for rep in 1 2; do
      for spec in "$@"; do
        v=${spec%%@*}
        opts=()
        if [ "$spec" != "$v" ]; then
          IFS='@' read -ra kv <<< "${spec#*@}"
          for o in "${kv[@]}"; do opts+=(--opt "$o"); done
        fi
        timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "${opts[@]}" \
          > gpurun_out/abopt_${v}_$rep.log 2>&1 || { tail -5 gpurun_out/abopt_${v}_$rep.log; exit 1; }
        python3 -c "import json; d=json.loads([l for l in open('gpurun_out/abopt_${v}_$rep.log') if l.startswith('{')][-1]); print('$spec', d['ms_per_step'], d['roofline']['achieved'], d['validation']['backward_error'])"
      done
    done ;;
  rehearse)
    K=${1:-48}; shift || true
    RANKS=${@:-2 4}
    for n in $RANKS; do
      for tr in host dry; do
        timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
          --master-port $((29500 + n)) bench.py --gpus $n --steps 3 --warmup 1 --k $K --transport $tr \
          > gpurun_out/rehearse_k${K}_n${n}_${tr}.log 2>&1 || { echo "rehearsal n=$n $tr failed"; tail -20 gpurun_out/rehearse_k${K}_n${n}_${tr}.log; exit 1; }
        grep '^{' gpurun_out/rehearse_k${K}_n${n}_${tr}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, '$tr', d['n_gpus'], d['ms_per_step'], d['value'], d['validation']['backward_error'], d['config']['work_share_per_rank'])"
      done
    done ;;
  project)
    timeout -k 10 900 python -u scripts/dist_project.py "$@" > gpurun_out/project.log 2>&1
    rc=$?; echo "project rc=$rc"; grep '^{' gpurun_out/project.log; exit $rc ;;
  rccl)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_rccl -o rccl -- \
      python3 scripts/rccl_emul.py 20 > gpurun_out/rccl_emul.log 2>&1
    rc=$?; echo "rccl rc=$rc"; grep -v "^$" gpurun_out/rccl_emul.log | tail -8; exit $rc ;;
  small)
    timeout -k 10 600 python3 scripts/small_configs.py > gpurun_out/small_configs.jsonl 2> gpurun_out/small_configs.err
    rc=$?; echo "small rc=$rc"; cat gpurun_out/small_configs.jsonl; [ $rc -eq 0 ] || exit $rc
    # kernel durations of the same runs (tiny tree, small-front levels)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_small -o small -- \
      python3 scripts/small_configs.py > /dev/null 2> gpurun_out/small_prof.err ;;
  tiny)  # tiny-path parity, small configs, and the tiny kernel's duration per variant
    timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tiny or not_positive" -x -q --timeout 120 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tiny.log 2>&1
    rc=$?; echo "pytest tiny rc=$rc"; tail -3 gpurun_out/pytest_tiny.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python3 scripts/small_configs.py > gpurun_out/small_configs.jsonl 2> gpurun_out/small_configs.err
    rc=$?; cat gpurun_out/small_configs.jsonl; [ $rc -eq 0 ] || exit $rc
    for v in main "$@"; do
      pkg=.; [ "$v" != main ] && pkg=gpurun_var/$v
      nc=""; [ "$v" = td_p1 ] && nc=1
      TINY_NOCHECK=$nc timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_tiny_$v -o tiny -- \
        python3 scripts/tiny_probe.py $pkg > gpurun_out/tiny_$v.log 2>&1 || { tail -3 gpurun_out/tiny_$v.log; exit 1; }
      python3 - "$v" <<'EOF'
import csv, glob, sys
for f in glob.glob(f"gpurun_out/prof_tiny_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "tiny" in r["Name"]:
            print(sys.argv[1], r["Name"][:40], "calls", r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 2),
                  "min_us", round(float(r["MinNs"]) / 1e3, 2))
EOF
    done ;;
  solve)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "solve" -x -v --timeout 240 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_solve.log 2>&1
    rc=$?; echo "pytest solve rc=$rc"; tail -5 gpurun_out/pytest_solve.log
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/sprof -o solve -- \
      python3 scripts/solve_prof.py 128 > gpurun_out/solve_prof.log 2>&1 || exit $?
    grep solve gpurun_out/solve_prof.log ;;
  *)
    echo "unknown task '$task' (see the header of scripts/gpu.sh)"; exit 2 ;;
esac
