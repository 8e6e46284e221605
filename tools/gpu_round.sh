# GPU-box runner for a round's checks, profiles and A/B runs (dev tool; replaces the
# round-specific r04_*.sh / r05_*.sh runners).  Every GPU step has its own time limit and
# the steps stop at the first failure.  Outputs under gpurun_out/ (TAG in the file names).
#
#   bash tools/gpu_round.sh check TAG         -m gpu suite, one evaluation's phases at n = 16384 /
#                                              4096, small-n times, row-block P = 1 / 2 timings
#   bash tools/gpu_round.sh suite TAG [FILES]  the -m gpu suite alone (or the given test files)
#   bash tools/gpu_round.sh profile TAG       smoke(), PMC GEMM traffic, the bench line,
#                                              rocprofv3 kernel stats of the single-stream bench
#   bash tools/gpu_round.sh pmc TAG           per-phase counters of one evaluation (tools/pmc_phases.py)
#   bash tools/gpu_round.sh dist TAG          row-block tests (loopback, RCCL ranks, C4) + timings
#   bash tools/gpu_round.sh small TAG         small-n times (one-launch and general paths), the
#                                              reference's example trainings
#   bash tools/gpu_round.sh c5 TAG            the C5 posterior sweep, its rocprofv3 stats and a PMC pass
#   bash tools/gpu_round.sh ab TAG VAR "V1 V2 .." [REPS]   alternate VAR=V1, VAR=V2, ... (REPS
#                                              rounds): one evaluation's phases + a 12-step bench
#   bash tools/gpu_round.sh libab TAG LIB1 LIB2 [REPS]     the same for two library builds
set -o pipefail
cmd=$1
TAG=${2:-head}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"

suite() {   # suite LOGNAME [test files...]
  local log=$1; shift
  local what=${*:-tests}
  timeout -k 10 900 python -u -m pytest $what -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$log.log 2>&1
  local rc=$?
  tail -3 gpurun_out/$log.log
  return $rc
}
phases() { timeout -k 10 120 python3 tools/quick_time.py ${1:-16384} 10; }
bench_short() {   # one 12-step bench line, summarised
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-other-configs --steps 12 > gpurun_out/benchab_$TAG.json 2>/dev/null || return 1
  python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=r['extra']; print('bench', round(r['value'], 3), 'single', round(e['single_eval_ms'], 2), 'value', round(e['value_only_ms'], 2), 'phases', {k: round(v, 2) for k, v in e['phase_ms'].items()})" gpurun_out/benchab_$TAG.json
}
dist_times() {
  for P in 1 2; do
    timeout -k 10 240 python3 tools/dist_objective.py --loopback $P --points 16384 --dims 10 --grad --check || return 1
    timeout -k 10 240 python3 tools/dist_objective.py --loopback $P --points 16384 --dims 10 --check || return 1
  done
}

case "$cmd" in
  check)
    suite gputest_$TAG || exit 1
    for n in 16384 4096; do phases $n || exit 1; done 2>&1 | tee gpurun_out/qt_$TAG.log
    timeout -k 10 120 python3 tools/small_n_time.py 2>&1 | tee gpurun_out/small_n_$TAG.log || exit 1
    dist_times 2>&1 | tee gpurun_out/dist_$TAG.log ;;
  suite)
    shift 2
    suite gputest_$TAG "$@" || exit 1 ;;
  profile)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
    tail -2 gpurun_out/smoke_$TAG.log
    # the PMC pass first: bench.py reads profiles/pmc_gemm_<tag>.json for roofline.traffic
    timeout -k 10 600 python3 tools/pmc_gemm.py 16384 10 $TAG > gpurun_out/pmc_$TAG.log 2>&1 || exit 1
    tail -1 gpurun_out/pmc_$TAG.log
    timeout -k 10 900 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
    cat gpurun_out/bench_$TAG.json
    # single stream (--concurrent 1): every k_gemm launch has the GPU to itself, as in the
    # default bench line's profiled step, so the two per-launch means are comparable
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o bench -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --concurrent 1 --no-other-configs \
      > gpurun_out/bench_prof_$TAG.json 2>&1 || exit 1
    tail -1 gpurun_out/bench_prof_$TAG.json ;;
  pmc)
    timeout -k 10 300 python3 tools/pmc_phases.py 16384 10 > gpurun_out/pmc_phases_$TAG.json 2> gpurun_out/pmc_phases_$TAG.err || exit 1
    python3 -c "import json,sys; r=json.load(open(sys.argv[1])); [print(k, {a: round(b, 3) for a, b in v.items()}) for k, v in r['phases'].items()]" gpurun_out/pmc_phases_$TAG.json ;;
  dist)
    timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_rccl_multirank.py tests/test_gpu_fullsize.py \
      tests/test_gpu_bench_ranks.py -x -q --timeout 400 --timeout-method thread > gpurun_out/gputest_dist_$TAG.log 2>&1
    rc=$?; tail -3 gpurun_out/gputest_dist_$TAG.log; [ $rc -eq 0 ] || exit $rc
    dist_times 2>&1 | tee gpurun_out/dist_$TAG.log ;;
  small)
    timeout -k 10 200 python3 tools/small_n_time.py 2>&1 | tee gpurun_out/small_n_$TAG.log || exit 1
    GPEMU_TINY=0 timeout -k 10 200 python3 tools/small_n_time.py 2>&1 | tee gpurun_out/small_n_general_$TAG.log || exit 1
    timeout -k 10 400 python3 tools/example_train_time.py > gpurun_out/example_train_$TAG.json 2> gpurun_out/example_train_$TAG.err || exit 1
    grep "{" gpurun_out/example_train_$TAG.err ;;
  c5)
    timeout -k 10 300 python3 tools/posterior_c5.py > gpurun_out/c5_$TAG.log 2>&1 || exit 1
    tail -3 gpurun_out/c5_$TAG.log
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o c5 -- \
      python3 tools/posterior_c5.py > gpurun_out/c5_prof_$TAG.log 2>&1 || exit 1
    # counters in passes of their own (FETCH_SIZE takes 3 of the 4 TCC slots)
    timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
      -d gpurun_out/pmc_c5a_$TAG -o c5 -- python3 tools/posterior_c5.py > gpurun_out/c5_pmca_$TAG.log 2>&1 || exit 1
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
      -d gpurun_out/pmc_c5b_$TAG -o c5 -- python3 tools/posterior_c5.py > gpurun_out/c5_pmcb_$TAG.log 2>&1 || exit 1 ;;
  ab)
    VAR=$3; VALS=$4; REPS=${5:-2}
    for i in $(seq $REPS); do
      for v in $VALS; do
        echo "== $VAR=$v rep $i"
        env $VAR=$v bash -c "$(declare -f phases bench_short); TAG=$TAG; phases 16384 && bench_short" || exit 1
      done
    done 2>&1 | tee gpurun_out/ab_$TAG.log ;;
  libab)
    L1=$3; L2=$4; REPS=${5:-2}
    for i in $(seq $REPS); do
      for lib in $L1 $L2; do
        echo "== $lib rep $i"
        GPEMU_LIB=$lib bash -c "$(declare -f phases bench_short); TAG=$TAG; phases 16384 && bench_short" || exit 1
      done
    done 2>&1 | tee gpurun_out/libab_$TAG.log ;;
  *) sed -n '1,20p' "$0"; exit 2 ;;
esac
