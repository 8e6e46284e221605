# Two-try bench: the auto Cholesky schedule (default: group launches for a lone
# evaluation, one launch per step beside others) against always-group and always-per-step
# (dev tool), alternating; then the schedule and concurrency tests.
set -e
run() {
  env $2 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 40 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['extra']; print('$1', 'bench', round(d['value'], 3), 'single', round(e['single_eval_ms'], 2), 'chol', round(e['phase_ms']['cholesky'], 2), 'vo', round(e['value_only_ms'], 2), flush=True)"
}
for rep in 1 2 3; do
  run auto "GPEMU_POTRF=auto"
  run group "GPEMU_POTRF=group"
  run fused "GPEMU_POTRF=fused"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_objective.py tests/test_gpu_concurrent.py -k "schedule or concurrent" 2>&1 | tail -2
