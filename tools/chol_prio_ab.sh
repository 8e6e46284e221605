# Fused Cholesky (GPEMU_CHOL_PRIO=1, default) and also the TRTRI levels (=2) on the
# context's high-priority stream against everything on the context stream (=0) (dev
# tool): the two-try bench, alternating.
set -e
run() {
  env $2 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 40 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['extra']; print('$1', 'bench', round(d['value'], 3), 'single', round(e['single_eval_ms'], 2), 'chol', round(e['phase_ms']['cholesky'], 2), 'trtri', round(e['phase_ms']['trtri'], 2), 'vo', round(e['value_only_ms'], 2), flush=True)"
}
for rep in 1 2 3; do
  run prio0 "GPEMU_CHOL_PRIO=0"
  run prio1 "GPEMU_CHOL_PRIO=1"
  run prio2 "GPEMU_CHOL_PRIO=2"
done
