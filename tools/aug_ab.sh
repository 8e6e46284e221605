# Augmented-row A/B on one box (dev tool): GPEMU_AUG=0 (forward substitution) vs default,
# two interleaved pairs of the two-try bench.  usage: bash tools/aug_ab.sh
set -e
for rep in 1 2; do
  for A in 1 0; do
    GPEMU_AUG=$A timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 15 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['extra']; print('aug', '$A', 'bench', round(d['value'], 3), 'single', round(e['single_eval_ms'], 2), 'value_only', round(e['value_only_ms'], 2), 'chol', round(e['phase_ms']['cholesky'], 2), 'trtri', round(e['phase_ms']['trtri'], 2), 'inv', round(e['phase_ms']['inverse'], 2), flush=True)"
  done
done
