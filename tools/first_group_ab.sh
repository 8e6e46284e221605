# Width of the Cholesky's first column group (GPEMU_POTRF_FIRST) vs the default 4 (dev
# tool): one evaluation's phases, value only, and the two-try bench.
set -e
for F in 0 1 2 0 1 2; do
  GPEMU_POTRF_FIRST=$F timeout -k 10 120 python3 tools/quick_time.py 16384 10 | grep -E "phases|value-only" | sed -e "s/.*'cholesky': \([0-9.]*\).*/chol \1/" -e "s/value-only s \[\([0-9.]*\), \([0-9.]*\).*/vo \2/" | tr '\n' ' ' | sed "s/^/first $F: /"; echo
done
for F in 0 1; do
  GPEMU_POTRF_FIRST=$F timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 15 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['extra']; print('first', '$F', 'bench', round(d['value'], 3), 'single', round(e['single_eval_ms'], 2), 'value_only', round(e['value_only_ms'], 2), flush=True)"
done
