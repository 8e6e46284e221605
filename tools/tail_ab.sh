# Overlapped Cholesky tail A/B (dev tool): GPEMU_TAIL_OVERLAP=1 vs 0 (default), single
# evaluation phases and the two-try bench, two interleaved pairs.
set -e
for rep in 1 2; do
  for O in 1 0; do
    GPEMU_TAIL_OVERLAP=$O timeout -k 10 120 python3 tools/quick_time.py 16384 10 | grep -E "eval s|phases" | tr '\n' ' ' | sed "s/^/overlap $O: /"; echo
    GPEMU_TAIL_OVERLAP=$O timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 15 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['extra']; print('overlap', '$O', 'bench', round(d['value'], 3), 'single', round(e['single_eval_ms'], 2), flush=True)"
  done
done
