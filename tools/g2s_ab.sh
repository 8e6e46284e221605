# Two-stream group schedule A/B (dev tool): GPEMU_POTRF=g2s vs the fused default, one
# evaluation's phases and the two-try bench, interleaved.
set -e
for rep in 1 2; do
  for M in g2s fused; do
    E=""; [ "$M" = g2s ] && E="GPEMU_POTRF=g2s"
    env $E timeout -k 10 120 python3 tools/quick_time.py 16384 10 | grep -E "eval s|phases|value-only" | tr '\n' ' ' | sed "s/^/$M: /"; echo
    env $E timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 15 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['extra']; print('$M', 'bench', round(d['value'], 3), 'single', round(e['single_eval_ms'], 2), 'value_only', round(e['value_only_ms'], 2), flush=True)"
  done
done
