# Leading-block inverse beside the middle of the sweep (GPEMU_TAIL_OVERLAP=2, plain second
# stream) at several split steps vs the default (dev tool): one evaluation's phases and
# the two-try bench.
set -e
for cfg in "0 64" "2 48" "2 64" "2 80" "0 64"; do
  set -- $cfg
  GPEMU_TAIL_OVERLAP=$1 GPEMU_TAIL_SPLIT=$2 timeout -k 10 120 python3 tools/quick_time.py 16384 10 | grep -E "eval s|phases" | tr '\n' ' ' | sed "s/^/mode $1 split $2: /"; echo
  GPEMU_TAIL_OVERLAP=$1 GPEMU_TAIL_SPLIT=$2 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 15 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['extra']; print('mode', '$1', 'split', '$2', 'bench', round(d['value'], 3), 'single', round(e['single_eval_ms'], 2), flush=True)"
done
