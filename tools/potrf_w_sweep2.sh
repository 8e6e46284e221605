# Cholesky column-group widths (GPEMU_POTRF_W) against phase times and the bench, second
# sweep after the K-loop work (dev tool).  usage: bash tools/potrf_w_sweep2.sh [widths ...]
set -e
mkdir -p gpurun_out
ws=("$@")
[ ${#ws[@]} -eq 0 ] && ws=("4:80,2:40" "8:96,4:48,2:24" "6:96,4:60,2:30" "8:80,4:40,2:20" "4:80,2:40")
for W in "${ws[@]}"; do
  echo "== W=$W"
  GPEMU_POTRF_W="$W" timeout -k 10 120 python3 tools/quick_time.py 16384 10 | grep phases
  GPEMU_POTRF_W="$W" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('bench', round(d['value'], 3), 'single', round(d['extra']['single_eval_ms'], 2))"
done
