# Cholesky column-group widths x tries in flight against the two-try bench (dev tool,
# round 3).  usage: bash tools/potrf_w_conc_sweep.sh
set -e
mkdir -p gpurun_out
for W in "4:80,2:40" "8:96,4:48,2:24" "8:64,4:32" "16:96,8:48,4:24"; do
  for K in 2 3; do
    GPEMU_POTRF_W="$W" timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 15 --warmup 3 --concurrent $K 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('W', '$W', 'tries', $K, 'bench', round(d['value'], 3), 'single', round(d['extra']['single_eval_ms'], 2), 'chol', round(d['extra']['phase_ms']['cholesky'], 2), flush=True)"
  done
done
