# round-5 super-block A/B (dev tool): the lone evaluation's phases (quick_time) and the
# two-try bench for GPEMU_POTRF_SB settings.  usage: bash tools/r05_sb_ab.sh TAG "1 2:80 ..."
set -o pipefail
TAG=${1:-r05}
SETS=${2:-"1 2:80 2:64 3:80 4:80"}
mkdir -p gpurun_out
for sb in $SETS; do
  echo "== SB=$sb"
  GPEMU_POTRF_SB=$sb timeout -k 10 120 python3 tools/quick_time.py 16384 10 2>&1 | grep -E "eval s|phases|value-only" || exit 1
  GPEMU_POTRF_SB=$sb timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 12 > gpurun_out/sbab_${TAG}_$sb.json 2>&1 || exit 1
  python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', round(r['value'], 3), 'single', round(r['extra']['single_eval_ms'], 2), 'value', round(r['extra']['value_only_ms'], 2))" gpurun_out/sbab_${TAG}_$sb.json
done 2>&1 | tee gpurun_out/sb_ab_$TAG.log
