# round-5 XCD tile-block A/B (dev tool): GPEMU_XCD_BLOCK = 0 (rows per XCD, default) / b (b x b
# blocks per XCD): lone-evaluation phases, the two-try bench, and the per-phase PMC (traffic,
# clock, MFMA busy).  usage: bash tools/r05_xcd_ab.sh TAG "0 8 4 0"
set -o pipefail
TAG=${1:-r05}
SETS=${2:-"0 8 4 0"}
mkdir -p gpurun_out
for xb in $SETS; do
  echo "== XCD_BLOCK=$xb"
  GPEMU_XCD_BLOCK=$xb timeout -k 10 120 python3 tools/quick_time.py 16384 10 2>&1 | grep -E "eval s|phases|value-only" || exit 1
  GPEMU_XCD_BLOCK=$xb timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs --steps 12 > gpurun_out/xcdab_${TAG}_$xb.json 2>&1 || exit 1
  python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', round(r['value'], 3), 'single', round(r['extra']['single_eval_ms'], 2), 'value', round(r['extra']['value_only_ms'], 2))" gpurun_out/xcdab_${TAG}_$xb.json
done 2>&1 | tee gpurun_out/xcd_ab_$TAG.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for xb in 0 8; do
  GPEMU_XCD_BLOCK=$xb timeout -k 10 300 python3 tools/pmc_phases.py 16384 10 > gpurun_out/pmc_phases_xcd${xb}_$TAG.json 2>> gpurun_out/pmc_phases_xcd_$TAG.err || exit 1
done
for xb in 0 8; do echo "== pmc XCD_BLOCK=$xb"; python3 -c "
import json,sys; t=open(sys.argv[1]).read(); r=json.loads(t[t.index('{'):])
for k,v in r['phases'].items(): print('%-12s'%k, ' '.join('%s=%.3f'%(a,b) for a,b in v.items()))" gpurun_out/pmc_phases_xcd${xb}_$TAG.json; done
