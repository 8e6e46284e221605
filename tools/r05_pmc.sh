# round-5 counters (dev tool): per-phase PMC of one evaluation (lone evaluation: group
# launches; with and without super-blocks; and per-step launches) and the cold / hot GEMM
# clock experiment.  usage: bash tools/r05_pmc.sh TAG
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "sb2" "sb1" "fused"; do
  case $v in
    sb2) E="GPEMU_POTRF_SB=2" ;;
    sb1) E="GPEMU_POTRF_SB=1" ;;
    fused) E="GPEMU_POTRF=fused" ;;
  esac
  env $E timeout -k 10 300 python3 tools/pmc_phases.py 16384 10 > gpurun_out/pmc_phases_${v}_$TAG.json 2>> gpurun_out/pmc_phases_$TAG.err || exit 1
  echo "== $v"; python3 -c "import json,sys; r=json.load(open(sys.argv[1])); [print(k, {a: round(b, 3) for a, b in v.items()}) for k, v in r['phases'].items()]" gpurun_out/pmc_phases_${v}_$TAG.json
done
timeout -k 10 600 python3 tools/clock_traffic.py 96 512 4096 > gpurun_out/clock_traffic_$TAG.log 2>&1 || exit 1
cat gpurun_out/clock_traffic_$TAG.log
