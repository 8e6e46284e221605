# round-5 counters (dev tool): per-phase PMC of one evaluation (lone: group launches; and
# per-step launches) and the cold / hot GEMM clock experiment.  usage: bash tools/r05_pmc.sh TAG
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/pmc_phases.py 16384 10 > gpurun_out/pmc_phases_group_$TAG.json 2> gpurun_out/pmc_phases_$TAG.err || exit 1
GPEMU_POTRF=fused timeout -k 10 300 python3 tools/pmc_phases.py 16384 10 > gpurun_out/pmc_phases_fused_$TAG.json 2>> gpurun_out/pmc_phases_$TAG.err || exit 1
timeout -k 10 600 python3 tools/clock_traffic.py 96 512 4096 > gpurun_out/clock_traffic_$TAG.log 2>&1 || exit 1
cat gpurun_out/clock_traffic_$TAG.log
