# round-5 dev tool: the row-block objective at P = 1 (loopback, n = 16384, d = 10) under
# several column-group schedules (GPEMU_DIST_W), value only and with the gradient, and a
# kernel trace of the value for tools/trace_timeline.py.  usage: bash tools/r05_dist_ab.sh TAG
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$NOTRACE" ] || timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dist1_$TAG -o k -- \
  python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --reps 3 > /dev/null 2>&1 || exit 1
for w in ${WLIST:-"8:160,4:80,2:40" "8:160,4:80,2:0" "8:160,4:40,2:0" "8:160,4:0" "8:160,4:80,2:40"}; do
  for g in "" "--grad"; do
    echo "W=$w $g"
    GPEMU_DIST_W=$w timeout -k 10 200 python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --reps 3 $g 2>&1 | tail -1 || exit 1
  done
done > gpurun_out/dist_w_$TAG.log
cat gpurun_out/dist_w_$TAG.log
