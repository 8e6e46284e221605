# row-block GPU tests, then P = 1 timings at n = 16384 with the int8 products on / off
# usage: bash tools/dist_ab_r06.sh TAG
set -o pipefail
mkdir -p gpurun_out
tag=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_dist_$tag.log 2>&1; rc=$?; tail -3 gpurun_out/gputest_dist_$tag.log; [ $rc -eq 0 ] || exit $rc
for oz in 1 0; do
  for g in --grad ""; do
    GPEMU_OZAKI=$oz timeout -k 10 240 python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --reps 4 --check $g | sed "s/^/oz=$oz /" || exit 1
  done
done 2>&1 | tee gpurun_out/dist_ab_$tag.log
