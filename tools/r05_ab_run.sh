# round-5 dev tool: GPU tests of the touched paths, then timings (small n, one evaluation at
# n = 16384, the row-block objective at P = 1 / 2 with both sweep schedules).
# usage: bash tools/r05_ab_run.sh TAG
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_snb.py tests/test_gpu_objective.py \
  tests/test_gpu_blocks.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/gputest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/gputest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/hip/tiny_bench_bin > gpurun_out/tiny_bench_$TAG.log 2>&1 || exit 1
timeout -k 10 60 ./tools/hip/snb_bench_bin > gpurun_out/snb_bench_$TAG.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/small_n_time.py > gpurun_out/small_n_$TAG.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/quick_time.py 16384 10 > gpurun_out/qt_$TAG.log 2>&1 || exit 1
for s in 1 0 1 0; do
  for g in "" "--grad"; do
    echo "NEXT_ON_CHAIN=$s $g"
    GPEMU_DIST_NEXT_ON_CHAIN=$s timeout -k 10 200 python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --reps 3 $g 2>&1 | tail -1 || exit 1
  done
done > gpurun_out/dist_ab_$TAG.log
GPEMU_DIST_NEXT_ON_CHAIN=1 timeout -k 10 240 python3 tools/dist_objective.py --loopback 2 --points 16384 --dims 10 --grad --check 2>&1 | tail -1 >> gpurun_out/dist_ab_$TAG.log || exit 1
cat gpurun_out/small_n_$TAG.log gpurun_out/qt_$TAG.log gpurun_out/dist_ab_$TAG.log
