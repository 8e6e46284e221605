# round-5 distributed check (dev tool): the row-block tests (loopback, RCCL multi-rank, C4,
# bench ranks) and the loopback timings at n = 16384.  usage: bash tools/r05_dist.sh TAG
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_rccl_multirank.py tests/test_gpu_fullsize.py \
  tests/test_gpu_bench_ranks.py tests/test_gpu_limits.py -x -q --timeout 400 --timeout-method thread \
  > gpurun_out/gputest_dist_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/gputest_dist_$TAG.log
[ $rc -eq 0 ] || exit $rc
for P in 1 2; do
  timeout -k 10 240 python3 tools/dist_objective.py --loopback $P --points 16384 --dims 10 --grad --check || exit 1
done 2>&1 | tee gpurun_out/dist_$TAG.log
