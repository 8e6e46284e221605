# round-5 small-n check (dev tool): the -m gpu suite (the tiny path runs under every test of
# n <= 128, the reference's example replays included), small-n times, the example trainings.
# usage: bash tools/r05_small.sh TAG
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gputest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/gputest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/small_n_time.py 2>&1 | tee gpurun_out/small_n_$TAG.log || exit 1
GPEMU_TINY=0 timeout -k 10 200 python3 tools/small_n_time.py 2>&1 | tee gpurun_out/small_n_general_$TAG.log || exit 1
timeout -k 10 400 python3 tools/example_train_time.py > gpurun_out/example_train_$TAG.json 2> gpurun_out/example_train_$TAG.err || exit 1
cat gpurun_out/example_train_$TAG.err | grep "{"
for P in 1 2; do
  timeout -k 10 240 python3 tools/dist_objective.py --loopback $P --points 16384 --dims 10 --grad --check || exit 1
  timeout -k 10 240 python3 tools/dist_objective.py --loopback $P --points 16384 --dims 10 --check || exit 1
done 2>&1 | tee gpurun_out/dist_$TAG.log
