# round-5 tiny-path check (dev tool): its tests, small-n times, the example trainings.
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_api.py tests/test_gpu_edges.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_tiny_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/gputest_tiny_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/small_n_time.py 2>&1 | tee gpurun_out/small_n_$TAG.log || exit 1
timeout -k 10 400 python3 tools/example_train_time.py > gpurun_out/example_train_$TAG.json 2> gpurun_out/example_train_$TAG.err || exit 1
grep "{" gpurun_out/example_train_$TAG.err
