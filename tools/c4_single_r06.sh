set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 600 --timeout-method thread > gpurun_out/gputest_full_c4a.log 2>&1; rc=$?; tail -2 gpurun_out/gputest_full_c4a.log; [ $rc -eq 0 ] || exit $rc
for oz in 1 0; do echo "GPEMU_OZAKI=$oz"; GPEMU_OZAKI=$oz timeout -k 10 300 python3 tools/quick_time.py 65536 20 || exit 1; done 2>&1 | tee gpurun_out/c4_single_oz.log
