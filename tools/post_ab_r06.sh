# posterior tests, then C5 (1e6 points) with V on the int8 cores / fp32 / fp64 (round 6)
set -o pipefail
mkdir -p gpurun_out
tag=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_posterior.py tests/test_gpu_headline.py tests/test_gpu_noise_fit.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_post_$tag.log 2>&1; rc=$?; tail -3 gpurun_out/gputest_post_$tag.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1 32" "0 32" "1 64" "0 64"; do
  set -- $cfg
  GPEMU_OZAKI=$1 timeout -k 10 300 python3 tools/posterior_c5.py --precision $2 | sed "s/^/oz=$1 /" || exit 1
done 2>&1 | tee gpurun_out/c5_ab_$tag.log
