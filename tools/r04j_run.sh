# round-4 check (dev tool): split-K reduction fix -- GPU tests touching the split launches,
# small-n times, the n = 1024 timeline
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_objective.py tests/test_gpu_blocks.py tests/test_gpu_posterior.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r04j.log 2>&1
rc=$?; tail -2 gpurun_out/gputest_r04j.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/small_n_time.py > gpurun_out/small_n_r04j.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_n1024_r04j -o ev -- python3 tools/eval_timeline.py run 1024 5 > gpurun_out/ev1024_r04j.log 2>&1 || exit 1
for n in 16384 4096; do timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1; done > gpurun_out/qt_r04j.log 2>&1
