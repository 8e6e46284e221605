# round-4 check (dev tool): the row-block objective's tests, timings and kernel breakdown;
# the kernel timeline of one evaluation at n = 1024
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_edges.py tests/test_gpu_rccl_multirank.py tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread > gpurun_out/gputest_dist_r04i.log 2>&1
rc=$?; tail -2 gpurun_out/gputest_dist_r04i.log; [ $rc -eq 0 ] || exit $rc
for P in 1 2; do timeout -k 10 240 python3 tools/dist_objective.py --loopback $P --points 16384 --dims 10 --grad --check || exit 1; done > gpurun_out/dist_r04i.log 2>&1
timeout -k 10 240 python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 >> gpurun_out/dist_r04i.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dist_r04i -o dist -- python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --grad --reps 2 > gpurun_out/dist_prof_r04i.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_n1024_r04i -o ev -- python3 tools/eval_timeline.py run 1024 5 > gpurun_out/ev1024_r04i.log 2>&1
