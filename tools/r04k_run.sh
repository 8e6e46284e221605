# round-4 check (dev tool): the -m gpu suite + timings of the head; n = 1024 timeline
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh r04k || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_n1024_r04k -o ev -- python3 tools/eval_timeline.py run 1024 5 > gpurun_out/ev1024_r04k.log 2>&1
