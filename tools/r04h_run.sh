# round-4 check (dev tool): the -m gpu suite + timings of the head, the row-block
# objective's kernel breakdown at P = 1 (loopback), value-only at P = 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh r04h || exit 1
timeout -k 10 240 python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 > gpurun_out/dist_value_r04h.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dist_r04h -o dist -- python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --grad --reps 2 > gpurun_out/dist_prof_r04h.log 2>&1
