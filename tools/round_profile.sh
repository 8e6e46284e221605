# PMC traffic, bench line and rocprofv3 kernel stats for the round (run on the GPU box).
# usage: bash tools/round_profile.sh r01
# The PMC pass runs first: bench.py reads profiles/pmc_gemm_<tag>.json for roofline.traffic.
set -e
tag=${1:-r01}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 tools/pmc_gemm.py 16384 10 ${tag} > gpurun_out/pmc_${tag}.log 2>&1
tail -1 gpurun_out/pmc_${tag}.log
timeout -k 10 900 python3 bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err
cat gpurun_out/bench_${tag}.json
# single stream (--concurrent 1): every k_gemm launch has the GPU to itself, as in the
# default bench line's profiled step, so the two per-launch means are comparable
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag} -o bench -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --concurrent 1 --no-other-configs > gpurun_out/bench_prof_${tag}.json 2>&1
cat gpurun_out/bench_prof_${tag}.json | tail -1
