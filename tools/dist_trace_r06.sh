# kernel traces of the P = 1 row-block objective -> timeline summaries (dev tool)
# usage: bash tools/dist_trace_r06.sh TAG [extra dist_objective.py args]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dtr_$tag -o tr -- \
  python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --reps 3 "$@" > gpurun_out/dtr_$tag.log 2>&1 || exit 1
f=$(find gpurun_out/dtr_$tag -name '*kernel_trace.csv' | head -1)
python3 tools/trace_timeline.py "$f" -2 2>&1 | tee gpurun_out/dist_trace_$tag.log
s=$(find gpurun_out/dtr_$tag -name '*kernel_stats.csv' | head -1)
cp "$s" gpurun_out/dist_stats_$tag.csv
