set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_c5_r06k -o c5 -- \
  python3 tools/posterior_c5.py > gpurun_out/c5_prof_r06k.log 2>&1 || exit 1
f=$(find gpurun_out/prof_c5_r06k -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/c5_kstats_r06k.csv
t=$(find gpurun_out/prof_c5_r06k -name '*kernel_trace.csv' | head -1); python3 tools/trace_timeline.py "$t" 0 > gpurun_out/c5_tl_r06k.log 2>&1 || true
rm -rf gpurun_out/prof_c5_r06k
