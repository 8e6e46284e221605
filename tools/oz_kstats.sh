# int8 helper kernels' per-launch times (dev tool): GPU tests of the int8 paths, then the
# kernel stats of a short single-stream bench.  usage: bash tools/oz_kstats.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_posterior.py tests/test_gpu_dist.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gputest_oz_$tag.log 2>&1; rc=$?; tail -2 gpurun_out/gputest_oz_$tag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ozk_$tag -o b -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --concurrent 1 --no-other-configs > gpurun_out/ozk_$tag.json 2>&1 || exit 1
f=$(find gpurun_out/ozk_$tag -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/ozk_stats_$tag.csv; rm -rf gpurun_out/ozk_$tag
python3 - gpurun_out/ozk_stats_$tag.csv <<'PY'
import csv, sys
for r in list(csv.reader(open(sys.argv[1])))[1:]:
    if 'oz' in r[0] or 'k_gemm' in r[0]:
        print(r[0][:60].ljust(60), r[1].rjust(5), '%9.1f us' % (float(r[3]) / 1e3))
PY
tail -1 gpurun_out/ozk_$tag.json | cut -c1-200
