# GPU check of the current head (dev tool): the -m gpu suite, then one evaluation's
# phases at n = 16384 and 4096 and the small-n times.  usage: bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-head}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gputest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/gputest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for n in 16384 4096; do timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1; done 2>&1 | tee gpurun_out/qt_$TAG.log
timeout -k 10 120 python3 tools/small_n_time.py 2>&1 | tee gpurun_out/small_n_$TAG.log
if [ -f gp_emu_uqsa_amd/libgpemu_trace.so ]; then
  for n in 16384 4096; do
    GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_trace.so timeout -k 10 120 python3 tools/chol_trace.py $n || exit 1
  done 2>&1 | tee gpurun_out/chol_trace_$TAG.log
fi
for P in 1 2; do
  timeout -k 10 240 python3 tools/dist_objective.py --loopback $P --points 16384 --dims 10 --grad --check || exit 1
done 2>&1 | tee gpurun_out/dist_$TAG.log
