# round-5 GPU check (dev tool): the -m gpu suite, phase timings at n = 16384 / 4096 with the
# super-block schedule (default) and without (GPEMU_POTRF_SB=1), then the bench line with its
# CPU baseline and an A/B bench without super-blocks.  usage: bash tools/r05_check.sh TAG
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gputest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/gputest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for sb in 2 1; do for n in 16384 4096; do echo "SB=$sb"; GPEMU_POTRF_SB=$sb timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1; done; done 2>&1 | tee gpurun_out/qt_$TAG.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cut -c1-400 gpurun_out/bench_$TAG.json
for sb in 1 2; do GPEMU_POTRF_SB=$sb timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-other-configs > gpurun_out/bench_${TAG}_sb$sb.json 2>&1 || exit 1; echo "SB=$sb $(cut -c1-200 gpurun_out/bench_${TAG}_sb$sb.json)"; done
