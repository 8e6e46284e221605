# round-5 dev tool: same-box A/B of the session-start library (tools/ab/libgpemu_r05start.so,
# built from d166a9c) against the head: one evaluation's phases at n = 16384 and a short bench
# line each, alternating twice.  usage: bash tools/r05_lib_ab.sh TAG
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
for i in 1 2; do
  for lib in tools/ab/libgpemu_r05start.so gp_emu_uqsa_amd/libgpemu.so; do
    echo "== $lib"
    GPEMU_LIB=$lib timeout -k 10 120 python3 tools/quick_time.py 16384 10 2>&1 | grep -v "^n " || exit 1
    GPEMU_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-other-configs 2>/dev/null | tail -1 | cut -c1-120 || exit 1
  done
done > gpurun_out/lib_ab_$TAG.log
cat gpurun_out/lib_ab_$TAG.log
