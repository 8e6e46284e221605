# round-5 dev tool: kernel statistics of the row-block objective at P = 1 (loopback) against
# the single-GPU objective, value only and with the gradient, n = 16384, d = 10; and the
# example trainings with the one-launch n <= 128 path.  usage: bash tools/r05_dist_prof.sh TAG
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in "" "--grad"; do
  name=dist1${g:+_grad}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${name}_$TAG -o k -- \
    python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --reps 3 $g > gpurun_out/${name}_$TAG.log 2>&1 || exit 1
  tail -1 gpurun_out/${name}_$TAG.log
done
timeout -k 10 400 python3 tools/example_train_time.py > gpurun_out/example_train_$TAG.json 2> gpurun_out/example_train_$TAG.err || exit 1
grep "{" gpurun_out/example_train_$TAG.err
