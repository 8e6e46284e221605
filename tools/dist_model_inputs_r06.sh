# P = 1 row-block timings that feed tools/dist_model.py (round 6): the P > 1 arithmetic is the
# int8 A^-1 partial with the fp64 TRTRI (GPEMU_OZAKI_TRI_MIN above every level)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dist_model_inputs_r06.log
: > $out
run() { echo "$1" | tee -a $out; shift; timeout -k 10 300 "$@" 2>&1 | tee -a $out || exit 1; }
run "n=16384 grad, int8 partial, fp64 TRTRI" env GPEMU_OZAKI_TRI_MIN=1000000000 python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --reps 4 --grad
run "n=16384 grad, default" python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --reps 4 --grad
run "n=16384 value" python3 tools/dist_objective.py --loopback 1 --points 16384 --dims 10 --reps 4
run "C4 P=1 grad, int8 partial (cap raised), fp64 TRTRI" env GPEMU_DIST_OZAKI_MB=100000 GPEMU_OZAKI_TRI_MIN=1000000000 python3 tools/dist_objective.py --loopback 1 --points 65536 --dims 20 --reps 1 --grad
run "C4 P=1 value" python3 tools/dist_objective.py --loopback 1 --points 65536 --dims 20 --reps 1
