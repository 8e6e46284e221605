# One launch per column group (GPEMU_POTRF=group), with and without the pinned diagonal
# tiles (GPEMU_GROUP_PIN=1), widths, against the per-step fused schedule (dev tool):
# schedule parity tests, the Cholesky phase and value-only times.
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_objective.py -k "schedule" 2>&1 | tail -4
run() { env $1 timeout -k 10 120 python3 tools/quick_time.py 16384 10 | grep -E "phases|value-only" | sed -e "s/.*'cholesky': \([0-9.]*\).*/chol \1/" -e "s/value-only s \[\([0-9.]*\), \([0-9.]*\).*/vo \2/" | tr '\n' ' ' | sed "s/^/$1: /"; echo; }
run "GPEMU_POTRF=fused"
for W in 4:80,2:40 6:96,4:64,3:48,2:32 8:96,4:48,2:24 8:64,4:32,2:16 4:80,3:56,2:32; do
  run "GPEMU_POTRF=group GPEMU_GROUP_P0=512 GPEMU_GROUP_STRIDE=896 GPEMU_POTRF_W=$W"
  run "GPEMU_POTRF=group GPEMU_GROUP_P0=512 GPEMU_GROUP_STRIDE=896 GPEMU_GROUP_PIN=1 GPEMU_POTRF_W=$W"
done
run "GPEMU_POTRF=group GPEMU_GROUP_P0=512 GPEMU_GROUP_STRIDE=640 GPEMU_GROUP_PIN=1 GPEMU_POTRF_W=6:96,4:64,3:48,2:32"
run "GPEMU_POTRF=fused"
