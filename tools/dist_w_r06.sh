# Row-block P = 1 column-group widths (GPEMU_DIST_W) at n = 16384: value and gradient times,
# alternating the settings twice.  Output: gpurun_out/dist_w_r06${WTAG:-}.log
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
mkdir -p gpurun_out
for rep in 1 2; do
  for W in ${WLIST:-"8:160,4:0" "8:64,4:0" "8:96,4:0" "8:0" "6:0"}; do
    for g in ${WG:-"" "--grad"}; do
      echo "== W=$W $g rep $rep"
      GPEMU_DIST_W=$W timeout -k 10 120 python3 tools/dist_objective.py --loopback ${WP:-1} --points ${WN:-16384} --dims ${WD:-10} $g \
        | python3 -c "import json,sys; r=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(r['ms_per_eval'], 2), r['llh'])" || exit 1
    done
  done
done 2>&1 | tee gpurun_out/dist_w_r06${WTAG:-}.log
