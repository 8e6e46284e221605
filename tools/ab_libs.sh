# A/B of library builds on one box (dev tool): one evaluation's phases at n = 16384 and
# 4096 per library / environment, alternating, twice.
# usage: bash tools/ab_libs.sh lib[:ENV=VAL[,ENV=VAL]] ...   (libs under gp_emu_uqsa_amd/)
mkdir -p gpurun_out
for rep in 1 2; do
  for V in "$@"; do
    L=${V%%:*}; E=""; [ "$V" != "$L" ] && E=$(echo "${V#*:}" | tr ',' ' ')
    for n in 16384 4096; do
      echo "== $V n=$n rep $rep"
      env GPEMU_LIB=gp_emu_uqsa_amd/$L $E timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1
    done
  done
done
