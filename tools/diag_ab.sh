# A/B of the diagonal-block factorisation and the panel tiles (dev tool): stand-alone
# 128x128 factor, then one evaluation's phases at n = 16384 and 4096 per variant,
# alternating.  usage: bash tools/diag_ab.sh lib[:ENV=VAL] ...   (libs under gp_emu_uqsa_amd/)
set -e
mkdir -p gpurun_out
for b in tools/hip/db_bench_*; do
  [ -x "$b" ] || continue
  echo "== $b"; timeout -k 5 30 "$b"
done
for rep in 1 2; do
  for V in "$@"; do
    L=${V%%:*}; E=""; [ "$V" != "$L" ] && E=${V#*:}
    for n in 16384 4096; do
      echo "== $V n=$n rep $rep"
      env GPEMU_LIB=gp_emu_uqsa_amd/$L $E timeout -k 10 120 python3 tools/quick_time.py $n 10
    done
  done
done
