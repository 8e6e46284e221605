# Round-4 A/B on one box (dev tool): leaf / factor probes, then per library build one
# evaluation's phases (n = 16384, 4096) and the two-try bench, alternating, twice.
mkdir -p gpurun_out
bash tools/gpu_micro.sh > gpurun_out/micro_$1.log 2>&1 || exit 1
shift
[ -f gp_emu_uqsa_amd/libgpemu_vF.so ] && set -- "$@" libgpemu_vF.so
for rep in 1 2; do
  for L in "$@"; do
    for n in 16384 4096; do
      echo "== $L n=$n rep $rep"
      GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1
    done
    echo "== bench $L rep $rep"
    GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline \
      --no-other-configs --no-profile 2>/dev/null | tail -1 | cut -c1-330 || exit 1
  done
done
