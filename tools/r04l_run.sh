# round-4 A/B (dev tool): the dev head (noinline diagonal factor, first-panel hand-off,
# column-split K-build / contraction at small n) -- its objective tests first -- against the
# head and the noinline-only build: phases, two-try bench (alternating, twice), chain traces,
# small n
mkdir -p gpurun_out
GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_pf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_objective.py tests/test_gpu_concurrent.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pf_tests_r04l.log 2>&1
rc=$?; tail -2 gpurun_out/pf_tests_r04l.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for L in libgpemu.so libgpemu_ni.so libgpemu_pf.so; do
    echo "== $L rep $rep"
    for n in 16384 4096; do GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1; done
    GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline \
      --no-other-configs --no-profile 2>/dev/null | tail -1 | cut -c1-200 || exit 1
  done
done > gpurun_out/ab_r04l.log 2>&1
for L in libgpemu_trace.so libgpemu_ni_trace.so libgpemu_pf_trace.so; do
  echo "== $L"; GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 120 python3 tools/chol_trace.py 16384 || exit 1
done > gpurun_out/chol_ab_r04l.log 2>&1
GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_pf.so timeout -k 10 120 python3 tools/small_n_time.py > gpurun_out/small_n_r04l_pf.log 2>&1
