# round-4 check (dev tool): block-layout micro-check, the -m gpu suite + timings of the
# head, then A/B builds (XOR-swizzled / padded diagonal-block layout, no split K)
mkdir -p gpurun_out
bash tools/gpu_micro.sh > gpurun_out/micro_r04f.log 2>&1 || exit 1
bash tools/gpu_check.sh r04f || exit 1
for L in xor pad nosk; do
  for n in 16384 4096; do
    echo "== $L n=$n"; GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_$L.so timeout -k 10 120 python3 tools/quick_time.py $n 10 || exit 1
  done
  echo "== $L small n"; GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_$L.so timeout -k 10 120 python3 tools/small_n_time.py || exit 1
done > gpurun_out/ab_r04f.log 2>&1
for L in pad xor; do
  GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_objective.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${L}_tests_r04f.log 2>&1 || exit 1
done
