# A/B of the GEMM staging: default build (global_load_lds) vs -DGEMM_REGSTAGE (dev tool).
# Build the second library on the CPU host first:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DGEMM_REGSTAGE \
#     -o gp_emu_uqsa_amd/libgpemu_probe_REG.so gp_emu_uqsa_amd/csrc/gpemu.hip \
#     gp_emu_uqsa_amd/csrc/gpemu_dist.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_blocks.py tests/test_gpu_objective.py tests/test_gpu_midsize.py tests/test_gpu_posterior.py
for L in libgpemu.so libgpemu_probe_REG.so; do
  echo "== $L"
  for cfg in "64 64 4096 0 0" "64 64 4096 1 1" "64 64 4096 1 0" "64 64 4096 0 1" "64 64 512 0 0"; do
    GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 60 python tools/gemm_one.py $cfg 10
  done
  GPEMU_LIB=gp_emu_uqsa_amd/$L timeout -k 10 120 python tools/quick_time.py 16384 10
done
