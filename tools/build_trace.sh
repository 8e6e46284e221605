# Dev build of libgpemu with the fused-Cholesky chain timeline (-DGEMM_TRACE) for
# tools/chol_trace.py (GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_trace.so).  CPU-side: run here,
# the .so travels to the GPU box with the tree.
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -w -DGEMM_TRACE \
  -o gp_emu_uqsa_amd/libgpemu_trace.so gp_emu_uqsa_amd/csrc/gpemu.hip gp_emu_uqsa_amd/csrc/gpemu_dist.hip \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
