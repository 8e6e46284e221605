# Build the per-tile-trace library (-DGEMM_TTRACE) in-tree (dev tool; run here, on the CPU).
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Wno-unused-result -Wno-unused-value \
  -DGEMM_TTRACE -DGPE_SOURCE_HASH='"ttrace"' -o gp_emu_uqsa_amd/libgpemu_ttrace.so \
  gp_emu_uqsa_amd/csrc/gpemu.hip gp_emu_uqsa_amd/csrc/gpemu_dist.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
