// Which workgroup indices share a CU with workgroup 0? (dev probe)
// 2048 workgroups of 256 threads with 76,864 B of dynamic LDS (two per CU, as k_gemm's
// launches); each spins ~`spin` cycles and records XCC_ID / HW_ID and a start time.
// hipcc --offload-arch=gfx950 -O3 tools/hip/placement_probe.hip -o tools/hip/placement_probe_bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(unsigned* out, unsigned long long* t, int spin) {
  extern __shared__ double lds[];
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);      // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);    // HW_REG_XCC_ID
  const unsigned long long t0 = wall_clock64();
  long long c0 = clock64();
  lds[threadIdx.x] = 1.0;
  while (clock64() - c0 < spin) {}
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc & 0xf;
    t[blockIdx.x] = t0;
  }
}

int main() {
  const int nwg = 2048;
  unsigned* d; unsigned long long* dt;
  (void)hipMalloc(&d, 2 * nwg * 4); (void)hipMalloc(&dt, nwg * 8);
  (void)hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 76864);
  std::vector<unsigned> h(2 * nwg);
  std::vector<unsigned long long> ht(nwg);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), 76864, 0, d, dt, 200000);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ht.data(), dt, ht.size() * 8, hipMemcpyDeviceToHost);
    auto key = [&](int i) { unsigned hw = h[2 * i]; return (h[2 * i + 1] << 16) | (((hw >> 13) & 3) << 12) | (((hw >> 12) & 1) << 8) | ((hw >> 8) & 0xf); };
    const unsigned k0 = key(0);
    printf("rep %d: wg0 = xcc %u se %u sh %u cu %u; co-located with wg0:", rep, k0 >> 16, (k0 >> 12) & 3, (k0 >> 8) & 1, k0 & 0xf);
    int cnt = 0;
    for (int i = 1; i < nwg; ++i)
      if (key(i) == k0) { if (cnt < 12) printf(" %d(+%.1fus)", i, (ht[i] - ht[0]) * 0.01); ++cnt; }
    printf("  [%d total]\n", cnt);
    // how many of wg 256..511 share a CU with wg (i - 256)?
    int same = 0;
    for (int i = 256; i < 512; ++i) same += key(i) == key(i - 256);
    printf("   wg i and i-256 on the same CU for %d of 256 (i in 256..511)\n", same);
  }
  return 0;
}
