// Which CUs does a stream's CU mask select on gfx950? (dev probe)
// Each workgroup records XCC_ID and HW_ID (SE / CU fields); the host prints, per mask,
// the set of (xcc, se, cu) the workgroups ran on.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void probe(unsigned* out, int spin) {
  unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);      // HW_REG_HW_ID
  unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);    // HW_REG_XCC_ID
  long long t0 = clock64();
  while (clock64() - t0 < spin) {}
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("CUs %d\n", p.multiProcessorCount);
  const int nwg = 8192;
  unsigned* d;
  (void)hipMalloc(&d, 2 * nwg * sizeof(unsigned));
  std::vector<unsigned> h(2 * nwg);
  const int words = (p.multiProcessorCount + 31) / 32;
  auto run = [&](const char* name, std::vector<unsigned> mask) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, words, mask.data()) != hipSuccess) { printf("%s: create failed\n", name); return; }
    (void)hipMemset(d, 0xff, 2 * nwg * sizeof(unsigned));
    hipLaunchKernelGGL(probe, dim3(nwg), dim3(64), 0, s, d, 20000);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    std::set<std::tuple<int, int, int>> used;
    std::vector<int> per_xcc(8, 0);
    for (int i = 0; i < nwg; ++i) {
      unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xf;
      int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x3;
      used.insert({(int)xcc, se * 2 + sh, cu});
    }
    for (auto& u : used) per_xcc[std::get<0>(u)]++;
    printf("%-24s distinct CUs %3zu  per XCC:", name, used.size());
    for (int x = 0; x < 8; ++x) printf(" %d", per_xcc[x]);
    printf("\n   first:");
    int k = 0;
    for (auto& u : used) { if (k++ < 12) printf(" (%d,%d,%d)", std::get<0>(u), std::get<1>(u), std::get<2>(u)); }
    printf("\n");
    (void)hipStreamDestroy(s);
  };
  std::vector<unsigned> all(words, 0xffffffffu);
  run("all", all);
  std::vector<unsigned> first64(words, 0u); first64[0] = first64[1] = 0xffffffffu;
  run("bits 0-63", first64);
  std::vector<unsigned> first32(words, 0u); first32[0] = 0xffffffffu;
  run("bits 0-31", first32);
  std::vector<unsigned> every4(words, 0x11111111u);
  run("every 4th bit", every4);
  // halves: are bits [0, 128) and [128, 256) disjoint CU sets?
  std::vector<unsigned> lo(words, 0u), hi(words, 0u);
  for (int w = 0; w < words; ++w) (w < words / 2 ? lo : hi)[w] = 0xffffffffu;
  run("bits 0-127", lo);
  run("bits 128-255", hi);
  {
    auto cus = [&](std::vector<unsigned> mask) {
      std::set<std::tuple<int, int, int>> used;
      hipStream_t s;
      if (hipExtStreamCreateWithCUMask(&s, words, mask.data()) != hipSuccess) return used;
      hipLaunchKernelGGL(probe, dim3(nwg), dim3(64), 0, s, d, 20000);
      (void)hipStreamSynchronize(s);
      (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
      for (int i = 0; i < nwg; ++i) {
        unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xf;
        used.insert({(int)xcc, (int)(((hw >> 13) & 3) * 2 + ((hw >> 12) & 1)), (int)((hw >> 8) & 0xf)});
      }
      (void)hipStreamDestroy(s);
      return used;
    };
    auto a = cus(lo), b = cus(hi);
    int both = 0;
    for (auto& u : a) both += b.count(u);
    printf("halves: %zu + %zu CUs, %d in both\n", a.size(), b.size(), both);
  }
  std::vector<unsigned> low8(words, 0u); low8[0] = 0xffu;
  run("bits 0-7", low8);
  std::vector<unsigned> not4(words, 0xeeeeeeeeu);
  run("all but every 4th", not4);
  return 0;
}
