// Issue/latency of v_mfma_f64_16x16x4f64 on one wave, and of an LDS read round trip (dev tool).
// hipcc --offload-arch=gfx950 -O3 -w tools/hip/mfma_lat.hip -o tools/hip/mfma_lat_bin
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

// CH independent accumulator chains, N MFMAs each
template <int CH>
__global__ void __launch_bounds__(512) k_chain(double* out, unsigned long long* t, int n) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + lane * 1e-3, b = 1.0 - lane * 1e-3;
  d4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
  const unsigned long long s0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][3];
  const unsigned long long s1 = clock64();
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) t[0] = s1 - s0;
}

// MFMA result read by VALU then fed back as an operand (the leaf's pattern)
__global__ void __launch_bounds__(64) k_roundtrip(double* out, unsigned long long* t, int n) {
  const int lane = threadIdx.x;
  double a = 1.0 + lane * 1e-3, b = 1e-3;
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
  const unsigned long long s0 = clock64();
  for (int i = 0; i < n; ++i) {
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    a = acc[1] * 1e-3 + 1.0;
  }
  const unsigned long long s1 = clock64();
  out[lane] = acc[0] + a;
  if (lane == 0) t[0] = s1 - s0;
}

// dependent LDS read chain
__global__ void __launch_bounds__(64) k_lds(double* out, unsigned long long* t, int n) {
  __shared__ double l[1024];
  const int lane = threadIdx.x;
  for (int e = lane; e < 1024; e += 64) l[e] = (double)((e + 1) & 1023);
  __syncthreads();
  double v = lane;
  const unsigned long long s0 = clock64();
  for (int i = 0; i < n; ++i) v = l[(int)v];
  const unsigned long long s1 = clock64();
  out[lane] = v;
  if (lane == 0) t[0] = s1 - s0;
}

int main() {
  double* out;
  unsigned long long* t;
  hipMalloc(&out, 512 * 8);
  hipMalloc(&t, 8);
  const int n = 4096;
  auto run = [&](const char* name, void (*k)(double*, unsigned long long*, int), int per, int threads = 64) {
    unsigned long long th = 0;
    for (int it = 0; it < 3; ++it) {
      hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, out, t, n);
      hipDeviceSynchronize();
      hipMemcpy(&th, t, 8, hipMemcpyDeviceToHost);
    }
    printf("%-28s %.1f cycles per step (%d ops per step)\n", name, (double)th / n, per);
  };
  run("mfma 1 chain", k_chain<1>, 1);
  run("mfma 2 chains", k_chain<2>, 2);
  run("mfma 4 chains", k_chain<4>, 4);
  run("mfma 8 chains", k_chain<8>, 8);
  run("mfma 4 chains, 4 waves", k_chain<4>, 4, 256);
  run("mfma 4 chains, 8 waves", k_chain<4>, 4, 512);
  run("mfma 2 chains, 8 waves", k_chain<2>, 2, 512);
  run("mfma 1 chain, 8 waves", k_chain<1>, 1, 512);
  run("mfma -> valu -> mfma", k_roundtrip, 1);
  run("dependent ds_read_b64", k_lds, 1);
  return 0;
}
