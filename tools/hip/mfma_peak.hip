// fp64 MFMA ceiling on this part (dev tool): 16 independent v_mfma_f64_16x16x4_f64
// chains per wave, no memory traffic; also the shader clock under that load.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_peak(double* out, int iters, unsigned long long* clk) {
  d4 acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
  double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
  const unsigned long long c0 = __builtin_readcyclecounter();
  const unsigned long long w0 = wall_clock64();
  for (int it = 0; it < iters; it += 32) {
#pragma unroll
    for (int u = 0; u < 32; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  const unsigned long long c1 = __builtin_readcyclecounter();
  const unsigned long long w1 = wall_clock64();
  double s = 0.0;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = c1 - c0; clk[1] = w1 - w0; }
}

int main() {
  const int blocks = 256 * 2, iters = 20000;
  double* out; unsigned long long* clk;
  hipMalloc(&out, blocks * 256 * 8); hipMalloc(&clk, 16);
  hipLaunchKernelGGL(k_peak, dim3(blocks), dim3(256), 0, 0, out, 100, clk);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int wpb = 1; wpb <= 2; ++wpb) {
    const int nb = 256 * wpb;
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_peak, dim3(nb), dim3(256), 0, 0, out, iters, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double flops = (double)nb * 4 * iters * 16 * 2048.0;
    printf("%d WG/CU: %.3f ms  %.2f TF/s  shader clock %.3f GHz (cycles %llu over %.1f us)\n", wpb, ms,
           flops / ms / 1e9, c[0] / (c[1] * 0.01) / 1e3, c[0], c[1] * 0.01);
  }
  return 0;
}
