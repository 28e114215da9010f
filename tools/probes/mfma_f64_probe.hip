// FP64 matrix-core probe (diagnostics for DESIGN.md, not part of the library): throughput and
// dependent-issue latency of v_mfma_f64_16x16x4_f64 and v_mfma_f64_4x4x4_4b_f64 on one MI355X.
// Throughput: 8 independent accumulators per wave, all CUs busy; latency: one dependent chain.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4_t __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ __launch_bounds__(256) void k16(double* out, int iters, double a, double b)
{
  f64x4_t acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f64x4_t{0.0, 0.0, 0.0, 0.0};
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  double s = 0.0;
  for (int c = 0; c < CHAINS; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
__global__ __launch_bounds__(256) void k4(double* out, int iters, double a, double b)
{
  double acc[CHAINS];
  for (int c = 0; c < CHAINS; ++c) acc[c] = 0.0;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[c], 0, 0, 0);
  double s = 0.0;
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class F>
static double time_ms(F launch)
{
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main()
{
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 8, threads = 256, iters = 4096;
  double* out;
  (void)hipMalloc(&out, sizeof(double) * blocks * threads);
  const double waves = double(blocks) * threads / 64.0;
  // throughput: 8 chains
  double ms = time_ms([&] { hipLaunchKernelGGL(k16<8>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0, 1e-9); });
  const double fl16 = waves * iters * 8 * 2.0 * 16 * 16 * 4;
  printf("16x16x4 f64: %.1f TF/s (%d CUs at the clock of this run)\n", fl16 / ms / 1e9, cus);
  ms = time_ms([&] { hipLaunchKernelGGL(k4<8>, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0, 1e-9); });
  const double fl4 = waves * iters * 8 * 2.0 * 4 * 4 * 4 * 4;  // 4 blocks of 4x4x4
  printf("4x4x4_4b f64: %.1f TF/s\n", fl4 / ms / 1e9);
  // dependent chain, one wave per SIMD: cycles per issue from the shader clock
  const int lat_iters = 1 << 16;
  ms = time_ms([&] { hipLaunchKernelGGL(k16<1>, dim3(cus), dim3(256), 0, 0, out, lat_iters, 1.0, 1e-9); });
  printf("16x16x4 f64 dependent chain: %.1f ns per MFMA\n", ms * 1e6 / lat_iters);
  ms = time_ms([&] { hipLaunchKernelGGL(k4<1>, dim3(cus), dim3(256), 0, 0, out, lat_iters, 1.0, 1e-9); });
  printf("4x4x4_4b f64 dependent chain: %.1f ns per MFMA\n", ms * 1e6 / lat_iters);
  (void)hipFree(out);
  return 0;
}
