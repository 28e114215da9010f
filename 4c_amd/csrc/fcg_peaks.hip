// fcg_peaks.hip -- on-box re-measurement of the two peaks SURVEY §8d prices the assembly against
// (HBM bandwidth, FP64 throughput): a STREAM triad over HBM-resident arrays, an FP64 VALU FMA loop
// and an FP64 MFMA loop (v_mfma_f64_16x16x4_f64), each timed with hipEvents over repeated
// launches that fill every CU.  bench.py reports these beside the spec peaks it divides by.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "fourc_gpu.h"
#include "fcg_status.hpp"

namespace {

template <int U>
__global__ __launch_bounds__(256) void triad_kernel(const double* __restrict__ b,
    const double* __restrict__ c, double* __restrict__ a, double s, int64_t n)
{
  // U 16-byte pieces per lane and array in flight (all loads issued before the stores), the
  // pieces of a wave one contiguous 1 KiB block apart; stores bypass the caches (written once)
  const int64_t step = 2 * int64_t(blockDim.x);
  const int64_t stride = int64_t(gridDim.x) * step * U;
  for (int64_t i = int64_t(blockIdx.x) * step * U + 2 * threadIdx.x; i < n; i += stride)
  {
    double2 bb[U], cc[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      bb[u] = *reinterpret_cast<const double2*>(b + i + u * step);
      cc[u] = *reinterpret_cast<const double2*>(c + i + u * step);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      double* dst = a + i + u * step;
      __builtin_nontemporal_store(bb[u].x + s * cc[u].x, dst);
      __builtin_nontemporal_store(bb[u].y + s * cc[u].y, dst + 1);
    }
  }
}

// copy: U 16-byte pieces per lane in flight, all loads before the stores; NT selects
// non-temporal stores
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const double2* __restrict__ b,
    double2* __restrict__ a, int64_t n2)
{
  const int64_t step = blockDim.x;
  const int64_t stride = int64_t(gridDim.x) * step * U;
  for (int64_t i = int64_t(blockIdx.x) * step * U + threadIdx.x; i < n2; i += stride)
  {
    double2 bb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) bb[u] = b[i + u * step];
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      if (NT)
      {
        __builtin_nontemporal_store(bb[u].x, &a[i + u * step].x);
        __builtin_nontemporal_store(bb[u].y, &a[i + u * step].y);
      }
      else
        a[i + u * step] = bb[u];
    }
  }
}

// write-only fill, U 16-byte stores per lane and iteration
template <int U, bool NT>
__global__ __launch_bounds__(256) void fill_kernel(double2* __restrict__ a, double v, int64_t n2)
{
  const int64_t step = blockDim.x;
  const int64_t stride = int64_t(gridDim.x) * step * U;
  for (int64_t i = int64_t(blockIdx.x) * step * U + threadIdx.x; i < n2; i += stride)
  {
#pragma unroll
    for (int u = 0; u < U; ++u)
    {
      if (NT)
      {
        __builtin_nontemporal_store(v, &a[i + u * step].x);
        __builtin_nontemporal_store(v, &a[i + u * step].y);
      }
      else
        a[i + u * step] = double2{v, v};
    }
  }
}

// NCH independent FMA chains per lane; the result is stored so nothing is dead code
constexpr int NCH = 16;
__global__ __launch_bounds__(256) void fma_kernel(double* out, int iters, double x)
{
  double v[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) v[k] = x + k + threadIdx.x;
  const double m = 0.999999, c = 1e-7;
  for (int i = 0; i < iters; ++i)
  {
#pragma unroll
    for (int k = 0; k < NCH; ++k) v[k] = fma(v[k], m, c);
  }
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < NCH; ++k) s += v[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// NACC independent accumulators of v_mfma_f64_16x16x4_f64 per wave (2 * 16 * 16 * 4 flop each)
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int NACC = 8;
__global__ __launch_bounds__(256) void mfma_kernel(double* out, int iters, double x)
{
  f64x4 acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = f64x4{0.0, 0.0, 0.0, 0.0};
  const double a = x + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int i = 0; i < iters; ++i)
  {
#pragma unroll
    for (int k = 0; k < NACC; ++k)
      acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < NACC; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class F>
float time_ms(hipStream_t s, int reps, F launch)
{
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();  // warm-up
  (void)hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms / reps;
}

}  // namespace

extern "C" int fcg_measure_peaks(int device, double* hbm_triad_gbs, double* fp64_valu_tflops,
    double* fp64_mfma_tflops)
{
  if (!fcg_use_device(device))
  {
    (void)hipGetLastError();  // do not leave the error for the caller's next HIP call
    return fcg_device_error();
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fcg_device_error();
  const int cus = std::max(1, prop.multiProcessorCount);
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return fcg_device_error();
  int rc = FCG_OK;
  // triad over 3 x 1 GiB (far beyond the 256 MB Infinity Cache)
  const int64_t n = int64_t(1) << 27;
  double *a = nullptr, *b = nullptr, *c = nullptr, *out = nullptr;
  const int grid_v = cus * 8, iters = 4096;
  if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&b, n * 8) != hipSuccess ||
      hipMalloc(&c, n * 8) != hipSuccess || hipMalloc(&out, int64_t(grid_v) * 256 * 8) != hipSuccess)
    rc = fcg_device_error();
  if (rc == FCG_OK)
  {
    (void)hipMemsetAsync(b, 0, n * 8, s);
    (void)hipMemsetAsync(c, 0, n * 8, s);
    // the best of a few in-flight depths / grid sizes (the figure is a peak)
    float ms = 1e30f;
    for (int g : {8, 16, 32})
    {
      ms = std::min(ms, time_ms(s, 10, [&] {
        hipLaunchKernelGGL(triad_kernel<4>, dim3(cus * g), dim3(256), 0, s, b, c, a, 3.0, n);
      }));
      ms = std::min(ms, time_ms(s, 10, [&] {
        hipLaunchKernelGGL(triad_kernel<2>, dim3(cus * g), dim3(256), 0, s, b, c, a, 3.0, n);
      }));
    }
    if (hbm_triad_gbs) *hbm_triad_gbs = 3.0 * 8.0 * double(n) / (ms * 1e-3) / 1e9;
    const float mv = time_ms(s, 5, [&] {
      hipLaunchKernelGGL(fma_kernel, dim3(grid_v), dim3(256), 0, s, out, iters, 1.0);
    });
    if (fp64_valu_tflops)
      *fp64_valu_tflops = 2.0 * NCH * double(iters) * grid_v * 256 / (mv * 1e-3) / 1e12;
    const float mm = time_ms(s, 5, [&] {
      hipLaunchKernelGGL(mfma_kernel, dim3(grid_v), dim3(256), 0, s, out, iters / NACC, 1.0);
    });
    // per wave and instruction: 16 x 16 x 4 multiply-adds
    if (fp64_mfma_tflops)
      *fp64_mfma_tflops =
          2.0 * 1024.0 * NACC * double(iters / NACC) * grid_v * 4 / (mm * 1e-3) / 1e12;
    if (hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess) rc = fcg_device_error();
  }
  for (double* p : {a, b, c, out})
    if (p) (void)hipFree(p);
  (void)hipStreamDestroy(s);
  return rc;
}

extern "C" int fcg_measure_hbm(int device, double* copy_gbs, double* write_gbs)
{
  if (!fcg_use_device(device))
  {
    (void)hipGetLastError();  // do not leave the error for the caller's next HIP call
    return fcg_device_error();
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fcg_device_error();
  const int cus = std::max(1, prop.multiProcessorCount);
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return fcg_device_error();
  int rc = FCG_OK;
  // 2 x 2 GiB: far beyond the 256 MB Infinity Cache
  const int64_t n2 = int64_t(1) << 27;  // double2 elements = 2 GiB
  double2 *a = nullptr, *b = nullptr;
  if (hipMalloc(&a, n2 * 16) != hipSuccess || hipMalloc(&b, n2 * 16) != hipSuccess) rc = fcg_device_error();
  if (rc == FCG_OK)
  {
    (void)hipMemsetAsync(b, 0, n2 * 16, s);
    float mc = 1e30f, mw = 1e30f;
    for (int g : {4, 8, 16, 32})
    {
      const dim3 grid(cus * g), blk(256);
      mc = std::min(mc, time_ms(s, 10, [&] { hipLaunchKernelGGL((copy_kernel<4, false>), grid, blk, 0, s, b, a, n2); }));
      mc = std::min(mc, time_ms(s, 10, [&] { hipLaunchKernelGGL((copy_kernel<4, true>), grid, blk, 0, s, b, a, n2); }));
      mc = std::min(mc, time_ms(s, 10, [&] { hipLaunchKernelGGL((copy_kernel<2, false>), grid, blk, 0, s, b, a, n2); }));
      mw = std::min(mw, time_ms(s, 10, [&] { hipLaunchKernelGGL((fill_kernel<4, false>), grid, blk, 0, s, a, 1.0, n2); }));
      mw = std::min(mw, time_ms(s, 10, [&] { hipLaunchKernelGGL((fill_kernel<4, true>), grid, blk, 0, s, a, 1.0, n2); }));
    }
    if (copy_gbs) *copy_gbs = 2.0 * 16.0 * double(n2) / (mc * 1e-3) / 1e9;
    if (write_gbs) *write_gbs = 16.0 * double(n2) / (mw * 1e-3) / 1e9;
    if (hipStreamSynchronize(s) != hipSuccess || hipGetLastError() != hipSuccess) rc = fcg_device_error();
  }
  for (double2* p : {a, b})
    if (p) (void)hipFree(p);
  (void)hipStreamDestroy(s);
  return rc;
}
