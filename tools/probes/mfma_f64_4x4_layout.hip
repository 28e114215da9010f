// Operand / result lane layout of v_mfma_f64_4x4x4_4b_f64 (diagnostic, not part of the library):
// A lane l holds 2^(l % 16) (block l / 16), B is 1 on lane t only; the result on every lane tells
// which A lanes of its block met B's lane t.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* out, int t)
{
  const int l = threadIdx.x;
  const double a = double(1u << (l % 16));
  const double b = l == t ? 1.0 : 0.0;
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}
int main()
{
  double* d;
  (void)hipMalloc(&d, 64 * sizeof(double));
  double h[64];
  for (int t = 0; t < 64; ++t)
  {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, t);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("B lane %2d:", t);
    for (int l = 0; l < 64; ++l)
      if (h[l] != 0.0) printf(" D%d=%x", l, unsigned(h[l]));
    printf("\n");
  }
  return 0;
}
