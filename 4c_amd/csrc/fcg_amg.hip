// fcg_amg.hip -- the numeric half of the smoothed-aggregation AMG (SURVEY §8f row 2 on meshes
// without a box hierarchy; the graph half and the algorithm's description are fcg_amg_setup.cpp).
// All matrices of the hierarchy are block CSR (BSR) in HBM: block rows = nodes (3 DOFs on the
// fine level, 6 = the rigid-body modes on the coarse levels), blocks row-major, int64 block row
// pointers.  Per tangent the hierarchy is recomputed on the device from the fixed patterns:
//   A_0 (BSR copy of the context's K)  -> P_0 = (I - omega D^-1 A_0) T_0   (T = tentative)
//   A_1 = P_0^T (A_0 P_0), and so on;   the coarsest A_L becomes dense (fcg_bsr_to_dense).
// Kernels: block SpMV (8 lanes per block row), block SpGEMM with a known output pattern (16 lanes
// per output row, one lane per output block, the right operand's rows binary-searched: fixed
// summation order, bitwise reproducible), block transpose, block-diagonal
// inverse (Gauss-Jordan in registers; empty coarse rows -- the zero columns of rank-deficient
// aggregates -- get a unit diagonal), and the prolongator smoothing.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "fourc_gpu.h"
#include "fcg_status.hpp"

namespace fcg_bsrk {

constexpr int kBlock = 256;

inline unsigned blocks_for(int64_t n, int per_block) { return unsigned((n + per_block - 1) / per_block); }

// y = alpha A x (+ y): LPN lanes per block row, blocks strided over the lanes, butterfly sum
template <int BR, int BC, int LPN = 8>
__global__ __launch_bounds__(kBlock) void bsr_spmv_kernel(int64_t n, const int64_t* __restrict__ ptr,
    const int32_t* __restrict__ col, const double* __restrict__ vals, const double* __restrict__ x,
    double* y, double alpha, int accumulate)
{
  const int64_t row = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / LPN;
  const int lane = threadIdx.x % LPN;
  double acc[BR];
#pragma unroll
  for (int r = 0; r < BR; ++r) acc[r] = 0.0;
  if (row < n)
  {
    const int64_t k1 = ptr[row + 1];
    for (int64_t k = ptr[row] + lane; k < k1; k += LPN)
    {
      const double* v = vals + k * (BR * BC);
      const double* xc = x + int64_t(col[k]) * BC;
      double xv[BC];
#pragma unroll
      for (int c = 0; c < BC; ++c) xv[c] = xc[c];
#pragma unroll
      for (int r = 0; r < BR; ++r)
#pragma unroll
        for (int c = 0; c < BC; ++c) acc[r] += v[r * BC + c] * xv[c];
    }
  }
#pragma unroll
  for (int o = LPN / 2; o >= 1; o >>= 1)
#pragma unroll
    for (int r = 0; r < BR; ++r) acc[r] += __shfl_xor(acc[r], o, LPN);
  if (row < n && lane == 0)
#pragma unroll
    for (int r = 0; r < BR; ++r)
      y[row * BR + r] = alpha * acc[r] + (accumulate ? y[row * BR + r] : 0.0);
}

// C = A B on C's given pattern: 16 lanes per block row of C (four rows per wavefront), one lane
// per output block (strided), walking A's row in order and binary-searching B's row for the
// block's column: a fixed summation order, bitwise reproducible.  (An LDS row image built
// sequentially over A's blocks measured slower: it serialises the dependent loads of every block.)
template <int BR, int BK, int BC>
__global__ __launch_bounds__(kBlock) void bsr_spgemm_kernel(int64_t n,
    const int64_t* __restrict__ a_ptr, const int32_t* __restrict__ a_col,
    const double* __restrict__ a_vals, const int64_t* __restrict__ b_ptr,
    const int32_t* __restrict__ b_col, const double* __restrict__ b_vals,
    const int64_t* __restrict__ c_ptr, const int32_t* __restrict__ c_col, double* c_vals)
{
  constexpr int LPR = 16;
  const int64_t row = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / LPR;
  const int lane = threadIdx.x % LPR;
  if (row >= n) return;
  const int64_t a0 = a_ptr[row], a1 = a_ptr[row + 1];
  const int64_t c1 = c_ptr[row + 1];
  for (int64_t ci = c_ptr[row] + lane; ci < c1; ci += LPR)
  {
    const int32_t tc = c_col[ci];
    double acc[BR * BC];
#pragma unroll
    for (int q = 0; q < BR * BC; ++q) acc[q] = 0.0;
    for (int64_t ak = a0; ak < a1; ++ak)
    {
      const int32_t k = a_col[ak];
      const int64_t e = b_ptr[k + 1];
      int64_t lo = b_ptr[k], hi = e;
      while (lo < hi)
      {
        const int64_t mid = (lo + hi) >> 1;
        if (b_col[mid] < tc) lo = mid + 1;
        else hi = mid;
      }
      if (lo < e && b_col[lo] == tc)
      {
        const double* A = a_vals + ak * (BR * BK);
        const double* B = b_vals + lo * (BK * BC);
#pragma unroll
        for (int r = 0; r < BR; ++r)
#pragma unroll
          for (int q = 0; q < BK; ++q)
          {
            const double av = A[r * BK + q];
#pragma unroll
            for (int c = 0; c < BC; ++c) acc[r * BC + c] += av * B[q * BC + c];
          }
      }
    }
    double* out = c_vals + ci * (BR * BC);
#pragma unroll
    for (int q = 0; q < BR * BC; ++q) out[q] = acc[q];
  }
}

// C = A B from a product plan (fcg_bsr_spgemm_planned): the (A block, B block) pairs of every C
// block, listed once on the host in A's row order -- the pairs bsr_spgemm_kernel finds by its
// searches, so the same products in the same order (bitwise equal).  One thread per C block.
template <int BR, int BK, int BC>
__global__ __launch_bounds__(kBlock) void bsr_spgemm_plan_kernel(int64_t n_out,
    const int64_t* __restrict__ pptr, const int32_t* __restrict__ pa, const int32_t* __restrict__ pb,
    const double* __restrict__ a_vals, const double* __restrict__ b_vals, double* c_vals,
    const int64_t* __restrict__ order)
{
  const int64_t t0 = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t0 >= n_out) return;
  const int64_t ci = order ? order[t0] : t0;
  double acc[BR * BC];
#pragma unroll
  for (int q = 0; q < BR * BC; ++q) acc[q] = 0.0;
  const int64_t t1 = pptr[ci + 1];
  for (int64_t t = pptr[ci]; t < t1; ++t)
  {
    const double* A = a_vals + int64_t(pa[t]) * (BR * BK);
    const double* B = b_vals + int64_t(pb[t]) * (BK * BC);
#pragma unroll
    for (int r = 0; r < BR; ++r)
#pragma unroll
      for (int q = 0; q < BK; ++q)
      {
        const double av = A[r * BK + q];
#pragma unroll
        for (int c = 0; c < BC; ++c) acc[r * BC + c] += av * B[q * BC + c];
      }
  }
  double* out = c_vals + ci * (BR * BC);
#pragma unroll
  for (int q = 0; q < BR * BC; ++q) out[q] = acc[q];
}

// t_vals[t] = vals[perm[t]]^T (BR x BC -> BC x BR)
template <int BR, int BC>
__global__ __launch_bounds__(kBlock) void bsr_transpose_kernel(int64_t nnzb,
    const int64_t* __restrict__ perm, const double* __restrict__ vals, double* t_vals)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= nnzb) return;
  const double* s = vals + perm[t] * (BR * BC);
  double* d = t_vals + t * (BR * BC);
#pragma unroll
  for (int r = 0; r < BR; ++r)
#pragma unroll
    for (int c = 0; c < BC; ++c) d[c * BR + r] = s[r * BC + c];
}

// the context's node-triple CSR (the 3 rows of block row b are rows 3b..3b+2, sharing one pattern
// of DOF triples) into 3 x 3 BSR blocks; 16 lanes per block row
__global__ __launch_bounds__(kBlock) void node_csr_to_bsr_kernel(int64_t n,
    const int64_t* __restrict__ rowptr, const int64_t* __restrict__ b_ptr,
    const double* __restrict__ K, double* b_vals)
{
  const int64_t b = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (b >= n) return;
  const int64_t r0 = rowptr[3 * b], r1 = rowptr[3 * b + 1], r2 = rowptr[3 * b + 2];
  const int64_t nb = b_ptr[b + 1] - b_ptr[b];
  for (int64_t m = lane; m < nb; m += 16)
  {
    double* o = b_vals + (b_ptr[b] + m) * 9;
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      o[c] = K[r0 + 3 * m + c];
      o[3 + c] = K[r1 + 3 * m + c];
      o[6 + c] = K[r2 + 3 * m + c];
    }
  }
}

// D_ii^-1 per block row (row-major), Gauss-Jordan on the diagonal block.  A scalar row that is
// zero across the whole block row (a coarse DOF of a zero tentative column) first gets a unit
// diagonal in `vals`, so that the coarse operator stays nonsingular and that DOF decoupled.
template <int B>
__global__ __launch_bounds__(kBlock) void bsr_block_inverse_kernel(int64_t n,
    const int64_t* __restrict__ ptr, const int64_t* __restrict__ diag_idx, double* vals,
    double* dinv, int32_t* bad)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t di = diag_idx[i];
  if (di < 0)
  {
    atomicMax(bad, 1);
    return;
  }
  double* D = vals + di * (B * B);
#pragma unroll
  for (int d = 0; d < B; ++d)
  {
    bool empty = true;
    for (int64_t k = ptr[i]; k < ptr[i + 1] && empty; ++k)
#pragma unroll
      for (int c = 0; c < B; ++c) empty = empty && vals[k * (B * B) + d * B + c] == 0.0;
    if (empty) D[d * B + d] = 1.0;
  }
  double a[B][B], v[B][B];
#pragma unroll
  for (int r = 0; r < B; ++r)
#pragma unroll
    for (int c = 0; c < B; ++c)
    {
      a[r][c] = D[r * B + c];
      v[r][c] = r == c ? 1.0 : 0.0;
    }
  bool ok = true;
#pragma unroll
  for (int p = 0; p < B; ++p)
  {
    const double piv = a[p][p];
    ok = ok && piv != 0.0 && piv == piv;
    const double ip = 1.0 / piv;
#pragma unroll
    for (int c = 0; c < B; ++c)
    {
      a[p][c] *= ip;
      v[p][c] *= ip;
    }
#pragma unroll
    for (int r = 0; r < B; ++r)
    {
      if (r == p) continue;
      const double f = a[r][p];
#pragma unroll
      for (int c = 0; c < B; ++c)
      {
        a[r][c] -= f * a[p][c];
        v[r][c] -= f * v[p][c];
      }
    }
  }
  double* o = dinv + i * (B * B);
#pragma unroll
  for (int r = 0; r < B; ++r)
#pragma unroll
    for (int c = 0; c < B; ++c) o[r * B + c] = ok ? v[r][c] : 0.0;
  if (!ok) atomicMax(bad, 2);
}

// z = scale D^-1 r (+ z)
template <int B>
__global__ __launch_bounds__(kBlock) void bsr_bj_apply_kernel(int64_t n,
    const double* __restrict__ dinv, const double* __restrict__ r, double* z, double scale,
    int accumulate)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  double rv[B];
#pragma unroll
  for (int c = 0; c < B; ++c) rv[c] = r[i * B + c];
  const double* D = dinv + i * (B * B);
#pragma unroll
  for (int q = 0; q < B; ++q)
  {
    double t = 0.0;
#pragma unroll
    for (int c = 0; c < B; ++c) t += D[q * B + c] * rv[c];
    z[i * B + q] = scale * t + (accumulate ? z[i * B + q] : 0.0);
  }
}

// P_iJ = [J == agg(i)] T_i - omega D_i^-1 (A T)_iJ on P's pattern (= the pattern of A T)
template <int BR>
__global__ __launch_bounds__(kBlock) void smooth_prolongator_kernel(int64_t n,
    const int64_t* __restrict__ p_ptr, const int32_t* __restrict__ p_col,
    const int32_t* __restrict__ agg, const double* __restrict__ tent,
    const double* __restrict__ dinv, const double* __restrict__ at, double omega, double* p_vals)
{
  constexpr int BC = 6;
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  double D[BR * BR];
#pragma unroll
  for (int q = 0; q < BR * BR; ++q) D[q] = dinv[i * (BR * BR) + q];
  const int32_t ai = agg[i];
  for (int64_t k = p_ptr[i]; k < p_ptr[i + 1]; ++k)
  {
    const double* s = at + k * (BR * BC);
    double* o = p_vals + k * (BR * BC);
    const bool own = p_col[k] == ai;
#pragma unroll
    for (int r = 0; r < BR; ++r)
#pragma unroll
      for (int c = 0; c < BC; ++c)
      {
        double t = 0.0;
#pragma unroll
        for (int q = 0; q < BR; ++q) t += D[r * BR + q] * s[q * BC + c];
        o[r * BC + c] = (own ? tent[i * (BR * BC) + r * BC + c] : 0.0) - omega * t;
      }
  }
}

// dense row-major copy (n B x n B) of a BSR matrix (the coarsest level's direct solve)
template <int B>
__global__ __launch_bounds__(kBlock) void bsr_to_dense_kernel(int64_t n,
    const int64_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const double* __restrict__ vals, double* dense)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t N = n * B;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
  {
    const int64_t c0 = int64_t(col[k]) * B;
#pragma unroll
    for (int r = 0; r < B; ++r)
#pragma unroll
      for (int c = 0; c < B; ++c) dense[(i * B + r) * N + c0 + c] = vals[k * (B * B) + r * B + c];
  }
}

inline int status(hipError_t e) { return e == hipSuccess ? FCG_OK : fcg_device_error(); }

}  // namespace fcg_bsrk

extern "C" {

int fcg_bsr_spmv(int device, int br, int bc, int64_t n_brows, const int64_t* d_ptr,
    const int32_t* d_col, const double* d_vals, const double* d_x, double* d_y, double alpha,
    int accumulate, void* stream)
{
  using namespace fcg_bsrk;
  if (n_brows < 0 || (n_brows > 0 && (!d_ptr || !d_col || !d_vals || !d_x || !d_y))) return FCG_ERR_ARG;
  if (n_brows == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(blocks_for(n_brows * 8, kBlock)), b(kBlock);
  // 3 x 3 (an AMG level 0: ~27 blocks per row): 32 lanes per row, about one block each (renumbered
  // 1M hex8 AMG Newton 0.350 / 0.341 / 0.330 s at 8 / 16 / 32 lanes, profiles/r04/r04_bsr_lpn_ab.txt;
  // FCG_BSR_LPN33 = 4, 8, 16 for A/B)
  static const int lpn33 = [] {
    const char* e = std::getenv("FCG_BSR_LPN33");
    return e ? std::atoi(e) : 32;
  }();
  static const int lpn63 = [] {  // restriction P^T: 8 lanes (32: no difference, r04_bsr_lpn63_ab.txt)
    const char* e = std::getenv("FCG_BSR_LPN63");
    return e ? std::atoi(e) : 8;
  }();
  static const int lpn66 = [] {  // 6 x 6 coarse levels: 32 lanes (0.329 -> 0.321 s, r04_bsr_lpn66_ab.txt)
    const char* e = std::getenv("FCG_BSR_LPN66");
    return e ? std::atoi(e) : 32;
  }();
  if (br == 3 && bc == 3 && lpn33 == 4)
    hipLaunchKernelGGL((bsr_spmv_kernel<3, 3, 4>), dim3(blocks_for(n_brows * 4, kBlock)), b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else if (br == 3 && bc == 3 && lpn33 == 16)
    hipLaunchKernelGGL((bsr_spmv_kernel<3, 3, 16>), dim3(blocks_for(n_brows * 16, kBlock)), b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else if (br == 3 && bc == 3 && lpn33 == 8)
    hipLaunchKernelGGL((bsr_spmv_kernel<3, 3>), g, b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else if (br == 3 && bc == 3)
    hipLaunchKernelGGL((bsr_spmv_kernel<3, 3, 32>), dim3(blocks_for(n_brows * 32, kBlock)), b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else if (br == 3 && bc == 6)
    hipLaunchKernelGGL((bsr_spmv_kernel<3, 6>), g, b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else if (br == 6 && bc == 3 && lpn63 == 8)
    hipLaunchKernelGGL((bsr_spmv_kernel<6, 3>), g, b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else if (br == 6 && bc == 3)
    hipLaunchKernelGGL((bsr_spmv_kernel<6, 3, 32>), dim3(blocks_for(n_brows * 32, kBlock)), b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else if (br == 6 && bc == 6 && lpn66 == 16)
    hipLaunchKernelGGL((bsr_spmv_kernel<6, 6, 16>), dim3(blocks_for(n_brows * 16, kBlock)), b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else if (br == 6 && bc == 6 && lpn66 == 8)
    hipLaunchKernelGGL((bsr_spmv_kernel<6, 6>), g, b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else if (br == 6 && bc == 6)
    hipLaunchKernelGGL((bsr_spmv_kernel<6, 6, 32>), dim3(blocks_for(n_brows * 32, kBlock)), b, 0, s, n_brows, d_ptr, d_col, d_vals, d_x, d_y, alpha, accumulate);
  else
    return FCG_ERR_ARG;
  return status(hipGetLastError());
}

int fcg_bsr_spgemm(int device, int br, int bk, int bc, int64_t n_brows, const int64_t* d_a_ptr,
    const int32_t* d_a_col, const double* d_a_vals, const int64_t* d_b_ptr, const int32_t* d_b_col,
    const double* d_b_vals, const int64_t* d_c_ptr, const int32_t* d_c_col, double* d_c_vals,
    void* stream)
{
  using namespace fcg_bsrk;
  if (n_brows < 0 || (n_brows > 0 && (!d_a_ptr || !d_a_col || !d_a_vals || !d_b_ptr || !d_b_col ||
                                      !d_b_vals || !d_c_ptr || !d_c_col || !d_c_vals)))
    return FCG_ERR_ARG;
  if (n_brows == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(blocks_for(n_brows * 16, kBlock)), b(kBlock);
#define FCG_SPGEMM(R, K, C)                                                                        \
  hipLaunchKernelGGL((bsr_spgemm_kernel<R, K, C>), g, b, 0, s, n_brows, d_a_ptr, d_a_col, d_a_vals, \
      d_b_ptr, d_b_col, d_b_vals, d_c_ptr, d_c_col, d_c_vals)
  if (br == 3 && bk == 3 && bc == 6) FCG_SPGEMM(3, 3, 6);
  else if (br == 6 && bk == 3 && bc == 6) FCG_SPGEMM(6, 3, 6);
  else if (br == 6 && bk == 6 && bc == 6) FCG_SPGEMM(6, 6, 6);
  else if (br == 3 && bk == 3 && bc == 3) FCG_SPGEMM(3, 3, 3);
  else return FCG_ERR_ARG;
#undef FCG_SPGEMM
  return status(hipGetLastError());
}

int fcg_bsr_spgemm_planned(int device, int br, int bk, int bc, int64_t nnzb_c, const int64_t* d_pair_ptr,
    const int32_t* d_pair_a, const int32_t* d_pair_b, const double* d_a_vals, const double* d_b_vals,
    double* d_c_vals, const int64_t* d_order, void* stream)
{
  using namespace fcg_bsrk;
  if (nnzb_c < 0 || (nnzb_c > 0 && (!d_pair_ptr || !d_pair_a || !d_pair_b || !d_a_vals || !d_b_vals || !d_c_vals)))
    return FCG_ERR_ARG;
  if (nnzb_c == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(blocks_for(nnzb_c, kBlock)), b(kBlock);
#define FCG_SPGEMM_P(R, K, C)                                                                      \
  hipLaunchKernelGGL((bsr_spgemm_plan_kernel<R, K, C>), g, b, 0, s, nnzb_c, d_pair_ptr, d_pair_a,  \
      d_pair_b, d_a_vals, d_b_vals, d_c_vals, d_order)
  if (br == 3 && bk == 3 && bc == 6) FCG_SPGEMM_P(3, 3, 6);
  else if (br == 6 && bk == 3 && bc == 6) FCG_SPGEMM_P(6, 3, 6);
  else if (br == 6 && bk == 6 && bc == 6) FCG_SPGEMM_P(6, 6, 6);
  else if (br == 3 && bk == 3 && bc == 3) FCG_SPGEMM_P(3, 3, 3);
  else return FCG_ERR_ARG;
#undef FCG_SPGEMM_P
  return status(hipGetLastError());
}

int fcg_bsr_transpose_values(int device, int br, int bc, int64_t nnzb, const int64_t* d_perm,
    const double* d_vals, double* d_t_vals, void* stream)
{
  using namespace fcg_bsrk;
  if (nnzb < 0 || (nnzb > 0 && (!d_perm || !d_vals || !d_t_vals))) return FCG_ERR_ARG;
  if (nnzb == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(blocks_for(nnzb, kBlock)), b(kBlock);
  if (br == 3 && bc == 6)
    hipLaunchKernelGGL((bsr_transpose_kernel<3, 6>), g, b, 0, s, nnzb, d_perm, d_vals, d_t_vals);
  else if (br == 6 && bc == 6)
    hipLaunchKernelGGL((bsr_transpose_kernel<6, 6>), g, b, 0, s, nnzb, d_perm, d_vals, d_t_vals);
  else
    return FCG_ERR_ARG;
  return status(hipGetLastError());
}

int fcg_bsr_from_node_csr(int device, int64_t n_brows, const int64_t* d_rowptr,
    const int64_t* d_b_ptr, const double* d_K, double* d_b_vals, void* stream)
{
  using namespace fcg_bsrk;
  if (n_brows < 0 || (n_brows > 0 && (!d_rowptr || !d_b_ptr || !d_K || !d_b_vals))) return FCG_ERR_ARG;
  if (n_brows == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(node_csr_to_bsr_kernel, dim3(blocks_for(n_brows * 16, kBlock)), dim3(kBlock), 0,
      s, n_brows, d_rowptr, d_b_ptr, d_K, d_b_vals);
  return status(hipGetLastError());
}

int fcg_bsr_block_jacobi_setup(int device, int b, int64_t n_brows, const int64_t* d_ptr,
    const int64_t* d_diag_idx, double* d_vals, double* d_dinv, int32_t* d_flag, void* stream)
{
  using namespace fcg_bsrk;
  if (n_brows < 0 || !d_flag || (n_brows > 0 && (!d_ptr || !d_diag_idx || !d_vals || !d_dinv)))
    return FCG_ERR_ARG;
  if (n_brows == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t he = hipMemsetAsync(d_flag, 0, sizeof(int32_t), s);
  if (he != hipSuccess) return fcg_device_error();
  const dim3 g(blocks_for(n_brows, kBlock)), bl(kBlock);
  if (b == 3)
    hipLaunchKernelGGL((bsr_block_inverse_kernel<3>), g, bl, 0, s, n_brows, d_ptr, d_diag_idx, d_vals, d_dinv, d_flag);
  else if (b == 6)
    hipLaunchKernelGGL((bsr_block_inverse_kernel<6>), g, bl, 0, s, n_brows, d_ptr, d_diag_idx, d_vals, d_dinv, d_flag);
  else
    return FCG_ERR_ARG;
  he = hipGetLastError();
  int32_t bad = 0;
  if (he == hipSuccess) he = hipMemcpyAsync(&bad, d_flag, sizeof(bad), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess) return fcg_device_error();
  return bad ? FCG_ERR_SINGULAR : FCG_OK;
}

int fcg_bsr_block_jacobi_apply(int device, int b, int64_t n_brows, const double* d_dinv,
    const double* d_r, double* d_z, double scale, int accumulate, void* stream)
{
  using namespace fcg_bsrk;
  if (n_brows < 0 || (n_brows > 0 && (!d_dinv || !d_r || !d_z))) return FCG_ERR_ARG;
  if (n_brows == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(blocks_for(n_brows, kBlock)), bl(kBlock);
  if (b == 3)
    hipLaunchKernelGGL((bsr_bj_apply_kernel<3>), g, bl, 0, s, n_brows, d_dinv, d_r, d_z, scale, accumulate);
  else if (b == 6)
    hipLaunchKernelGGL((bsr_bj_apply_kernel<6>), g, bl, 0, s, n_brows, d_dinv, d_r, d_z, scale, accumulate);
  else
    return FCG_ERR_ARG;
  return status(hipGetLastError());
}

int fcg_amg_smooth_prolongator(int device, int br, int64_t n_brows, const int64_t* d_p_ptr,
    const int32_t* d_p_col, const int32_t* d_agg, const double* d_tent, const double* d_dinv,
    const double* d_at, double omega, double* d_p_vals, void* stream)
{
  using namespace fcg_bsrk;
  if (n_brows < 0 || (n_brows > 0 && (!d_p_ptr || !d_p_col || !d_agg || !d_tent || !d_dinv ||
                                      !d_at || !d_p_vals)))
    return FCG_ERR_ARG;
  if (n_brows == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(blocks_for(n_brows, kBlock)), bl(kBlock);
  if (br == 3)
    hipLaunchKernelGGL((smooth_prolongator_kernel<3>), g, bl, 0, s, n_brows, d_p_ptr, d_p_col, d_agg, d_tent, d_dinv, d_at, omega, d_p_vals);
  else if (br == 6)
    hipLaunchKernelGGL((smooth_prolongator_kernel<6>), g, bl, 0, s, n_brows, d_p_ptr, d_p_col, d_agg, d_tent, d_dinv, d_at, omega, d_p_vals);
  else
    return FCG_ERR_ARG;
  return status(hipGetLastError());
}

int fcg_bsr_to_dense(int device, int b, int64_t n_brows, const int64_t* d_ptr, const int32_t* d_col,
    const double* d_vals, double* d_dense, void* stream)
{
  using namespace fcg_bsrk;
  if (n_brows < 0 || (n_brows > 0 && (!d_ptr || !d_col || !d_vals || !d_dense))) return FCG_ERR_ARG;
  if (n_brows == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(blocks_for(n_brows, kBlock)), bl(kBlock);
  if (b == 3)
    hipLaunchKernelGGL((bsr_to_dense_kernel<3>), g, bl, 0, s, n_brows, d_ptr, d_col, d_vals, d_dense);
  else if (b == 6)
    hipLaunchKernelGGL((bsr_to_dense_kernel<6>), g, bl, 0, s, n_brows, d_ptr, d_col, d_vals, d_dense);
  else
    return FCG_ERR_ARG;
  return status(hipGetLastError());
}

}  // extern "C"
