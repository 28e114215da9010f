// fcg_dsolve.hip -- the linear solve across ranks behind the C ABI (fcg_dfcg_solve): what 4C's
// Newton hands to Belos CG with a MueLu / Ifpack preconditioner on every rank
// (4C_solver_nonlin_nox_linearsystem.cpp:275-353, 4C_linear_solver_preconditioner_muelu.cpp),
// on the ghost-layer partition of the element evaluation (SURVEY §8e option A):
//   * the SpMV of the rank's owned rows needs the search direction on the column map: one import
//     per iteration (Epetra_CrsMatrix::Multiply's Importer = fcg_halo_import over RCCL);
//   * the preconditioner: the rank's fcg_amg -- aggregation and level-0 smoothing on the owned
//     block (MueLu's uncoupled aggregation also aggregates within a rank), the coarse levels
//     coupled across the ranks (A_1 = P_0^T A P_0 of the global operator, gathered and solved
//     redundantly; fcg_amgs::Coupled in fcg_amg_solver.hip) when the transport names its rank and
//     rank count -- or the nodal block Jacobi;
//   * the inner products are fixed-order partial sums on each rank plus one all-reduce of a small
//     device buffer (two per iteration), so the iterates are independent of the launch geometry.
// Flexible CG (Polak-Ribiere beta), as the single-rank fcg_amg_iterate: the V-cycle with a loose
// coarsest solve is not a fixed linear operator.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>

#include "fcg_internal.hpp"
#include "fcg_status.hpp"
#include "fourc_gpu.h"

namespace {

constexpr int kBlock = 256;
constexpr int kParts = 512;  // partial sums per inner product (fixed: run-to-run reproducible)

unsigned blocks_for(int64_t n) { return unsigned(std::max<int64_t>(1, (n + kBlock - 1) / kBlock)); }

__device__ inline double block_sum(double v, double* sbuf)
{
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sbuf[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < int(blockDim.x >> 6); ++i) t += sbuf[i];
  return t;
}

// partial[blockIdx][k] = block's share of a_k . b_k for up to 3 pairs at once
__global__ __launch_bounds__(kBlock) void dots_kernel(const double* __restrict__ a0,
    const double* __restrict__ b0, const double* __restrict__ a1, const double* __restrict__ b1,
    const double* __restrict__ a2, const double* __restrict__ b2, int np, int64_t n, double* partial)
{
  __shared__ double sbuf[kBlock / 64];
  double t[3] = {0.0, 0.0, 0.0};
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
  {
    t[0] += a0[i] * b0[i];
    if (np > 1) t[1] += a1[i] * b1[i];
    if (np > 2) t[2] += a2[i] * b2[i];
  }
  for (int k = 0; k < np; ++k)
  {
    const double v = block_sum(t[k], sbuf);
    if (threadIdx.x == 0) partial[3 * blockIdx.x + k] = v;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void sum_parts_kernel(const double* __restrict__ partial, int nparts,
    int np, double* out)
{
  __shared__ double sbuf[kBlock / 64];
  for (int k = 0; k < np; ++k)
  {
    double t = 0.0;
    for (int i = threadIdx.x; i < nparts; i += kBlock) t += partial[3 * i + k];
    const double v = block_sum(t, sbuf);
    if (threadIdx.x == 0) out[k] = v;
    __syncthreads();
  }
}

// x += alpha p; r_old = r; r -= alpha q
__global__ __launch_bounds__(kBlock) void cg_step_kernel(double alpha, const double* __restrict__ p,
    const double* __restrict__ q, double* x, double* r, double* r_old, int64_t n)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n)
  {
    x[i] += alpha * p[i];
    r_old[i] = r[i];
    r[i] -= alpha * q[i];
  }
}

// y = x + beta y
__global__ __launch_bounds__(kBlock) void xpby_kernel(const double* __restrict__ x, double beta, double* y,
    int64_t n)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) y[i] = x[i] + beta * y[i];
}

struct Fail {
  int code;
  std::string msg;
};

void ck(hipError_t e, const char* what)
{
  if (e != hipSuccess)
  {
    (void)hipGetLastError();
    throw Fail{FCG_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e)};
  }
}
void ck(int rc, const char* what)
{
  if (rc != FCG_OK) throw Fail{rc, what};
}

int rccl_import(void* user, const double* d_x_row, double* d_x_col, void* stream)
{
  auto* p = static_cast<fcg_rccl_pair*>(user);
  return fcg_halo_import(p->halo, p->comm, d_x_row, d_x_col, stream);
}

int rccl_allreduce(void* user, double* d_vals, int64_t n, void* stream)
{
  auto* p = static_cast<fcg_rccl_pair*>(user);
  return fcg_comm_allreduce(p->comm, d_vals, n, FCG_OP_SUM, stream);
}

int rccl_exchange(void* user, const double* d_send, const int64_t* send_counts, double* d_recv,
    const int64_t* recv_counts, void* stream)
{
  auto* p = static_cast<fcg_rccl_pair*>(user);
  return fcg_comm_exchange_device(p->comm, d_send, send_counts, d_recv, recv_counts, stream);
}

}  // namespace

extern "C" {

int fcg_transport_rccl(fcg_rccl_pair* pair, fcg_transport* out)
{
  if (!pair || !out || !pair->comm || !pair->halo) return FCG_ERR_ARG;
  out->import_fn = rccl_import;
  out->allreduce_fn = rccl_allreduce;
  out->exchange_fn = rccl_exchange;
  out->user = pair;
  int n = 1, r = 0;
  if (fcg_comm_size(pair->comm, &n) != FCG_OK || fcg_comm_rank(pair->comm, &r) != FCG_OK) return FCG_ERR_DEVICE;
  out->nranks = n;
  out->rank = r;
  return FCG_OK;
}

int fcg_dfcg_solve(fcg_ctx* ctx, fcg_amg* amg, const fcg_transport* tr, const double* d_K,
    const double* d_b, double* d_x, double rtol, int max_iter, void* stream, int* iterations,
    double* rel_residual)
{
  if (iterations) *iterations = 0;
  if (rel_residual) *rel_residual = 0.0;
  if (!ctx || !tr || !tr->import_fn || !tr->allreduce_fn || !d_K || !d_b || !d_x || !(rtol >= 0.0) ||
      max_iter < 0)
    return FCG_ERR_ARG;
  const fcg::DeviceMesh& m = ctx->mesh;
  if (!m.owned_cols_first)
  {
    ctx->last_error = "fcg_dfcg_solve: the column map must start with the owned DOFs in row order";
    return FCG_ERR_ARG;
  }
  const int64_t n = m.n_rows, nc = m.n_cols;
  if (!fcg_use_device(ctx->device)) return fcg_device_error();
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  double *r = nullptr, *z = nullptr, *p = nullptr, *pc = nullptr, *q = nullptr, *ro = nullptr,
         *dinv = nullptr, *part = nullptr, *sc = nullptr;
  auto release = [&] {
    for (double* v : {r, z, p, pc, q, ro, dinv, part, sc})
      if (v) (void)hipFree(v);
  };
  int it = 0;
  double rel = 0.0;
  try
  {
    auto alloc = [&](double** v, int64_t k) { ck(hipMalloc(v, sizeof(double) * size_t(std::max<int64_t>(1, k))), "hipMalloc"); };
    alloc(&r, n);
    alloc(&z, n);
    alloc(&p, n);
    alloc(&pc, nc);
    alloc(&q, n);
    alloc(&ro, n);
    alloc(&part, 3 * kParts);
    alloc(&sc, 4);
    ck(hipMemsetAsync(pc, 0, sizeof(double) * size_t(std::max<int64_t>(1, nc)), s), "memset");
    // preconditioner: the rank's AMG on its owned block, or the nodal block Jacobi
    if (amg)
    {
      // the return code first: the setup rewrites the handle's error string on failure
      const int rc = fcg_amg_precond_setup(amg, d_K, tr, s);
      if (rc != FCG_OK) throw Fail{rc, fcg_amg_last_error(amg)};
    }
    else
    {
      alloc(&dinv, 9 * (n / 3));
      ck(fcg_block_jacobi_setup(ctx, d_K, dinv, s), "block Jacobi: singular nodal block");
    }
    auto precond = [&](const double* rr, double* zz) {
      if (amg)
      {
        const int rc = fcg_amg_precond_apply(amg, d_K, tr, rr, zz, s);
        if (rc != FCG_OK) throw Fail{rc, fcg_amg_last_error(amg)};
      }
      else
        ck(fcg_block_jacobi_apply(ctx, dinv, rr, zz, 1.0, 0, s), "block Jacobi apply");
    };
    // global inner products: local fixed-order partials, then the transport's all-reduce
    auto dots = [&](int np, const double* a0, const double* b0, const double* a1, const double* b1,
                    const double* a2, const double* b2, double* out) {
      const unsigned g = unsigned(std::min<int64_t>(kParts, blocks_for(n)));
      hipLaunchKernelGGL(dots_kernel, dim3(g), dim3(kBlock), 0, s, a0, b0, a1, b1, a2, b2, np, n, part);
      hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(kBlock), 0, s, part, int(g), np, sc);
      ck(hipGetLastError(), "dot kernels");
      ck(tr->allreduce_fn(tr->user, sc, np, s), "transport all-reduce");
      ck(hipMemcpyAsync(out, sc, sizeof(double) * size_t(np), hipMemcpyDeviceToHost, s), "copy");
      ck(hipStreamSynchronize(s), "hipStreamSynchronize");
    };
    const dim3 g(blocks_for(n)), bl(kBlock);
    ck(hipMemsetAsync(d_x, 0, sizeof(double) * size_t(std::max<int64_t>(1, n)), s), "memset");
    ck(hipMemcpyAsync(r, d_b, sizeof(double) * size_t(n), hipMemcpyDeviceToDevice, s), "copy");
    double h3[3];
    dots(1, d_b, d_b, nullptr, nullptr, nullptr, nullptr, h3);
    const double bn = std::sqrt(h3[0]);
    if (bn > 0.0)
    {
      precond(r, z);
      ck(hipMemcpyAsync(p, z, sizeof(double) * size_t(n), hipMemcpyDeviceToDevice, s), "copy");
      dots(1, r, z, nullptr, nullptr, nullptr, nullptr, h3);
      double rz = h3[0], rn = bn;
      if (!(rz > 0.0)) throw Fail{FCG_ERR_SINGULAR, "fcg_dfcg_solve: indefinite preconditioner (r.z <= 0)"};
      while (it < max_iter)
      {
        ++it;
        ck(tr->import_fn(tr->user, p, pc, s), "transport import");  // set_state of the direction
        ck(fcg_spmv(ctx, d_K, pc, q, s), "fcg_spmv");
        dots(1, p, q, nullptr, nullptr, nullptr, nullptr, h3);
        if (!(h3[0] > 0.0)) throw Fail{FCG_ERR_SINGULAR, "fcg_dfcg_solve: p.Kp <= 0 (K not positive definite)"};
        hipLaunchKernelGGL(cg_step_kernel, g, bl, 0, s, rz / h3[0], p, q, d_x, r, ro, n);
        precond(r, z);
        dots(3, r, r, r, z, z, ro, h3);  // |r|^2, r.z, z.r_old
        rn = std::sqrt(h3[0]);
        if (!std::isfinite(rn)) throw Fail{FCG_ERR_SINGULAR, "fcg_dfcg_solve: non-finite residual"};
        if (rn <= rtol * bn) break;
        if (!(h3[1] > 0.0)) throw Fail{FCG_ERR_SINGULAR, "fcg_dfcg_solve: indefinite preconditioner (r.z <= 0)"};
        const double beta = (h3[1] - h3[2]) / rz;  // Polak-Ribiere (flexible)
        hipLaunchKernelGGL(xpby_kernel, g, bl, 0, s, z, beta, p, n);
        rz = h3[1];
      }
      rel = rn / bn;
    }
  }
  catch (const Fail& f)
  {
    (void)hipStreamSynchronize(s);
    release();
    ctx->last_error = f.msg;
    if (iterations) *iterations = it;
    if (rel_residual) *rel_residual = rel;
    return f.code;
  }
  (void)hipStreamSynchronize(s);
  release();
  if (iterations) *iterations = it;
  if (rel_residual) *rel_residual = rel;
  return FCG_OK;
}

}  // extern "C"
