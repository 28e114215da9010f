// fcg_amg_solver.hip -- the smoothed-aggregation AMG solve as a native C++ object behind the C ABI
// (fcg_amg_create / fcg_amg_solve / fcg_amg_level_info / fcg_amg_destroy): what a C++ host such as
// 4C calls in place of its Belos CG + MueLu preconditioner (4C_solver_nonlin_nox_linearsystem.cpp:
// 275-353, 4C_linear_solver_preconditioner_muelu.cpp) on the tangent a context assembled.  The
// hierarchy and cycle are those of 4c_amd/amg.py (which stays the Python-side mirror and test
// reference): graph setup on the host once (fcg_amg_setup.cpp), numeric setup per tangent and the
// flexible-CG / V-cycle / Chebyshev iteration on the device (fcg_amg.hip kernels, the context's
// fcg_spmv / block-Jacobi on level 0).  Differences from amg.py: the coarsest level is inverted
// densely on the device per tangent (Gauss-Jordan, up to kDenseMax DOFs; above that, or when a
// pivot fails, block-Jacobi CG to a loose tolerance), the scalars of every iteration stay on the
// device except one read per FCG iteration, and with the dense coarsest level one FCG iteration can
// be replayed as a captured HIP graph (FCG_AMG_GRAPH=1).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "fcg_internal.hpp"
#include "fourc_gpu.h"

namespace fcg_amgs {

constexpr int kBlock = 256;
constexpr int kMaxPartials = 1024;
constexpr int64_t kDenseMax = 4096;  // largest coarsest level inverted densely (2 x 134 MB)
inline unsigned blocks_for(int64_t n) { return unsigned((n + kBlock - 1) / kBlock); }
inline unsigned capped(int64_t n) { return unsigned(std::max<int64_t>(1, std::min<int64_t>(kMaxPartials, (n + kBlock - 1) / kBlock))); }

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
  __syncthreads();
  return t;
}

// partial[block] = sum over the block's grid-stride share of a . b (fixed assignment)
__global__ __launch_bounds__(kBlock) void dot_kernel(const double* __restrict__ a,
    const double* __restrict__ b, int64_t n, double* partial)
{
  __shared__ double sbuf[kBlock / 64];
  double t = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
    t += a[i] * b[i];
  const double s = block_sum(t, sbuf);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// out = sum of n partials (one block, fixed order)
__global__ __launch_bounds__(kBlock) void reduce_kernel(const double* __restrict__ partial, int n,
    double* out)
{
  __shared__ double sbuf[kBlock / 64];
  double t = 0.0;
  for (int i = threadIdx.x; i < n; i += kBlock) t += partial[i];
  const double s = block_sum(t, sbuf);
  if (threadIdx.x == 0) *out = s;
}

// y = b - y
__global__ __launch_bounds__(kBlock) void rsub_kernel(const double* __restrict__ b, double* y, int64_t n)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) y[i] = b[i] - y[i];
}

// y = a x + b y
__global__ __launch_bounds__(kBlock) void axpby_kernel(double a, const double* __restrict__ x,
    double b, double* y, int64_t n)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) y[i] = a * x[i] + b * y[i];
}

// FCG step, scalars on the device (sc[0] = r.z, sc[1] = p.q): alpha = r.z / p.q; x += alpha p;
// r_old = r; r -= alpha q
__global__ __launch_bounds__(kBlock) void fcg_step_kernel(const double* __restrict__ sc,
    const double* __restrict__ p, const double* __restrict__ q, double* x, double* r, double* r_old,
    int64_t n)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const double alpha = sc[0] / sc[1];
  x[i] += alpha * p[i];
  r_old[i] = r[i];
  r[i] -= alpha * q[i];
}
// FCG direction (Polak-Ribiere): p = z + beta p, beta = (r.z new - z.r_old) / r.z (sc[2], sc[5], sc[0])
__global__ __launch_bounds__(kBlock) void fcg_dir_kernel(const double* __restrict__ sc,
    const double* __restrict__ z, double* p, int64_t n)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const double beta = (sc[2] - sc[5]) / sc[0];
  p[i] = z[i] + beta * p[i];
}

// ---- the coarsest level as a dense inverse ------------------------------------------------------
// (4C's MueLu coarsest level is a direct solve, Amesos/KLU: 4C_linear_solver_preconditioner_muelu.cpp
// via the xml's "coarse: type"; here the coarsest level has at most coarse_max DOFs, so its inverse
// is formed densely once per tangent and applied as one matrix-vector product per V-cycle)

// D = the 6 x 6 BSR matrix as dense row-major n x n (n = 6 nb; D zeroed before): one thread per
// (block row, block entry)
__global__ __launch_bounds__(kBlock) void bsr6_dense_kernel(int64_t nb, const int64_t* __restrict__ ptr,
    const int32_t* __restrict__ col, const double* __restrict__ vals, double* D)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= nb * 36) return;
  const int64_t i = t / 36;
  const int e = int(t - 36 * i), a = e / 6, b = e % 6;
  const int64_t n = 6 * nb;
  for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
    D[(6 * i + a) * n + 6 * int64_t(col[k]) + b] = vals[36 * k + e];
}

// Block Gauss-Jordan inversion (no pivoting: the coarsest Galerkin operator is symmetric positive
// definite), kGJ pivots per step, A -> B out of place.  With the pivot block P = A[K, K], its row
// panel R = A[K, :] and column panel C = A[:, K]:
//   B[K, K] = P^-1,  B[K, j] = P^-1 R_j,  B[i, K] = -C_i P^-1,  B[i, j] = A_ij - C_i P^-1 R_j;
// after ceil(n / kGJ) steps the buffer holds A^-1.  Step part 1 (gj_panel_kernel): every
// workgroup inverts P in LDS (scalar Gauss-Jordan; a pivot that is not positive sets *bad), then
// W = P^-1 R for its 256 columns and the copy C of the column panel for its 256 rows (both zero
// beyond the last pivot of a short final block); workgroup 0 stores P^-1.  Part 2 (gj_update_kernel)
// forms B.
constexpr int kGJ = 32;

__global__ __launch_bounds__(kBlock) void gj_panel_kernel(const double* __restrict__ A, int64_t n, int64_t k0,
    double* __restrict__ Pinv, double* __restrict__ W, double* __restrict__ C, int32_t* bad)
{
  __shared__ double P[kGJ][kGJ + 1];
  const int t = threadIdx.x;
  const int b = int(min<int64_t>(kGJ, n - k0));
  for (int e = t; e < kGJ * kGJ; e += kBlock)
  {
    const int r = e / kGJ, c = e % kGJ;
    P[r][c] = (r < b && c < b) ? A[(k0 + r) * n + k0 + c] : (r == c ? 1.0 : 0.0);
  }
  __syncthreads();
  for (int m = 0; m < kGJ; ++m)
  {
    const double piv = P[m][m];
    double v[kGJ * kGJ / kBlock];
    const double inv = 1.0 / piv;
#pragma unroll
    for (int u = 0; u < kGJ * kGJ / kBlock; ++u)
    {
      const int e = t + kBlock * u, r = e / kGJ, c = e % kGJ;
      if (r == m) v[u] = c == m ? inv : P[m][c] * inv;
      else if (c == m) v[u] = -P[r][m] * inv;
      else v[u] = P[r][c] - P[r][m] * (P[m][c] * inv);
    }
    if (blockIdx.x == 0 && t == 0 && !(piv > 0.0)) *bad = 1;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kGJ * kGJ / kBlock; ++u)
    {
      const int e = t + kBlock * u;
      P[e / kGJ][e % kGJ] = v[u];
    }
    __syncthreads();
  }
  if (blockIdx.x == 0)
    for (int e = t; e < kGJ * kGJ; e += kBlock) Pinv[e] = P[e / kGJ][e % kGJ];
  const int64_t j = int64_t(blockIdx.x) * kBlock + t;
  if (j >= n) return;
  double w[kGJ];
#pragma unroll
  for (int m = 0; m < kGJ; ++m) w[m] = 0.0;
  for (int q = 0; q < b; ++q)
  {
    const double r = A[(k0 + q) * n + j];
#pragma unroll
    for (int m = 0; m < kGJ; ++m) w[m] += P[m][q] * r;
  }
#pragma unroll
  for (int m = 0; m < kGJ; ++m) W[int64_t(m) * n + j] = w[m];
#pragma unroll
  for (int m = 0; m < kGJ; ++m) C[j * kGJ + m] = m < b ? A[j * n + k0 + m] : 0.0;
}

// grid (ceil(n / kBlock), n): blockIdx.y = row i (its C_i is uniform over the workgroup)
__global__ __launch_bounds__(kBlock) void gj_update_kernel(const double* __restrict__ A, double* __restrict__ B,
    int64_t n, int64_t k0, const double* __restrict__ Pinv, const double* __restrict__ W,
    const double* __restrict__ C)
{
  const int64_t i = blockIdx.y;
  const int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= n) return;
  const int64_t ik = i - k0, jk = j - k0;
  const bool i_in = ik >= 0 && ik < kGJ && i < n, j_in = jk >= 0 && jk < kGJ;
  double v;
  if (i_in)
    v = j_in ? Pinv[ik * kGJ + jk] : W[ik * n + j];
  else
  {
    const double* c = C + i * kGJ;
    double s = 0.0;
    if (j_in)
    {
#pragma unroll
      for (int m = 0; m < kGJ; ++m) s += c[m] * Pinv[m * kGJ + jk];
      v = -s;
    }
    else
    {
#pragma unroll
      for (int m = 0; m < kGJ; ++m) s += c[m] * W[int64_t(m) * n + j];
      v = A[i * n + j] - s;
    }
  }
  B[i * n + j] = v;
}

// y = D x, D dense row-major n x n: one wavefront per row (fixed-order reduction)
__global__ __launch_bounds__(kBlock) void dense_mv_kernel(const double* __restrict__ D,
    const double* __restrict__ x, double* y, int64_t n)
{
  const int64_t row = int64_t(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const double* d = D + row * n;
  double t = 0.0;
  for (int64_t j = lane; j < n; j += 64) t += d[j] * x[j];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
  if (lane == 0) y[row] = t;
}

// coarse CG, scalars on the device: sc[0] = r.z, sc[1] = p.q, sc[2] = r.z new, sc[3] = r.r
__global__ __launch_bounds__(kBlock) void cg_step_kernel(const double* __restrict__ sc,
    const double* __restrict__ p, const double* __restrict__ q, double* x, double* r, int64_t n)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const double alpha = sc[1] > 0.0 ? sc[0] / sc[1] : 0.0;
  x[i] += alpha * p[i];
  r[i] -= alpha * q[i];
}
__global__ __launch_bounds__(kBlock) void cg_dir_kernel(const double* __restrict__ sc,
    const double* __restrict__ z, double* p, int64_t n)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const double beta = sc[0] != 0.0 ? sc[2] / sc[0] : 0.0;
  p[i] = z[i] + beta * p[i];
}
__global__ void shift_kernel(double* sc) { sc[0] = sc[2]; }

// deterministic pseudo-random vector in [-0.5, 0.5) times mask (Lanczos start)
__global__ __launch_bounds__(kBlock) void random_kernel(double* v, const double* __restrict__ mask,
    int64_t n, uint32_t seed)
{
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  uint64_t h = uint64_t(i) * 0x9E3779B97F4A7C15ull + seed;
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  const double u = double(h >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  v[i] = mask ? u * mask[i] : u;
}

// the context's node-triple K into the reordered BSR copy: block m of level-0 row p is triple
// old_k of context row new2old[p] (16 lanes per row, as node_csr_to_bsr_kernel)
__global__ __launch_bounds__(kBlock) void perm_csr_to_bsr_kernel(int64_t n, const int64_t* __restrict__ rowptr,
    const int64_t* __restrict__ b_ptr, const int32_t* __restrict__ new2old, const int32_t* __restrict__ old_k,
    const double* __restrict__ K, double* b_vals)
{
  const int64_t p = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (p >= n) return;
  const int64_t r = new2old[p];
  const int64_t r0 = rowptr[3 * r], r1 = rowptr[3 * r + 1], r2 = rowptr[3 * r + 2];
  for (int64_t q = b_ptr[p] + lane; q < b_ptr[p + 1]; q += 16)
  {
    const int64_t k3 = 3 * int64_t(old_k[q]);
    double* o = b_vals + q * 9;
#pragma unroll
    for (int c = 0; c < 3; ++c)
    {
      o[c] = K[r0 + k3 + c];
      o[3 + c] = K[r1 + k3 + c];
      o[6 + c] = K[r2 + k3 + c];
    }
  }
}

// node triples between the context's order and level 0's: gather dst[3p + d] = src[3 new2old[p] + d]
// (to_ctx = 0) or scatter dst[3 new2old[p] + d] = src[3p + d] (to_ctx = 1)
__global__ __launch_bounds__(kBlock) void node_perm_kernel(int64_t nb, const int32_t* __restrict__ new2old,
    const double* __restrict__ src, double* __restrict__ dst, int to_ctx)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= 3 * nb) return;
  const int64_t p = t / 3, d = t - 3 * p;
  const int64_t o = 3 * int64_t(new2old[p]) + d;
  if (to_ctx) dst[o] = src[t];
  else dst[t] = src[o];
}

struct Bsr {
  int64_t n = 0, nnzb = 0, n_cols = 0;
  int br = 0, bc = 0;
  std::vector<int64_t> ptr_h;
  std::vector<int32_t> col_h;
  int64_t* ptr = nullptr;
  int32_t* col = nullptr;
  double* vals = nullptr;
};

// product plan of one Galerkin SpGEMM (fcg_bsr_product_plan): per C block its (A, B) block pairs
struct Plan {
  int64_t* ptr = nullptr;
  int32_t *a = nullptr, *b = nullptr;
  int64_t* order = nullptr;  // C blocks by (aggregate of the row, row), or NULL
};

struct Step {  // level l -> l + 1
  int bs = 3;
  int64_t n_agg = 0;
  Bsr T, P, AT, AP, Pt;
  Plan pAT, pAP, pC;  // A T, A P, P^T (A P); empty: the searching kernel (FCG_AMG_PLAN=0)
  int32_t* agg = nullptr;
  double* tent = nullptr;   // [n][bs][6], every row's T_i
  int64_t* perm = nullptr;  // P^T block -> P block
};

struct Level {  // coarse level (6 x 6 blocks)
  Bsr A;
  int64_t* diag = nullptr;
  double* dinv = nullptr;
  double lmax = 0.0;
  double *x = nullptr, *b = nullptr, *r = nullptr, *d = nullptr, *z = nullptr, *p = nullptr, *q = nullptr;
};

struct Coupled;

}  // namespace fcg_amgs

struct fcg_amg {
  fcg_ctx* ctx = nullptr;
  int device = 0;
  fcg_amg_options opt{};
  int64_t n0 = 0, nb0 = 0;
  fcg_amgs::Bsr A0;
  int64_t* A0_diag = nullptr;
  double* A0_dinv = nullptr;    // BSR block inverses of level 0 (prolongator smoothing)
  double* ctx_dinv = nullptr;   // the context's block-Jacobi of level 0 (smoother)
  double* mask0 = nullptr;      // 0 on the Dirichlet rows
  double lmax0 = 0.0;
  double *r0 = nullptr, *d0 = nullptr, *z0 = nullptr, *q0 = nullptr, *p0 = nullptr, *ro0 = nullptr,
         *fr = nullptr, *fz = nullptr, *fx = nullptr;
  std::vector<fcg_amgs::Step> steps;
  std::vector<fcg_amgs::Level> levels;  // levels[l] = hierarchy level l + 1
  double* partial = nullptr;  // dot partials
  double* sc = nullptr;       // device scalars
  int32_t* flag = nullptr;
  double* agree = nullptr;    // [2] fcg_amg_precond_setup's go/no-go all-reduce
  std::string last_error;
  std::vector<void*> allocs;
  double setup_ms = 0.0;
  bool ready = false;  // a numeric setup has been made (fcg_amg_setup or the coupled setup)
  // the rank-local hierarchy (lmax0, the Galerkin levels, the coarse inverse) matches the last K:
  // set by fcg_amg_setup, cleared by the coupled numeric setup, which refreshes only the block
  // inverses the coupled V-cycle smooths with -- fcg_amg_apply / fcg_amg_iterate need it
  bool local_ready = false;
  // rank-local preconditioner of a multi-rank context: level 0 is the owned block (ghost column
  // triples dropped) and is applied through its BSR copy instead of the context's fcg_spmv
  bool local = false;
  std::vector<double> ns1;  // level 1's near-null space [n_agg][6][6] (R factors of step 0)
  std::vector<int64_t> full_ptr;  // local: block pattern of the rank's whole rows (column nodes)
  std::vector<int32_t> full_col;
  // the coarse levels coupled across ranks (fcg_dfcg_solve with a local handle): built on the
  // first solve through its transport, see fcg_amgs::Coupled
  fcg_amgs::Coupled* cpl = nullptr;
  // the coarsest level's dense inverse (coarse_solve applies it when set; else block-Jacobi CG):
  // formed per tangent by block Gauss-Jordan between the two buffers when the level has at most
  // kDenseMax DOFs (FCG_AMG_DENSE=0: never)
  double* cbuf[2] = {nullptr, nullptr};
  double* cwork = nullptr;  // the block elimination's pivot inverse and panels
  double* cinv = nullptr;
  int64_t cn = 0;
  // one FCG iteration of fcg_amg_iterate captured as a HIP graph on a private stream (re-captured
  // after every numeric setup and when K or x move), opt-in with FCG_AMG_GRAPH=1: at the 1M-element
  // scale the kernels leave no launch gaps to remove and the replay measured 1-2 % slower.  Only
  // with the dense coarsest inverse: the CG coarse solve reads its residual on the host.
  hipStream_t gs = nullptr;
  hipEvent_t gev[2] = {nullptr, nullptr};
  hipGraphExec_t gexec = nullptr;
  const double* g_K = nullptr;
  double* g_x = nullptr;
  bool graph_off = false;
  int graph_launches = 0;
  // single rank: level 0 renumbered in the Morton order of the node coordinates (a renumbered
  // mesh's input order scatters every row's neighbours over the vectors; FCG_AMG_REORDER=0 keeps
  // the context's order).  Level 0 is then the BSR copy A0 in that order: its SpMV and block
  // Jacobi run on A0, the iteration's vectors are permuted on entry and exit.
  int32_t* new2old = nullptr;  // [nb0] context node of level-0 node p (NULL: no reordering)
  int32_t* old_k = nullptr;    // [A0.nnzb] triple index of each A0 block in its context row
  double *pb = nullptr, *px = nullptr;  // permuted right-hand side / solution
};

namespace fcg_amgs {

struct Fail {
  int code;
  std::string msg;
};

inline void ck(hipError_t e, const char* what)
{
  if (e != hipSuccess)
  {
    (void)hipGetLastError();  // leave no sticky status for the caller (fcg_status.hpp)
    throw Fail{FCG_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e)};
  }
}
inline void ck(int rc, const char* what)
{
  if (rc != FCG_OK) throw Fail{rc, what};
}

template <typename T>
T* dalloc(fcg_amg* h, int64_t n)
{
  void* p = nullptr;
  ck(hipMalloc(&p, sizeof(T) * size_t(std::max<int64_t>(n, 1))), "hipMalloc");
  h->allocs.push_back(p);
  return static_cast<T*>(p);
}
template <typename T>
T* upload(fcg_amg* h, const std::vector<T>& v)
{
  T* d = dalloc<T>(h, int64_t(v.size()));
  if (!v.empty()) ck(hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice), "hipMemcpy");
  return d;
}

void make_bsr(fcg_amg* h, Bsr& M, std::vector<int64_t> ptr, std::vector<int32_t> col, int br, int bc,
    int64_t n_cols)
{
  M.n = int64_t(ptr.size()) - 1;
  M.nnzb = ptr.back();
  M.br = br;
  M.bc = bc;
  M.n_cols = n_cols;
  M.ptr_h = std::move(ptr);
  M.col_h = std::move(col);
  M.ptr = upload(h, M.ptr_h);
  M.col = upload(h, M.col_h);
  M.vals = dalloc<double>(h, M.nnzb * br * bc);
  ck(hipMemset(M.vals, 0, sizeof(double) * size_t(std::max<int64_t>(M.nnzb * br * bc, 1))), "hipMemset");
}

void symbolic(const Bsr& A, const std::vector<int64_t>& bp, const std::vector<int32_t>& bc_,
    int64_t n_cols, std::vector<int64_t>& cp, std::vector<int32_t>& cc)
{
  cp.assign(size_t(A.n) + 1, 0);
  const int64_t nnz = fcg_bsr_symbolic(A.n, A.ptr_h.data(), A.col_h.data(), bp.data(), bc_.data(),
      n_cols, cp.data(), nullptr);
  if (nnz < 0) throw Fail{FCG_ERR_ARG, "AMG: symbolic product failed"};
  cc.assign(size_t(std::max<int64_t>(nnz, 1)), 0);
  if (fcg_bsr_symbolic(A.n, A.ptr_h.data(), A.col_h.data(), bp.data(), bc_.data(), n_cols, cp.data(),
          cc.data()) != nnz)
    throw Fail{FCG_ERR_ARG, "AMG: symbolic fill pass"};
  cc.resize(size_t(nnz));
}

std::vector<int64_t> diag_index(const Bsr& A)
{
  std::vector<int64_t> d(size_t(A.n), -1);
  for (int64_t i = 0; i < A.n; ++i)
    for (int64_t k = A.ptr_h[size_t(i)]; k < A.ptr_h[size_t(i) + 1]; ++k)
      if (A.col_h[size_t(k)] == i) d[size_t(i)] = k;
  for (int64_t v : d)
    if (v < 0) throw Fail{FCG_ERR_ARG, "AMG: block row without a diagonal block"};
  return d;
}

bool env_off(const char* name);

// the pairs of C = X Y on C's pattern, listed on the host and uploaded (the numeric SpGEMM per
// tangent then streams them instead of searching Y's rows for every C block)
Plan make_plan(fcg_amg* h, const Bsr& X, const Bsr& Y, const Bsr& C, const std::vector<int32_t>* agg = nullptr)
{
  Plan pl;
  if (agg)
  {
    // rows of one aggregate are neighbours: forming their blocks together re-reads the Y rows of
    // their shared neighbours from cache (on a renumbered mesh storage order scatters them)
    std::vector<int64_t> rows(size_t(C.n));
    for (int64_t i = 0; i < C.n; ++i) rows[size_t(i)] = i;
    std::stable_sort(rows.begin(), rows.end(), [&](int64_t p, int64_t q) {
      return (*agg)[size_t(p)] < (*agg)[size_t(q)];  // unaggregated rows (-1) first
    });
    std::vector<int64_t> ord;
    ord.reserve(size_t(C.nnzb));
    for (int64_t i : rows)
      for (int64_t ci = C.ptr_h[size_t(i)]; ci < C.ptr_h[size_t(i) + 1]; ++ci) ord.push_back(ci);
    pl.order = upload(h, ord);
  }
  std::vector<int64_t> ptr(size_t(C.nnzb) + 1, 0);
  const int64_t np = fcg_bsr_product_plan(X.n, X.ptr_h.data(), X.col_h.data(), Y.ptr_h.data(),
      Y.col_h.data(), C.ptr_h.data(), C.col_h.data(), C.n_cols, ptr.data(), nullptr, nullptr);
  if (np < 0) throw Fail{FCG_ERR_ARG, "AMG: product plan (count)"};
  std::vector<int32_t> a(size_t(std::max<int64_t>(np, 1))), b(size_t(std::max<int64_t>(np, 1)));
  if (fcg_bsr_product_plan(X.n, X.ptr_h.data(), X.col_h.data(), Y.ptr_h.data(), Y.col_h.data(),
          C.ptr_h.data(), C.col_h.data(), C.n_cols, ptr.data(), a.data(), b.data()) != np)
    throw Fail{FCG_ERR_ARG, "AMG: product plan (fill)"};
  pl.ptr = upload(h, ptr);
  pl.a = upload(h, a);
  pl.b = upload(h, b);
  return pl;
}

// aggregation hierarchy below A_start (block size bs, near-null space ns [n][bs][6]; skip: level-0
// nodes left out of the aggregation, NULL on a coarse start): appends steps and coarse levels until
// a level has at most coarse_max DOFs (and always one step from an empty hierarchy)
void coarsen(fcg_amg* h, const Bsr* A_start, int bs, std::vector<double> ns, const uint8_t* skip)
{
  const Bsr* A = A_start;
  bool first = skip != nullptr;
  while ((A->n * bs > h->opt.coarse_max || h->steps.empty()) && int(h->steps.size()) + 1 < h->opt.max_levels)
  {
    std::vector<int32_t> agg(size_t(A->n));
    const int64_t n_agg = fcg_amg_aggregate(A->n, A->ptr_h.data(), A->col_h.data(), first ? skip : nullptr, agg.data());
    if (n_agg <= 0 || n_agg >= A->n) break;
    std::vector<double> tent(size_t(A->n) * bs * 6), nsc(size_t(n_agg) * 36);
    int64_t nd = 0;
    ck(fcg_amg_tentative(A->n, bs, ns.data(), agg.data(), n_agg, tent.data(), nsc.data(), &nd), "fcg_amg_tentative");
    h->steps.emplace_back();
    Step& st = h->steps.back();
    st.bs = bs;
    st.n_agg = n_agg;
    std::vector<int64_t> tptr(size_t(A->n) + 1, 0);
    std::vector<int32_t> tcol;
    std::vector<double> tvals;
    for (int64_t i = 0; i < A->n; ++i)
    {
      tptr[size_t(i) + 1] = tptr[size_t(i)] + (agg[size_t(i)] >= 0 ? 1 : 0);
      if (agg[size_t(i)] >= 0)
      {
        tcol.push_back(agg[size_t(i)]);
        tvals.insert(tvals.end(), tent.begin() + i * bs * 6, tent.begin() + (i + 1) * bs * 6);
      }
    }
    make_bsr(h, st.T, tptr, tcol, bs, 6, n_agg);
    if (!tvals.empty())
      ck(hipMemcpy(st.T.vals, tvals.data(), sizeof(double) * tvals.size(), hipMemcpyHostToDevice), "hipMemcpy");
    st.agg = upload(h, agg);
    st.tent = upload(h, tent);
    std::vector<int64_t> pp, app, tp, cp;
    std::vector<int32_t> pc, apc, tc, cc;
    symbolic(*A, st.T.ptr_h, st.T.col_h, n_agg, pp, pc);
    make_bsr(h, st.P, pp, pc, bs, 6, n_agg);
    make_bsr(h, st.AT, pp, pc, bs, 6, n_agg);
    symbolic(*A, pp, pc, n_agg, app, apc);
    make_bsr(h, st.AP, app, apc, bs, 6, n_agg);
    tp.assign(size_t(n_agg) + 1, 0);
    tc.assign(size_t(std::max<int64_t>(pp.back(), 1)), 0);
    std::vector<int64_t> perm(size_t(std::max<int64_t>(pp.back(), 1)));
    ck(fcg_bsr_transpose_pattern(A->n, n_agg, pp.data(), pc.data(), tp.data(), tc.data(), perm.data()), "fcg_bsr_transpose_pattern");
    tc.resize(size_t(pp.back()));
    perm.resize(size_t(pp.back()));
    make_bsr(h, st.Pt, tp, tc, 6, bs, A->n);
    st.perm = upload(h, perm);
    symbolic(st.Pt, app, apc, n_agg, cp, cc);
    const bool plans = !env_off("FCG_AMG_PLAN");
    if (plans)  // (before the level list grows: A may point into it)
    {
      const bool by_agg = !env_off("FCG_AMG_PLAN_ORDER");
      st.pAT = make_plan(h, *A, st.T, st.AT, by_agg ? &agg : nullptr);
      st.pAP = make_plan(h, *A, st.P, st.AP, by_agg ? &agg : nullptr);
    }
    h->levels.emplace_back();
    Level& c = h->levels.back();
    make_bsr(h, c.A, cp, cc, 6, 6, n_agg);
    if (plans) st.pC = make_plan(h, st.Pt, st.AP, c.A);
    c.diag = upload(h, diag_index(c.A));
    c.dinv = dalloc<double>(h, 36 * n_agg);
    for (double** v : {&c.x, &c.b, &c.r, &c.d, &c.z, &c.p, &c.q}) *v = dalloc<double>(h, 6 * n_agg);
    if (first) h->ns1 = nsc;  // level 1's near-null space (the coupled coarse level gathers it)
    ns.swap(nsc);
    A = &c.A;
    bs = 6;
    first = false;
  }
}

// ---- device helpers --------------------------------------------------------------------------
double dot_host(fcg_amg* h, const double* a, const double* b, int64_t n, hipStream_t s)
{
  const unsigned g = capped(n);
  hipLaunchKernelGGL(dot_kernel, dim3(g), dim3(kBlock), 0, s, a, b, n, h->partial);
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kBlock), 0, s, h->partial, int(g), h->sc + 6);
  double v = 0.0;
  ck(hipMemcpyAsync(&v, h->sc + 6, sizeof(double), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  ck(hipStreamSynchronize(s), "hipStreamSynchronize");
  return v;
}
void dot_dev(fcg_amg* h, const double* a, const double* b, int64_t n, double* out, hipStream_t s)
{
  const unsigned g = capped(n);
  hipLaunchKernelGGL(dot_kernel, dim3(g), dim3(kBlock), 0, s, a, b, n, h->partial);
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kBlock), 0, s, h->partial, int(g), out);
}

// level 0: the context's SpMV (single rank), or the owned block's BSR copy (local)
void apply_A0(fcg_amg* h, const double* K, const double* x, double* y, hipStream_t s)
{
  if (h->local || h->new2old)
    ck(fcg_bsr_spmv(h->device, 3, 3, h->A0.n, h->A0.ptr, h->A0.col, h->A0.vals, x, y, 1.0, 0, s),
        "fcg_bsr_spmv (level 0)");
  else
    ck(fcg_spmv(h->ctx, K, x, y, s), "fcg_spmv");
}

// a level's operator and smoother pieces: l = 0 the context, l >= 1 levels[l - 1]
void coupled_spmv(fcg_amg* h, const double* K, const fcg_transport* tr, const double* x, double* y, hipStream_t s);
double& coupled_lmax0_ref(fcg_amg* h);
// level 1 distributed across the ranks (struct Dist below)
struct Dist;
int64_t dist_n(const Dist* d);
void dist_spmv(fcg_amg* h, Dist* d, const fcg_transport* tr, const double* x, double* y, hipStream_t s);
void dist_dinv(fcg_amg* h, const Dist* d, const double* r, double* z, double scale, bool acc, hipStream_t s);
double& dist_lmax(Dist* d);
double* dist_vec(Dist* d, int which);  // 0 r, 1 d, 2 z, 3 p, 4 q

struct Ops {
  fcg_amg* h;
  int l;
  const double* K;  // level 0 values
  hipStream_t s;
  // level 0 of a rank-local handle with coupled coarse levels: the global operator (import + the
  // rank's SpMV) and its lambda_max instead of the owned block's
  const fcg_transport* tr = nullptr;
  Dist* dl = nullptr;  // the distributed level 1 (tr: its imports and inner products)
  int64_t n() const { return dl ? dist_n(dl) : l == 0 ? h->n0 : h->levels[size_t(l - 1)].A.n * 6; }
  void spmv(const double* x, double* y) const
  {
    if (dl)
      dist_spmv(h, dl, tr, x, y, s);
    else if (l == 0 && tr)
      coupled_spmv(h, K, tr, x, y, s);
    else if (l == 0)
      apply_A0(h, K, x, y, s);
    else
    {
      const Bsr& A = h->levels[size_t(l - 1)].A;
      ck(fcg_bsr_spmv(h->device, 6, 6, A.n, A.ptr, A.col, A.vals, x, y, 1.0, 0, s), "fcg_bsr_spmv");
    }
  }
  void dinv(const double* r, double* z, double scale, bool acc) const
  {
    if (dl)
      dist_dinv(h, dl, r, z, scale, acc, s);
    else if (l == 0 && h->new2old)  // reordered level 0: its BSR block inverses
      ck(fcg_bsr_block_jacobi_apply(h->device, 3, h->nb0, h->A0_dinv, r, z, scale, acc ? 1 : 0, s),
          "fcg_bsr_block_jacobi_apply (level 0)");
    else if (l == 0)
      ck(fcg_block_jacobi_apply(h->ctx, h->ctx_dinv, r, z, scale, acc ? 1 : 0, s), "fcg_block_jacobi_apply");
    else
    {
      const Level& L = h->levels[size_t(l - 1)];
      ck(fcg_bsr_block_jacobi_apply(h->device, 6, L.A.n, L.dinv, r, z, scale, acc ? 1 : 0, s),
          "fcg_bsr_block_jacobi_apply");
    }
  }
  double& lmax() const
  {
    return dl ? dist_lmax(dl) : l == 0 ? (tr ? coupled_lmax0_ref(h) : h->lmax0) : h->levels[size_t(l - 1)].lmax;
  }
  double* r() const { return dl ? dist_vec(dl, 0) : l == 0 ? h->r0 : h->levels[size_t(l - 1)].r; }
  double* d() const { return dl ? dist_vec(dl, 1) : l == 0 ? h->d0 : h->levels[size_t(l - 1)].d; }
  double* z() const { return dl ? dist_vec(dl, 2) : l == 0 ? h->z0 : h->levels[size_t(l - 1)].z; }
  double* p() const { return dl ? dist_vec(dl, 3) : l == 0 ? h->p0 : h->levels[size_t(l - 1)].p; }
  double* q() const { return dl ? dist_vec(dl, 4) : l == 0 ? h->q0 : h->levels[size_t(l - 1)].q; }
};

// largest eigenvalue of D^-1 A from a 10-step Lanczos (block-Jacobi CG on a random vector); with
// o.tr the operator is the global one and the inner products are summed over the ranks
void estimate_lmax(const Ops& o)
{
  fcg_amg* h = o.h;
  const int64_t n = o.n();
  double *b = o.d(), *r = o.r(), *z = o.z(), *p = o.p(), *q = o.q();
  auto dot_host = [&](fcg_amg* hh, const double* x, const double* y, int64_t nn, hipStream_t ss) {
    if (!o.tr) return fcg_amgs::dot_host(hh, x, y, nn, ss);
    dot_dev(hh, x, y, nn, hh->sc + 6, ss);
    ck(o.tr->allreduce_fn(o.tr->user, hh->sc + 6, 1, ss), "transport all-reduce (Lanczos)");
    double v = 0.0;
    ck(hipMemcpyAsync(&v, hh->sc + 6, sizeof(double), hipMemcpyDeviceToHost, ss), "hipMemcpyAsync");
    ck(hipStreamSynchronize(ss), "hipStreamSynchronize");
    return v;
  };
  hipLaunchKernelGGL(random_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, o.s, b,
      o.l == 0 && !o.dl ? h->mask0 : nullptr, n, 20251015u);
  ck(hipMemcpyAsync(r, b, sizeof(double) * size_t(n), hipMemcpyDeviceToDevice, o.s), "copy");
  o.dinv(r, z, 1.0, false);
  ck(hipMemcpyAsync(p, z, sizeof(double) * size_t(n), hipMemcpyDeviceToDevice, o.s), "copy");
  double rz = dot_host(h, r, z, n, o.s);
  std::vector<double> al, be;
  for (int it = 0; it < 10; ++it)
  {
    o.spmv(p, q);
    const double pq = dot_host(h, p, q, n, o.s);
    if (!(pq > 0.0))
    {
      if (al.empty()) throw Fail{FCG_ERR_SINGULAR, "AMG Lanczos estimate: p.Ap <= 0"};
      break;
    }
    const double alpha = rz / pq;
    hipLaunchKernelGGL(axpby_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, o.s, -alpha, q, 1.0, r, n);
    o.dinv(r, z, 1.0, false);
    const double rzn = dot_host(h, r, z, n, o.s);
    al.push_back(alpha);
    if (!(rzn > 0.0)) break;
    be.push_back(rzn / rz);
    hipLaunchKernelGGL(axpby_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, o.s, 1.0, z, rzn / rz, p, n);
    rz = rzn;
  }
  // largest eigenvalue of the Lanczos tridiagonal (bisection on the Sturm sequence)
  const int k = int(al.size());
  std::vector<double> a(static_cast<size_t>(k)), e(static_cast<size_t>(k), 0.0);
  for (int i = 0; i < k; ++i)
  {
    a[size_t(i)] = 1.0 / al[size_t(i)] + (i > 0 ? be[size_t(i - 1)] / al[size_t(i - 1)] : 0.0);
    if (i + 1 < k) e[size_t(i)] = std::sqrt(be[size_t(i)]) / al[size_t(i)];
  }
  double hi = 0.0;
  for (int i = 0; i < k; ++i)
    hi = std::max(hi, a[size_t(i)] + (i > 0 ? std::fabs(e[size_t(i - 1)]) : 0.0) + (i + 1 < k ? std::fabs(e[size_t(i)]) : 0.0));
  double lo = 0.0;
  auto count_below = [&](double x) {  // eigenvalues < x
    int c = 0;
    double dd = 1.0;
    for (int i = 0; i < k; ++i)
    {
      dd = a[size_t(i)] - x - (i > 0 ? e[size_t(i - 1)] * e[size_t(i - 1)] / dd : 0.0);
      if (dd == 0.0) dd = -1e-300;
      if (dd < 0.0) ++c;
    }
    return c;
  };
  for (int it = 0; it < 200 && hi - lo > 1e-14 * hi; ++it)
  {
    const double mid = 0.5 * (lo + hi);
    if (count_below(mid) >= k) hi = mid;
    else lo = mid;
  }
  o.lmax() = hi;
}

void cheb(const fcg_amg* hc, const Ops& o, const double* b, double* x, bool x_zero)
{
  const fcg_amg_options& op = hc->opt;
  const int64_t n = o.n();
  const double lmax = op.boost * o.lmax();
  const double lmin = lmax / op.ratio;
  const double theta = 0.5 * (lmax + lmin), delta = 0.5 * (lmax - lmin);
  const double sigma = theta / delta;
  double rho = 1.0 / sigma;
  double *r = o.r(), *d = o.d();
  const dim3 g(blocks_for(n)), bl(kBlock);
  if (x_zero)
  {
    o.dinv(b, d, 1.0 / theta, false);
    ck(hipMemcpyAsync(x, d, sizeof(double) * size_t(n), hipMemcpyDeviceToDevice, o.s), "copy");
  }
  else
  {
    o.spmv(x, r);
    hipLaunchKernelGGL(rsub_kernel, g, bl, 0, o.s, b, r, n);
    o.dinv(r, d, 1.0 / theta, false);
    hipLaunchKernelGGL(axpby_kernel, g, bl, 0, o.s, 1.0, d, 1.0, x, n);
  }
  for (int k = 1; k < op.nu; ++k)
  {
    o.spmv(x, r);
    hipLaunchKernelGGL(rsub_kernel, g, bl, 0, o.s, b, r, n);
    const double rho_n = 1.0 / (2.0 * sigma - rho);
    hipLaunchKernelGGL(axpby_kernel, g, bl, 0, o.s, 0.0, d, rho_n * rho, d, n);
    o.dinv(r, d, 2.0 * rho_n / delta, true);
    hipLaunchKernelGGL(axpby_kernel, g, bl, 0, o.s, 1.0, d, 1.0, x, n);
    rho = rho_n;
  }
}

// coarsest level: block-Jacobi CG from x = 0 to |r| <= coarse_rtol |b| (checked every 8 steps;
// scalars on the device in between)
void coarse_solve(fcg_amg* h, const Ops& o, const double* b, double* x)
{
  const int64_t n = o.n();
  if (h->cinv && h->cn == n)
  {
    hipLaunchKernelGGL(dense_mv_kernel, dim3(unsigned((n + kBlock / 64 - 1) / (kBlock / 64))), dim3(kBlock), 0,
        o.s, h->cinv, b, x, n);
    ck(hipGetLastError(), "dense_mv_kernel");
    return;
  }
  double *r = o.r(), *z = o.z(), *p = o.p(), *q = o.q();
  // its own scalars (the outer FCG keeps r.r in sc[3] across the V-cycle): 0 r.z, 1 p.q,
  // 2 r.z new, 3 r.r, 4 b.b
  double* sc = h->sc + 8;
  const dim3 g(blocks_for(n)), bl(kBlock);
  ck(hipMemsetAsync(x, 0, sizeof(double) * size_t(n), o.s), "memset");
  ck(hipMemcpyAsync(r, b, sizeof(double) * size_t(n), hipMemcpyDeviceToDevice, o.s), "copy");
  o.dinv(r, z, 1.0, false);
  ck(hipMemcpyAsync(p, z, sizeof(double) * size_t(n), hipMemcpyDeviceToDevice, o.s), "copy");
  dot_dev(h, r, z, n, sc + 0, o.s);
  dot_dev(h, b, b, n, sc + 4, o.s);
  const double tol2 = h->opt.coarse_rtol * h->opt.coarse_rtol;
  for (int it = 0; it < h->opt.coarse_max_iter;)
  {
    for (int k = 0; k < 8 && it < h->opt.coarse_max_iter; ++k, ++it)
    {
      o.spmv(p, q);
      dot_dev(h, p, q, n, sc + 1, o.s);
      hipLaunchKernelGGL(cg_step_kernel, g, bl, 0, o.s, sc, p, q, x, r, n);
      o.dinv(r, z, 1.0, false);
      dot_dev(h, r, z, n, sc + 2, o.s);
      hipLaunchKernelGGL(cg_dir_kernel, g, bl, 0, o.s, sc, z, p, n);
      hipLaunchKernelGGL(shift_kernel, dim3(1), dim3(1), 0, o.s, sc);
    }
    dot_dev(h, r, r, n, sc + 3, o.s);
    double hs[5];
    ck(hipMemcpyAsync(hs, sc, sizeof(hs), hipMemcpyDeviceToHost, o.s), "hipMemcpyAsync");
    ck(hipStreamSynchronize(o.s), "hipStreamSynchronize");
    if (!std::isfinite(hs[3])) throw Fail{FCG_ERR_SINGULAR, "AMG coarsest CG: non-finite residual"};
    if (hs[3] <= tol2 * hs[4]) break;
  }
}

void vcycle(fcg_amg* h, int l, const double* K, const double* b, double* x, hipStream_t s)
{
  const Ops o{h, l, K, s};
  if (l == int(h->levels.size()))
  {
    coarse_solve(h, o, b, x);
    return;
  }
  cheb(h, o, b, x, true);
  double* r = o.r();
  o.spmv(x, r);
  const int64_t n = o.n();
  hipLaunchKernelGGL(rsub_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, b, r, n);
  const Step& st = h->steps[size_t(l)];
  Level& c = h->levels[size_t(l)];
  ck(fcg_bsr_spmv(h->device, 6, st.bs, st.Pt.n, st.Pt.ptr, st.Pt.col, st.Pt.vals, r, c.b, 1.0, 0, s),
      "restriction");
  vcycle(h, l + 1, K, c.b, c.x, s);
  ck(fcg_bsr_spmv(h->device, st.bs, 6, st.P.n, st.P.ptr, st.P.col, st.P.vals, c.x, x, 1.0, 1, s),
      "prolongation");
  cheb(h, o, b, x, false);
}

void galerkin_from(fcg_amg* h, size_t l0, const double* K, hipStream_t s);
void coarse_factor(fcg_amg* h, hipStream_t s);

// numeric setup for the tangent K (level-0 values in the context's CSR order)
void setup(fcg_amg* h, const double* K, hipStream_t s)
{
  if (h->new2old)
  {
    // the context's nodal blocks first, for their singularity check (4C's block Jacobi throws on a
    // singular block; the BSR setup below completes empty rows with a unit diagonal instead)
    ck(fcg_block_jacobi_setup(h->ctx, K, h->ctx_dinv, s), "singular nodal block of K (block Jacobi)");
    // reordered level 0: the BSR copy in level 0's order, its block inverses (the smoother's too)
    hipLaunchKernelGGL(perm_csr_to_bsr_kernel, dim3(blocks_for(h->nb0 * 16)), dim3(kBlock), 0, s, h->nb0,
        h->ctx->mesh.rowptr, h->A0.ptr, h->new2old, h->old_k, K, h->A0.vals);
    ck(hipGetLastError(), "perm_csr_to_bsr_kernel");
    ck(fcg_bsr_block_jacobi_setup(h->device, 3, h->nb0, h->A0.ptr, h->A0_diag, h->A0.vals, h->A0_dinv,
           h->flag, s),
        "singular nodal block of K");
    estimate_lmax(Ops{h, 0, K, s});
    galerkin_from(h, 0, K, s);
    return;
  }
  ck(fcg_block_jacobi_setup(h->ctx, K, h->ctx_dinv, s), "singular nodal block of K (block Jacobi)");
  // the BSR copy first: the local level 0 applies it in the lambda_max estimate
  ck(fcg_bsr_from_node_csr(h->device, h->nb0, h->ctx->mesh.rowptr, h->A0.ptr, K, h->A0.vals, s),
      "fcg_bsr_from_node_csr");
  estimate_lmax(Ops{h, 0, K, s});
  ck(fcg_bsr_block_jacobi_setup(h->device, 3, h->nb0, h->A0.ptr, h->A0_diag, h->A0.vals, h->A0_dinv,
         h->flag, s),
      "singular nodal block of K");
  galerkin_from(h, 0, K, s);
}

// The numeric setup a rank-local handle needs when its coarse levels are coupled across ranks
// (fcg_amg_precond_setup): the nodal block inverses of the smoother and of P_0's smoothing only --
// the coupled path builds its own lambda_max, P_0, A_1 and hierarchy, so the rank-local Galerkin
// products, their Lanczos estimates and the dense coarsest inverse are skipped
void setup_coupled_local(fcg_amg* h, const double* K, hipStream_t s)
{
  ck(fcg_block_jacobi_setup(h->ctx, K, h->ctx_dinv, s), "singular nodal block of K (block Jacobi)");
  ck(fcg_bsr_from_node_csr(h->device, h->nb0, h->ctx->mesh.rowptr, h->A0.ptr, K, h->A0.vals, s),
      "fcg_bsr_from_node_csr");
  ck(fcg_bsr_block_jacobi_setup(h->device, 3, h->nb0, h->A0.ptr, h->A0_diag, h->A0.vals, h->A0_dinv,
         h->flag, s),
      "singular nodal block of K");
}

// the Galerkin hierarchy below level l0 (its operator and block inverses already set): per step
// l >= l0, P_l = (I - omega D^-1 A_l) T_l and A_{l+1} = P_l^T (A_l P_l) on the fixed patterns
void galerkin_from(fcg_amg* h, size_t l0, const double* K, hipStream_t s)
{
  const Bsr* A = l0 == 0 ? &h->A0 : &h->levels[l0 - 1].A;
  const double* dinv = l0 == 0 ? h->A0_dinv : h->levels[l0 - 1].dinv;
  for (size_t l = l0; l < h->steps.size(); ++l)
  {
    Step& st = h->steps[l];
    const double lm = l == 0 ? h->lmax0 : h->levels[l - 1].lmax;
    auto product = [&](Bsr& C, const Bsr& X, const Bsr& Y, const Plan& pl) {
      if (pl.ptr)
        ck(fcg_bsr_spgemm_planned(h->device, X.br, X.bc, Y.bc, C.nnzb, pl.ptr, pl.a, pl.b, X.vals,
               Y.vals, C.vals, pl.order, s),
            "fcg_bsr_spgemm_planned");
      else
        ck(fcg_bsr_spgemm(h->device, X.br, X.bc, Y.bc, X.n, X.ptr, X.col, X.vals, Y.ptr, Y.col, Y.vals,
               C.ptr, C.col, C.vals, s),
            "fcg_bsr_spgemm");
    };
    product(st.AT, *A, st.T, st.pAT);
    ck(fcg_amg_smooth_prolongator(h->device, st.bs, A->n, st.P.ptr, st.P.col, st.agg, st.tent, dinv,
           st.AT.vals, h->opt.omega / lm, st.P.vals, s),
        "fcg_amg_smooth_prolongator");
    product(st.AP, *A, st.P, st.pAP);
    ck(fcg_bsr_transpose_values(h->device, st.bs, 6, st.P.nnzb, st.perm, st.P.vals, st.Pt.vals, s),
        "fcg_bsr_transpose_values");
    Level& c = h->levels[l];
    product(c.A, st.Pt, st.AP, st.pC);
    ck(fcg_bsr_block_jacobi_setup(h->device, 6, c.A.n, c.A.ptr, c.diag, c.A.vals, c.dinv, h->flag, s),
        "AMG coarse level: singular diagonal block");
    if (l + 1 < h->steps.size()) estimate_lmax(Ops{h, int(l) + 1, K, s});
    A = &c.A;
    dinv = c.dinv;
  }
  coarse_factor(h, s);
}

bool env_off(const char* name)
{
  const char* v = std::getenv(name);
  return v && std::strcmp(v, "0") == 0;
}

// the coarsest level's dense inverse (h->cinv), or none (the CG coarse solve) when the level is
// larger than kDenseMax DOFs, FCG_AMG_DENSE=0 or a pivot is not positive
void coarse_factor(fcg_amg* h, hipStream_t s)
{
  h->cinv = nullptr;
  if (h->levels.empty() || env_off("FCG_AMG_DENSE")) return;
  const Bsr& A = h->levels.back().A;
  const int64_t n = 6 * A.n;
  if (n == 0 || n > kDenseMax) return;
  if (h->cn != n)
  {
    h->cbuf[0] = dalloc<double>(h, n * n);
    h->cbuf[1] = dalloc<double>(h, n * n);
    h->cwork = dalloc<double>(h, 2 * kGJ * n + kGJ * kGJ);
    h->cn = n;
  }
  double *Pinv = h->cwork, *W = Pinv + kGJ * kGJ, *C = W + kGJ * n;
  ck(hipMemsetAsync(h->cbuf[0], 0, sizeof(double) * size_t(n * n), s), "memset");
  ck(hipMemsetAsync(h->flag, 0, sizeof(int32_t), s), "memset");
  hipLaunchKernelGGL(bsr6_dense_kernel, dim3(blocks_for(A.n * 36)), dim3(kBlock), 0, s, A.n, A.ptr, A.col,
      A.vals, h->cbuf[0]);
  const int64_t steps = (n + kGJ - 1) / kGJ;
  for (int64_t t = 0; t < steps; ++t)
  {
    const double* src = h->cbuf[t & 1];
    hipLaunchKernelGGL(gj_panel_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, src, n, t * kGJ, Pinv, W, C,
        h->flag);
    hipLaunchKernelGGL(gj_update_kernel, dim3(blocks_for(n), unsigned(n)), dim3(kBlock), 0, s, src,
        h->cbuf[(t + 1) & 1], n, t * kGJ, Pinv, W, C);
  }
  ck(hipGetLastError(), "gj_update_kernel");
  int32_t bad = 0;
  ck(hipMemcpyAsync(&bad, h->flag, sizeof(bad), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  ck(hipStreamSynchronize(s), "hipStreamSynchronize");
  if (!bad) h->cinv = h->cbuf[steps & 1];
}

// flexible CG (Polak-Ribiere) preconditioned by one V-cycle; one host read per iteration
void run_fcg_ordered(fcg_amg* h, const double* K, const double* b, double* x, double rtol, int max_iter,
    int* iterations, double* rel, hipStream_t s);

// level 0 reordered: the iteration runs on permuted copies of b and x
void run_fcg(fcg_amg* h, const double* K, const double* b, double* x, double rtol, int max_iter,
    int* iterations, double* rel, hipStream_t s)
{
  if (!h->new2old)
  {
    run_fcg_ordered(h, K, b, x, rtol, max_iter, iterations, rel, s);
    return;
  }
  const dim3 g(blocks_for(h->n0)), bl(kBlock);
  hipLaunchKernelGGL(node_perm_kernel, g, bl, 0, s, h->nb0, h->new2old, b, h->pb, 0);
  ck(hipGetLastError(), "node_perm_kernel");
  run_fcg_ordered(h, K, h->pb, h->px, rtol, max_iter, iterations, rel, s);
  hipLaunchKernelGGL(node_perm_kernel, g, bl, 0, s, h->nb0, h->new2old, h->px, x, 1);
  ck(hipGetLastError(), "node_perm_kernel");
}

void run_fcg_ordered(fcg_amg* h, const double* K, const double* b, double* x, double rtol, int max_iter,
    int* iterations, double* rel, hipStream_t s)
{
  const int64_t n = h->n0;
  const dim3 g(blocks_for(n)), bl(kBlock);
  // FCG vectors (the V-cycle's level-0 work vectors r0 / d0 are separate)
  double *r = h->fr, *z = h->fz, *pp = h->fx, *q = h->q0, *ro = h->ro0;
  double* sc = h->sc;
  // device scalars: 0 r.z, 1 p.q, 2 r.z new, 3 r.r, 5 z.r_old
  auto body = [&](hipStream_t q_s) {
    apply_A0(h, K, pp, q, q_s);
    dot_dev(h, pp, q, n, sc + 1, q_s);
    hipLaunchKernelGGL(fcg_step_kernel, g, bl, 0, q_s, sc, pp, q, x, r, ro, n);
    dot_dev(h, r, r, n, sc + 3, q_s);
    vcycle(h, 0, K, r, z, q_s);
    dot_dev(h, r, z, n, sc + 2, q_s);
    dot_dev(h, z, ro, n, sc + 5, q_s);
  };
  // the graph (the iteration body has no host synchronisation once the coarsest solve is dense):
  // its kernel arguments bake in K, x and the setup's lambda_max values
  const char* ge = std::getenv("FCG_AMG_GRAPH");
  const bool use_graph = !h->graph_off && h->cinv && ge && std::strcmp(ge, "1") == 0;
  hipStream_t w = s;
  if (use_graph)
  {
    if (!h->gs)
    {
      ck(hipStreamCreateWithFlags(&h->gs, hipStreamNonBlocking), "hipStreamCreateWithFlags");
      ck(hipEventCreateWithFlags(&h->gev[0], hipEventDisableTiming), "hipEventCreate");
      ck(hipEventCreateWithFlags(&h->gev[1], hipEventDisableTiming), "hipEventCreate");
    }
    ck(hipEventRecord(h->gev[0], s), "hipEventRecord");
    ck(hipStreamWaitEvent(h->gs, h->gev[0], 0), "hipStreamWaitEvent");
    w = h->gs;
    if (h->gexec && (h->g_K != K || h->g_x != x))
    {
      (void)hipGraphExecDestroy(h->gexec);
      h->gexec = nullptr;
    }
  }
  // the caller's stream waits for the private one on every exit
  struct Join {
    fcg_amg* h;
    hipStream_t s, w;
    ~Join()
    {
      if (w != s && hipEventRecord(h->gev[1], w) == hipSuccess) (void)hipStreamWaitEvent(s, h->gev[1], 0);
    }
  } join{h, s, w};
  ck(hipMemsetAsync(x, 0, sizeof(double) * size_t(n), w), "memset");
  const double bn = std::sqrt(dot_host(h, b, b, n, w));
  *iterations = 0;
  *rel = 0.0;
  if (bn == 0.0) return;
  ck(hipMemcpyAsync(r, b, sizeof(double) * size_t(n), hipMemcpyDeviceToDevice, w), "copy");
  vcycle(h, 0, K, r, z, w);
  ck(hipMemcpyAsync(pp, z, sizeof(double) * size_t(n), hipMemcpyDeviceToDevice, w), "copy");
  dot_dev(h, r, z, n, sc + 0, w);
  double rz = 0.0;
  ck(hipMemcpyAsync(&rz, sc, sizeof(double), hipMemcpyDeviceToHost, w), "hipMemcpyAsync");
  ck(hipStreamSynchronize(w), "hipStreamSynchronize");
  if (!(rz > 0.0)) throw Fail{FCG_ERR_SINGULAR, "AMG: indefinite V-cycle (r.z <= 0)"};
  double rn = bn;
  int it = 0;
  while (it < max_iter)
  {
    ++it;
    if (use_graph && !h->gexec && !h->graph_off)
    {
      hipGraph_t graph = nullptr;
      bool ok = hipStreamBeginCapture(w, hipStreamCaptureModeRelaxed) == hipSuccess;
      if (ok)
      {
        try
        {
          body(w);
        }
        catch (const Fail&)
        {
          ok = false;
        }
        ok = hipStreamEndCapture(w, &graph) == hipSuccess && ok && graph;
        ok = ok && hipGraphInstantiate(&h->gexec, graph, nullptr, nullptr, 0) == hipSuccess;
        if (graph) (void)hipGraphDestroy(graph);
      }
      if (!ok)
      {
        (void)hipGetLastError();
        if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
        h->gexec = nullptr;
        h->graph_off = true;  // eager from here on
      }
      h->g_K = K;
      h->g_x = x;
    }
    if (h->gexec)
    {
      ck(hipGraphLaunch(h->gexec, w), "hipGraphLaunch");
      ++h->graph_launches;
    }
    else
      body(w);
    double hs[6];
    ck(hipMemcpyAsync(hs, sc, sizeof(hs), hipMemcpyDeviceToHost, w), "hipMemcpyAsync");
    ck(hipStreamSynchronize(w), "hipStreamSynchronize");
    rn = std::sqrt(hs[3]);
    if (!std::isfinite(rn)) throw Fail{FCG_ERR_SINGULAR, "AMG FCG: non-finite residual"};
    if (rn <= rtol * bn) break;
    if (!(hs[2] > 0.0)) throw Fail{FCG_ERR_SINGULAR, "AMG: indefinite V-cycle (r.z <= 0)"};
    hipLaunchKernelGGL(fcg_dir_kernel, g, bl, 0, w, sc, z, pp, n);
    hipLaunchKernelGGL(shift_kernel, dim3(1), dim3(1), 0, w, sc);
  }
  *iterations = it;
  *rel = rn / bn;
}


// ---- coarse levels coupled across ranks (fcg_dfcg_solve with a rank-local handle) -------------
// 4C's MueLu hierarchy spans every rank (4C_linear_solver_preconditioner_muelu.cpp:97: one
// Xpetra operator over the global matrix).  Here the aggregation stays rank-local (as MueLu's
// uncoupled aggregation), everything else is of the GLOBAL matrix, solved redundantly on every rank
// below level 1:
//   * T_0's rows of the ghost nodes come from their owners through the transport's import (the
//     global aggregate id, then the 3 x 6 block's six columns), so that the prolongator is smoothed
//     with the global operator, P = (I - omega D^-1 A) T_ext, lambda_max of D^-1 A by a Lanczos over
//     the ranks: P's rows near a rank boundary reach the neighbours' aggregates;
//   * P's ghost rows the same way (fixed-width channels per block slot, M the widest row over the
//     ranks), then this rank's part of A_1 = P^T (A_full P_ext) by the block SpGEMM on host-built
//     patterns (A_full: the rank's whole rows, ghost columns included);
//   * the global A_1 pattern is the union of the ranks' parts (their (row, column) pairs gathered
//     once, sorted identically everywhere); per tangent each rank scatters its blocks into a zeroed
//     global buffer and the transport's all-reduce sums them;
//   * a hierarchy built from the gathered A_1 by the same aggregation code (coarsen), replicated and
//     identical on every rank (same input, deterministic build and kernels);
//   * application: one V-cycle of the global system -- Chebyshev on the global operator (each of
//     its SpMVs one import + the rank's rows), the residual restricted into the global level-1
//     vector (all-reduce), the replicated hierarchy, prolongation, Chebyshev again (coupled_apply).
struct DevBuf {
  double* p = nullptr;
  explicit DevBuf(int64_t n) { ck(hipMalloc(&p, sizeof(double) * size_t(std::max<int64_t>(1, n))), "hipMalloc"); }
  ~DevBuf() { if (p) (void)hipFree(p); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
};

// a fixed point-to-point exchange pattern of the distributed level: items per rank in rank
// order (the width of an item is chosen per call)
struct Xch {
  std::vector<int64_t> scnt, rcnt;  // items to / from each rank
  int64_t ns = 0, nr = 0;
  std::vector<int64_t> sd, rd;      // the current call's doubles per rank
  void finish()
  {
    ns = nr = 0;
    for (int64_t v : scnt) ns += v;
    for (int64_t v : rcnt) nr += v;
  }
};

// Level 1 distributed across the ranks (fcg_transport::exchange_fn; MueLu keeps every level of its
// hierarchy a distributed Xpetra operator, 4C_linear_solver_preconditioner_muelu.cpp:97).  Global
// aggregate ids are numbered by rank (rank q owns [agg_off[q], agg_off[q + 1])).  Each rank keeps
//   * LA: the aggregates its P_0 rows and their ghost rows reach, ascending global id (its own at
//     [own0, own0 + na)); P_0, P_0^T, P_ext and this rank's partial A_1 = P^T A P_ext (C) use it;
//   * A: the owned rows of A_1, columns DA = ascending global ids (own at [d0, d0 + na)), summed
//     from C's own rows and the partial rows the other ranks send to the owner (fixed order: own
//     blocks, then the senders in rank order -- bitwise reproducible);
//   * three exchange patterns: the partial rows (36 doubles per block, per numeric setup), the
//     import of A's ghost columns (per level-1 SpMV), and LA's other-rank entries with their owners
//     (restriction: sent and added by the owner; prolongation: the reverse);
//   * level 2: a rank-local aggregation of A's owned block, its tentative prolongator T_1 smoothed
//     with the distributed A_1, P_1 = (I - w D^-1 A_1) T_1,ext (T_1's ghost rows imported once,
//     P_1's per tangent in M1 fixed slots), and A_2 = P_1^T (A_1 P_1,ext) gathered by the all-reduce
//     and solved redundantly by the replicated hierarchy (the replication moves down one level;
//     with T_1 unsmoothed, 32^3 hex27 on 4 ranks took 184 FCG iterations against 130 on one);
//   * or, while level 2 is still past the replication threshold (distribute_level), level 2 is a
//     Dist of its own (next) built the same way from C2, down to the level that is replicated:
//     the replicated bytes then stay bounded by the threshold whatever the rank count.
struct Dist {
  int R = 1, me = 0;
  std::vector<int64_t> agg_off;  // [R + 1]
  int64_t na = 0, off = 0;
  int64_t NL = 0, own0 = 0;
  int64_t NA = 0, d0 = 0;
  Bsr A;
  int64_t* diag = nullptr;
  double* dinv = nullptr;
  double lmax = 0.0;
  int64_t c_lo = 0, c_hi = 0;  // C's owned-row blocks
  int64_t* pos_own = nullptr;  // [c_hi - c_lo] their blocks of A
  Xch rows;
  int64_t* pos_recv = nullptr;  // [rows.nr] A block of each received partial block
  double *rows_s = nullptr, *rows_r = nullptr;
  Xch imp;
  int32_t* imp_idx = nullptr;  // [imp.ns] owned aggregate of each item sent
  std::vector<int32_t> imp_idx_h;
  double *imp_s = nullptr, *imp_r = nullptr, *xe = nullptr;
  Xch pex;
  int32_t* pex_idx = nullptr;  // [pex.nr] owned aggregate of each item received (restriction)
  double *pex_s = nullptr, *pex_r = nullptr, *y = nullptr;
  double *x = nullptr, *b = nullptr, *r = nullptr, *dd = nullptr, *z = nullptr, *p = nullptr, *q = nullptr;
  int64_t n2 = 0, off2 = 0, n2_tot = 0;
  int32_t* agg1 = nullptr;  // [na] global level-2 aggregate of each owned level-1 node (-1 = none)
  double* tent1 = nullptr;  // [na][6][6] T_1's blocks
  Bsr T1ext;  // NA x n2_tot: T_1's rows of A's columns (global level-2 ids)
  Bsr AT1;    // na x n2_tot
  Bsr P1;     // na x n2_tot: (I - w D^-1 A) T_1,ext
  Bsr P1t;    // n2_tot x na
  int64_t* p1_perm = nullptr;
  int M1 = 0;        // blocks per row of P_1, widest over the ranks
  Bsr P1ext;  // NA x n2_tot: P_1's rows of A's columns, the ghost ones imported per tangent
  double *p1_s = nullptr, *p1_r = nullptr;
  Bsr AP1;    // na x n2_tot
  Bsr C2;     // n2_tot x n2_tot: this rank's part of A_2 = P_1^T A P_1,ext
  // the next level distributed in turn (its global size past the replication threshold): the
  // columns of P_1 (and P_1,ext, AP_1, C2's rows and columns, agg1) are then numbered by the next
  // level's LA (its NL entries) instead of the global level-2 ids, and C2 is its partial-rows input
  int level = 1;
  int64_t n2_cols = 0;  // the column space of P_1: n2_tot, or the next level's NL
  Dist* next = nullptr;
  ~Dist() { delete next; }
};

struct Coupled {
  int rank = 0, nranks = 1;
  int64_t nc_nodes = 0;            // column nodes of the context (owned first, then ghosts)
  int64_t off = 0, n_agg_tot = 0;  // this rank's first global aggregate; all ranks' aggregates
  int M = 0;                       // blocks per row of P, widest over the ranks
  Bsr Afull;                       // owned block rows x column nodes (3 x 3)
  Bsr Text;                        // column nodes x aggregates: T_0 rows, ghosts imported
  Bsr AT;                          // owned block rows x aggregates (3 x 6)
  Bsr P;                           // owned block rows x aggregates: (I - w D^-1 A) T
  Bsr Pt;                          // its transpose: aggregates x owned block rows
  int64_t* p_perm = nullptr;       // P^T block -> P block
  int32_t* agg = nullptr;          // [nb0] aggregate of each owned node in P's numbering (-1 = none)
  Bsr Pext;                        // column nodes x aggregates: P rows, ghosts imported
  Bsr AP;                          // owned block rows x aggregates (3 x 6)
  Bsr C;                           // this rank's part of A_1 = P^T A P
  // the replicated level (A_1, or A_2 with a distributed level 1): this rank's blocks and their
  // positions in the replicated operator, which the all-reduce sums
  const Bsr* rep_part = nullptr;
  int64_t* rep_pos = nullptr;      // [rep_part->nnzb] block position in the replicated operator
  int64_t rep_nnzb = 0, rep_n = 0; // replicated operator: blocks, block rows
  double *chan = nullptr, *chan_col = nullptr, *q = nullptr, *w = nullptr, *gb = nullptr, *ge = nullptr;
  fcg_amg* g = nullptr;            // the replicated hierarchy: g->levels[0].A = the replicated operator
  double lmax0 = 0.0;              // lambda_max of D^-1 A for the global operator
  Dist* d = nullptr;               // level 1 distributed (with exchange_fn), else NULL (A_1 replicated)
  // collective traffic (doubles; fcg_amg_coupled_stats): counters of the running phase, and the
  // last numeric setup's and preconditioner application's totals
  int64_t ctr_ar = 0, ctr_x = 0;
  int64_t ar_setup = 0, ar_apply = 0, x_setup = 0, x_apply = 0;
  ~Coupled() { delete d; }
};

double& coupled_lmax0_ref(fcg_amg* h) { return h->cpl->lmax0; }

int64_t dist_n(const Dist* d) { return 6 * d->na; }
double& dist_lmax(Dist* d) { return d->lmax; }
double* dist_vec(Dist* d, int which)
{
  double* v[5] = {d->r, d->dd, d->z, d->p, d->q};
  return v[which];
}

// element-wise sum over the ranks of a host vector, through the transport's device all-reduce
void host_allsum(const fcg_transport* tr, std::vector<double>& v, hipStream_t s)
{
  DevBuf d(int64_t(v.size()));
  if (!v.empty())
    ck(hipMemcpyAsync(d.p, v.data(), sizeof(double) * v.size(), hipMemcpyHostToDevice, s), "hipMemcpyAsync");
  ck(tr->allreduce_fn(tr->user, d.p, int64_t(v.size()), s), "transport all-reduce");
  if (!v.empty())
    ck(hipMemcpyAsync(v.data(), d.p, sizeof(double) * v.size(), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  ck(hipStreamSynchronize(s), "hipStreamSynchronize");
}

// the all-reduce of the coupled levels, counted
void allreduce_counted(Coupled* c, const fcg_transport* tr, double* p, int64_t n, hipStream_t s, const char* what)
{
  ck(tr->allreduce_fn(tr->user, p, n, s), what);
  c->ctr_ar += n;
}

// one exchange of w-double items on pattern x (reverse: the owner -> requester direction), counted
void exchange_counted(Coupled* c, const fcg_transport* tr, Xch& x, int w, bool reverse, const double* sb,
    double* rb, hipStream_t s, const char* what)
{
  const std::vector<int64_t>& sc = reverse ? x.rcnt : x.scnt;
  const std::vector<int64_t>& rc = reverse ? x.scnt : x.rcnt;
  x.sd.assign(sc.size(), 0);
  x.rd.assign(rc.size(), 0);
  for (size_t q = 0; q < sc.size(); ++q)
  {
    x.sd[q] = sc[q] * w;
    x.rd[q] = rc[q] * w;
    c->ctr_x += x.sd[q];
  }
  ck(tr->exchange_fn(tr->user, sb, x.sd.data(), rb, x.rd.data(), s), what);
}

// build-time exchange of host vectors: out[q] goes to rank q (out[me] empty), returns what every
// rank sent to this one (counts first, then the payload, both through exchange_fn)
std::vector<std::vector<double>> host_exchange(const fcg_transport* tr, const std::vector<std::vector<double>>& out,
    hipStream_t s)
{
  const int R = tr->nranks, me = tr->rank;
  std::vector<int64_t> one(static_cast<size_t>(R), 1);
  one[static_cast<size_t>(me)] = 0;
  std::vector<double> cnt_s, cnt_r(static_cast<size_t>(R - 1), 0.0);
  for (int q = 0; q < R; ++q)
    if (q != me) cnt_s.push_back(double(out[static_cast<size_t>(q)].size()));
  DevBuf ds(R), dr(R);
  ck(hipMemcpyAsync(ds.p, cnt_s.data(), sizeof(double) * cnt_s.size(), hipMemcpyHostToDevice, s), "hipMemcpyAsync");
  ck(tr->exchange_fn(tr->user, ds.p, one.data(), dr.p, one.data(), s), "transport exchange (counts)");
  ck(hipMemcpyAsync(cnt_r.data(), dr.p, sizeof(double) * cnt_r.size(), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  ck(hipStreamSynchronize(s), "hipStreamSynchronize");
  std::vector<int64_t> sc(static_cast<size_t>(R), 0), rc(static_cast<size_t>(R), 0);
  std::vector<double> flat;
  for (int q = 0, k = 0; q < R; ++q)
  {
    if (q == me) continue;
    sc[static_cast<size_t>(q)] = int64_t(out[static_cast<size_t>(q)].size());
    rc[static_cast<size_t>(q)] = int64_t(cnt_r[static_cast<size_t>(k++)]);
    flat.insert(flat.end(), out[static_cast<size_t>(q)].begin(), out[static_cast<size_t>(q)].end());
  }
  int64_t nr = 0;
  for (int64_t v : rc) nr += v;
  DevBuf ps(int64_t(flat.size())), pr(nr);
  if (!flat.empty())
    ck(hipMemcpyAsync(ps.p, flat.data(), sizeof(double) * flat.size(), hipMemcpyHostToDevice, s), "hipMemcpyAsync");
  ck(tr->exchange_fn(tr->user, ps.p, sc.data(), pr.p, rc.data(), s), "transport exchange (build)");
  std::vector<double> got(static_cast<size_t>(nr));
  if (nr) ck(hipMemcpyAsync(got.data(), pr.p, sizeof(double) * static_cast<size_t>(nr), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  ck(hipStreamSynchronize(s), "hipStreamSynchronize");
  std::vector<std::vector<double>> in(static_cast<size_t>(R));
  for (int q = 0, o = 0; q < R; ++q)
  {
    in[static_cast<size_t>(q)].assign(got.begin() + o, got.begin() + o + rc[static_cast<size_t>(q)]);
    o += int(rc[static_cast<size_t>(q)]);
  }
  return in;
}

// channel (k, col) of a 3 x 6 BSR's rows as a DOF vector: DOF d of owned node i gets entry
// (d, col) of the row's k-th block (col < 0: the block's global column id -- l2g[col] or col +
// off --, -1 past the row's end)
__global__ __launch_bounds__(kBlock) void pack_channel_kernel(int64_t nb, const int64_t* __restrict__ ptr,
    const int32_t* __restrict__ col, const double* __restrict__ vals, int k, int c, int64_t off,
    double* out)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= 3 * nb) return;
  const int64_t i = t / 3, d = t - 3 * i;
  const int64_t p = ptr[i] + k;
  const bool in = p < ptr[i + 1];
  out[t] = c < 0 ? (in ? double(int64_t(col[p]) + off) : -1.0) : (in ? vals[p * 18 + d * 6 + c] : 0.0);
}

// ... and back into the ghost rows (column nodes nb .. nc-1) of an extended BSR
__global__ __launch_bounds__(kBlock) void scatter_channel_kernel(int64_t nb, int64_t nc,
    const int64_t* __restrict__ ptr, const double* __restrict__ in, int k, int c, double* vals)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  const int64_t i = nb + t / 3, d = t % 3;
  if (i >= nc) return;
  const int64_t p = ptr[i] + k;
  if (p < ptr[i + 1]) vals[p * 18 + d * 6 + c] = in[3 * i + d];
}

// out[pos[k]] = vals[k] (36 doubles per block): this rank's blocks into the replicated operator
__global__ __launch_bounds__(kBlock) void scatter_blocks_kernel(int64_t nnzb, const int64_t* __restrict__ pos,
    const double* __restrict__ vals, double* out)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= nnzb * 36) return;
  const int64_t k = t / 36, q = t - 36 * k;
  out[pos[k] * 36 + q] = vals[t];
}

// out[pos[k]] += vals[k] (36 doubles per block; pos unique within one launch)
__global__ __launch_bounds__(kBlock) void add_blocks_kernel(int64_t nnzb, const int64_t* __restrict__ pos,
    const double* __restrict__ vals, double* out)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= nnzb * 36) return;
  const int64_t k = t / 36, q = t - 36 * k;
  out[pos[k] * 36 + q] += vals[t];
}

// dst[k] = src[idx[k]] (6 doubles per item)
__global__ __launch_bounds__(kBlock) void gather_items_kernel(int64_t n, const int32_t* __restrict__ idx,
    const double* __restrict__ src, double* dst)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= n * 6) return;
  const int64_t k = t / 6, c = t - 6 * k;
  dst[t] = src[int64_t(idx[k]) * 6 + c];
}

// dst[idx[k]] += src[k] (6 doubles per item; idx unique within one launch)
__global__ __launch_bounds__(kBlock) void add_items_kernel(int64_t n, const int32_t* __restrict__ idx,
    const double* __restrict__ src, double* dst)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= n * 6) return;
  const int64_t k = t / 6, c = t - 6 * k;
  dst[int64_t(idx[k]) * 6 + c] += src[t];
}

// M slots of 36 doubles per item: the P_1 row of owned node idx[k] (zeros past the row's end)
__global__ __launch_bounds__(kBlock) void pack_rows_kernel(int64_t n, const int32_t* __restrict__ idx, int M,
    const int64_t* __restrict__ ptr, const double* __restrict__ vals, double* out)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= n * M * 36) return;
  const int64_t k = t / (int64_t(M) * 36), rem = t - k * M * 36, j = rem / 36, e = rem - 36 * j;
  const int64_t l = idx[k], p = ptr[l] + j;
  out[t] = p < ptr[l + 1] ? vals[p * 36 + e] : 0.0;
}

// ... into the ghost rows of an extended BSR (item k = ghost k in column order: row k below d0,
// k + na above)
__global__ __launch_bounds__(kBlock) void unpack_rows_kernel(int64_t n, int64_t d0, int64_t na, int M,
    const int64_t* __restrict__ ptr, const double* __restrict__ in, double* vals)
{
  const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (t >= n * M * 36) return;
  const int64_t k = t / (int64_t(M) * 36), rem = t - k * M * 36, j = rem / 36, e = rem - 36 * j;
  const int64_t row = k < d0 ? k : k + na, p = ptr[row] + j;
  if (p < ptr[row + 1]) vals[p * 36 + e] = in[t];
}

void copy_dd(double* dst, const double* src, int64_t n, hipStream_t s)
{
  if (n > 0) ck(hipMemcpyAsync(dst, src, sizeof(double) * static_cast<size_t>(n), hipMemcpyDeviceToDevice, s), "copy");
}

// the owned rows of a 3 x 6 BSR (global ids) followed by the ghost rows' ids, imported from their
// owners one block slot at a time (M slots); returns the extended pattern in global ids
void extend_pattern(fcg_amg* h, Coupled* c, const Bsr& B, int64_t off, int M, const fcg_transport* tr,
    hipStream_t s, std::vector<int64_t>& pp, std::vector<int32_t>& pc)
{
  const fcg::DeviceMesh& m = h->ctx->mesh;
  const int64_t nb0 = h->nb0, nc = c->nc_nodes;
  std::vector<std::vector<int32_t>> gid(static_cast<size_t>(nc - nb0));
  std::vector<double> colv(static_cast<size_t>(m.n_cols));
  const dim3 gp(blocks_for(3 * std::max<int64_t>(1, nb0))), bl(kBlock);
  for (int k = 0; k < M; ++k)
  {
    hipLaunchKernelGGL(pack_channel_kernel, gp, bl, 0, s, nb0, B.ptr, B.col, B.vals, k, -1, off, c->chan);
    ck(hipGetLastError(), "pack_channel_kernel");
    ck(tr->import_fn(tr->user, c->chan, c->chan_col, s), "transport import (ghost row ids)");
    ck(hipMemcpyAsync(colv.data(), c->chan_col, sizeof(double) * colv.size(), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    ck(hipStreamSynchronize(s), "hipStreamSynchronize");
    for (int64_t i = nb0; i < nc; ++i)
    {
      const double id = colv[static_cast<size_t>(3 * i)];
      if (id >= 0.0) gid[static_cast<size_t>(i - nb0)].push_back(int32_t(id));
    }
  }
  pp.assign(static_cast<size_t>(nc) + 1, 0);
  pc.clear();
  for (int64_t i = 0; i < nb0; ++i)
  {
    for (int64_t k = B.ptr_h[static_cast<size_t>(i)]; k < B.ptr_h[static_cast<size_t>(i) + 1]; ++k) pc.push_back(int32_t(B.col_h[static_cast<size_t>(k)] + off));
    pp[static_cast<size_t>(i) + 1] = int64_t(pc.size());
  }
  for (int64_t i = nb0; i < nc; ++i)
  {
    const auto& row = gid[static_cast<size_t>(i - nb0)];
    for (size_t k = 1; k < row.size(); ++k)
      if (row[k] <= row[k - 1]) throw Fail{FCG_ERR_ARG, "coupled AMG: ghost row not sorted"};
    pc.insert(pc.end(), row.begin(), row.end());
    pp[static_cast<size_t>(i) + 1] = int64_t(pc.size());
  }
}

// the ghost rows' values of an extended BSR (pattern from extend_pattern), 6 channels per slot
void extend_values(fcg_amg* h, Coupled* c, const Bsr& B, Bsr& E, int M, const fcg_transport* tr, hipStream_t s)
{
  const int64_t nb0 = h->nb0, nc = c->nc_nodes;
  if (B.nnzb > 0)
    ck(hipMemcpyAsync(E.vals, B.vals, sizeof(double) * static_cast<size_t>(B.nnzb) * 18, hipMemcpyDeviceToDevice, s), "copy");
  const dim3 gp(blocks_for(3 * std::max<int64_t>(1, nb0))), gg(blocks_for(3 * std::max<int64_t>(1, nc - nb0))),
      bl(kBlock);
  for (int k = 0; k < M; ++k)
    for (int col = 0; col < 6; ++col)
    {
      hipLaunchKernelGGL(pack_channel_kernel, gp, bl, 0, s, nb0, B.ptr, B.col, B.vals, k, col, int64_t(0), c->chan);
      ck(hipGetLastError(), "pack_channel_kernel");
      ck(tr->import_fn(tr->user, c->chan, c->chan_col, s), "transport import (ghost rows)");
      if (nc > nb0)
        hipLaunchKernelGGL(scatter_channel_kernel, gg, bl, 0, s, nb0, nc, E.ptr, c->chan_col, k, col, E.vals);
      ck(hipGetLastError(), "scatter_channel_kernel");
    }
}

int widest_over_ranks(const Bsr& B, int rank, int R, const fcg_transport* tr, hipStream_t s)
{
  std::vector<double> v(static_cast<size_t>(R), 0.0);
  int64_t w = 0;
  for (int64_t i = 0; i < B.n; ++i) w = std::max(w, B.ptr_h[static_cast<size_t>(i) + 1] - B.ptr_h[static_cast<size_t>(i)]);
  v[static_cast<size_t>(rank)] = double(w);
  host_allsum(tr, v, s);
  int M = 0;
  for (double x : v) M = std::max(M, int(x));
  return M;
}

// a BSR whose device arrays hold the pattern only (no values), freed with the object
struct TmpPattern {
  Bsr b;
  TmpPattern(const std::vector<int64_t>& ptr, const std::vector<int32_t>& col)
  {
    b.n = int64_t(ptr.size()) - 1;
    b.nnzb = ptr.back();
    b.ptr_h = ptr;
    b.col_h = col;
    ck(hipMalloc(&b.ptr, sizeof(int64_t) * ptr.size()), "hipMalloc");
    ck(hipMalloc(&b.col, sizeof(int32_t) * std::max<size_t>(1, col.size())), "hipMalloc");
    ck(hipMemcpy(b.ptr, ptr.data(), sizeof(int64_t) * ptr.size(), hipMemcpyHostToDevice), "hipMemcpy");
    if (!col.empty()) ck(hipMemcpy(b.col, col.data(), sizeof(int32_t) * col.size(), hipMemcpyHostToDevice), "hipMemcpy");
  }
  ~TmpPattern()
  {
    if (b.ptr) (void)hipFree(b.ptr);
    if (b.col) (void)hipFree(b.col);
  }
  TmpPattern(const TmpPattern&) = delete;
  TmpPattern& operator=(const TmpPattern&) = delete;
};

// the replicated operator's pattern: the union of every rank's blocks (rows row_off + i of its
// part, global columns), gathered once, sorted and deduplicated identically everywhere; pos =
// each of this rank's blocks in it
void gather_replicated(Coupled* c, const fcg_transport* tr, const std::vector<int64_t>& cp,
    const std::vector<int32_t>& cc, int64_t row_off, int64_t n_tot, hipStream_t s,
    std::vector<int64_t>& gptr, std::vector<int32_t>& gcol, std::vector<int64_t>& pos)
{
  const int64_t R = c->nranks;
  std::vector<int64_t> keys;
  {
    std::vector<double> cnt(static_cast<size_t>(R), 0.0);
    cnt[static_cast<size_t>(c->rank)] = double(cc.size());
    host_allsum(tr, cnt, s);
    int64_t first = 0, total = 0;
    for (int64_t q = 0; q < R; ++q)
    {
      if (q < c->rank) first += int64_t(cnt[static_cast<size_t>(q)]);
      total += int64_t(cnt[static_cast<size_t>(q)]);
    }
    std::vector<double> pairs(static_cast<size_t>(2 * total), 0.0);
    const int64_t nrows = int64_t(cp.size()) - 1;
    for (int64_t i = 0; i < nrows; ++i)
      for (int64_t k = cp[static_cast<size_t>(i)]; k < cp[static_cast<size_t>(i) + 1]; ++k)
      {
        pairs[static_cast<size_t>(2 * (first + k))] = double(row_off + i);
        pairs[static_cast<size_t>(2 * (first + k) + 1)] = double(cc[static_cast<size_t>(k)]);
      }
    host_allsum(tr, pairs, s);
    keys.resize(static_cast<size_t>(total));
    for (int64_t k = 0; k < total; ++k)
      keys[static_cast<size_t>(k)] = int64_t(pairs[static_cast<size_t>(2 * k)]) * n_tot + int64_t(pairs[static_cast<size_t>(2 * k + 1)]);
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  }
  gptr.assign(static_cast<size_t>(n_tot) + 1, 0);
  gcol.assign(keys.size(), 0);
  for (size_t k = 0; k < keys.size(); ++k)
  {
    gptr[static_cast<size_t>(keys[k] / n_tot) + 1] += 1;
    gcol[k] = int32_t(keys[k] % n_tot);
  }
  for (int64_t i = 0; i < n_tot; ++i) gptr[static_cast<size_t>(i) + 1] += gptr[static_cast<size_t>(i)];
  pos.assign(cc.size(), 0);
  const int64_t nrows = int64_t(cp.size()) - 1;
  for (int64_t i = 0; i < nrows; ++i)
    for (int64_t k = cp[static_cast<size_t>(i)]; k < cp[static_cast<size_t>(i) + 1]; ++k)
      pos[static_cast<size_t>(k)] = int64_t(std::lower_bound(keys.begin(), keys.end(), (row_off + i) * n_tot + cc[static_cast<size_t>(k)]) - keys.begin());
}

// the replicated hierarchy below the replicated operator (pattern gptr / gcol, near-null space ns)
void build_replicated(fcg_amg* h, Coupled* c, std::vector<int64_t> gptr, std::vector<int32_t> gcol,
    int64_t n_tot, std::vector<double> ns)
{
  fcg_amg* g = new fcg_amg();
  c->g = g;
  g->ctx = h->ctx;
  g->device = h->device;
  g->opt = h->opt;
  g->steps.emplace_back();  // step 0 (into the replicated level) is the ranks' prolongator
  g->levels.emplace_back();
  {
    Level& L1 = g->levels[0];
    make_bsr(g, L1.A, std::move(gptr), std::move(gcol), 6, 6, n_tot);
    L1.diag = upload(g, diag_index(L1.A));
    L1.dinv = dalloc<double>(g, 36 * n_tot);
    for (double** v : {&L1.x, &L1.b, &L1.r, &L1.d, &L1.z, &L1.p, &L1.q}) *v = dalloc<double>(g, 6 * n_tot);
  }
  c->rep_nnzb = g->levels[0].A.nnzb;
  c->rep_n = n_tot;
  coarsen(g, &g->levels[0].A, 6, std::move(ns), nullptr);
  g->partial = dalloc<double>(g, kMaxPartials);
  g->sc = dalloc<double>(g, 16);
  g->flag = dalloc<int32_t>(g, 1);
  c->gb = dalloc<double>(h, 6 * n_tot);
  c->ge = dalloc<double>(h, 6 * n_tot);
}

// Is coarse level `level` (global size n_agg_tot block rows, at least min_agg_per_rank on every
// rank) distributed across the ranks?  Default: when its global size passes FCG_AMG_DIST_MIN DOFs
// (50000), so that the replicated level below stays under that size whatever the rank count.
// FCG_AMG_DIST=1 forces level 1 (the deeper levels keep the size rule), 0 distributes none;
// FCG_AMG_DIST_LEVELS caps the distributed levels (default 8).  The inputs are the same on every
// rank, so every rank decides alike.
bool distribute_level(const fcg_transport* tr, int level, int64_t n_agg_tot, int64_t min_agg_per_rank)
{
  if (!tr->exchange_fn || min_agg_per_rank < 1) return false;
  const char* e = std::getenv("FCG_AMG_DIST");
  if (e && e[0] == '0') return false;
  const char* lv = std::getenv("FCG_AMG_DIST_LEVELS");
  if (level > (lv ? std::atoi(lv) : 8)) return false;
  if (level == 1 && e && e[0] == '1') return true;
  const char* m = std::getenv("FCG_AMG_DIST_MIN");
  const int64_t min_dofs = m ? std::atoll(m) : 50000;
  return 6 * n_agg_tot > min_dofs;
}

Dist* build_dist(fcg_amg* h, Coupled* c, const fcg_transport* tr, const std::vector<int64_t>& counts,
    const std::vector<int64_t>& LA, const Bsr& C, const std::vector<double>& ns, int level, hipStream_t s);

void coupled_build(fcg_amg* h, const fcg_transport* tr, hipStream_t s)
{
  const fcg::DeviceMesh& m = h->ctx->mesh;
  Coupled* c = new Coupled();
  h->cpl = c;
  c->rank = tr->rank;
  c->nranks = tr->nranks;
  c->nc_nodes = m.n_cols / 3;
  const int64_t nb0 = h->nb0, nc = c->nc_nodes, R = c->nranks;
  const Step& st0 = h->steps[0];
  // aggregates per rank: the global numbering by rank offsets
  std::vector<int64_t> counts(static_cast<size_t>(R), 0);
  int64_t min_agg = 0;
  {
    std::vector<double> v(static_cast<size_t>(R), 0.0);
    v[static_cast<size_t>(c->rank)] = double(st0.n_agg);
    host_allsum(tr, v, s);
    min_agg = int64_t(v[0]);
    for (int64_t q = 0; q < R; ++q)
    {
      counts[static_cast<size_t>(q)] = int64_t(v[static_cast<size_t>(q)]);
      if (q < c->rank) c->off += counts[static_cast<size_t>(q)];
      c->n_agg_tot += counts[static_cast<size_t>(q)];
      min_agg = std::min(min_agg, counts[static_cast<size_t>(q)]);
    }
  }
  const bool dist = distribute_level(tr, 1, c->n_agg_tot, min_agg);
  c->chan = dalloc<double>(h, 3 * nb0);
  c->chan_col = dalloc<double>(h, m.n_cols);
  c->q = dalloc<double>(h, 3 * nb0);
  c->w = dalloc<double>(h, 3 * nb0);
  make_bsr(h, c->Afull, h->full_ptr, h->full_col, 3, 3, nc);
  // T_0 with the ghost rows of its owners (one block per row), then P = (I - w D^-1 A) T_ext on
  // the pattern of A_full T_ext: P's rows reach the neighbour ranks' aggregates (global ids)
  std::vector<int64_t> pp, ap, tp, cp;
  std::vector<int32_t> pc, apc, tc, cc;
  extend_pattern(h, c, st0.T, c->off, widest_over_ranks(st0.T, c->rank, int(R), tr, s), tr, s, pp, pc);
  std::vector<int64_t> LA;  // P's aggregate numbering: global ids (replicated) or LA (distributed)
  int64_t n_p_cols = c->n_agg_tot;
  std::vector<int64_t> pp2;
  std::vector<int32_t> pc2;
  {
    // P's pattern and its ghost rows (global ids)
    symbolic(c->Afull, pp, pc, c->n_agg_tot, ap, apc);
    TmpPattern Pg(ap, apc);
    c->M = widest_over_ranks(Pg.b, c->rank, int(R), tr, s);
    extend_pattern(h, c, Pg.b, 0, c->M, tr, s, pp2, pc2);
  }
  std::vector<int32_t> agg_h(static_cast<size_t>(nb0));
  ck(hipMemcpy(agg_h.data(), st0.agg, sizeof(int32_t) * agg_h.size(), hipMemcpyDeviceToHost), "hipMemcpy");
  if (dist)
  {
    // LA: the aggregates P_ext reaches, ascending (the order of every pattern row is kept)
    LA.assign(pc2.begin(), pc2.end());
    std::sort(LA.begin(), LA.end());
    LA.erase(std::unique(LA.begin(), LA.end()), LA.end());
    auto g2l = [&](int32_t g) {
      const auto it = std::lower_bound(LA.begin(), LA.end(), int64_t(g));
      if (it == LA.end() || *it != g) throw Fail{FCG_ERR_ARG, "coupled AMG: aggregate outside P_ext's columns"};
      return int32_t(it - LA.begin());
    };
    for (auto* v : {&pc, &apc, &pc2})
      for (auto& x : *v) x = g2l(x);
    n_p_cols = int64_t(LA.size());
    const int64_t own0 = int64_t(std::lower_bound(LA.begin(), LA.end(), c->off) - LA.begin());
    for (auto& a : agg_h)
      if (a >= 0) a = int32_t(a + own0);
  }
  else
    for (auto& a : agg_h)
      if (a >= 0) a = int32_t(a + c->off);
  c->agg = upload(h, agg_h);
  make_bsr(h, c->Text, pp, pc, 3, 6, n_p_cols);
  make_bsr(h, c->AT, ap, apc, 3, 6, n_p_cols);
  make_bsr(h, c->P, ap, apc, 3, 6, n_p_cols);
  tp.assign(static_cast<size_t>(n_p_cols) + 1, 0);
  tc.assign(static_cast<size_t>(std::max<int64_t>(ap.back(), 1)), 0);
  std::vector<int64_t> perm(static_cast<size_t>(std::max<int64_t>(ap.back(), 1)));
  ck(fcg_bsr_transpose_pattern(nb0, n_p_cols, ap.data(), apc.data(), tp.data(), tc.data(), perm.data()),
      "fcg_bsr_transpose_pattern");
  tc.resize(static_cast<size_t>(ap.back()));
  perm.resize(static_cast<size_t>(ap.back()));
  make_bsr(h, c->Pt, tp, tc, 6, 3, nb0);
  c->p_perm = upload(h, perm);
  // this rank's part of A_1 = P^T (A P_ext)
  make_bsr(h, c->Pext, pp2, pc2, 3, 6, n_p_cols);
  std::vector<int64_t> app;
  std::vector<int32_t> appc;
  symbolic(c->Afull, c->Pext.ptr_h, c->Pext.col_h, n_p_cols, app, appc);
  make_bsr(h, c->AP, app, appc, 3, 6, n_p_cols);
  symbolic(c->Pt, app, appc, n_p_cols, cp, cc);
  make_bsr(h, c->C, cp, cc, 6, 6, n_p_cols);
  if (dist)
    c->d = build_dist(h, c, tr, counts, LA, c->C, h->ns1, 1, s);
  else
  {
    std::vector<int64_t> gptr, pos;
    std::vector<int32_t> gcol;
    gather_replicated(c, tr, cp, cc, 0, c->n_agg_tot, s, gptr, gcol, pos);
    c->rep_part = &c->C;
    c->rep_pos = upload(h, pos);
    // level 1's near-null space: each aggregate's R factor from its owner
    std::vector<double> ns(static_cast<size_t>(36 * c->n_agg_tot), 0.0);
    std::copy(h->ns1.begin(), h->ns1.end(), ns.begin() + 36 * c->off);
    host_allsum(tr, ns, s);
    build_replicated(h, c, std::move(gptr), std::move(gcol), c->n_agg_tot, std::move(ns));
  }
  // T_0's ghost rows: the tentative prolongator is fixed at create, so they are imported once
  extend_values(h, c, st0.T, c->Text, 1, tr, s);
}

// Coarse level `level` distributed: its owned rows from the partial rows C of the level above (C's
// rows and columns numbered by LA, this level's ids the level above's prolongator reaches, own
// range included), its import plans, and the prolongator to the next level, which is distributed
// in turn (d->next, recursively) or replicated (C2 gathered, the replicated hierarchy built).  ns:
// the near-null space of this rank's nodes of the level (36 doubles each).
Dist* build_dist(fcg_amg* h, Coupled* c, const fcg_transport* tr, const std::vector<int64_t>& counts,
    const std::vector<int64_t>& LA, const Bsr& C, const std::vector<double>& ns, int level, hipStream_t s)
{
  Dist* d = new Dist();
  std::unique_ptr<Dist> guard_d(d);  // freed if the build throws before it is linked
  d->level = level;
  const int R = c->nranks, me = c->rank;
  d->R = R;
  d->me = me;
  d->agg_off.assign(static_cast<size_t>(R) + 1, 0);
  for (int q = 0; q < R; ++q) d->agg_off[static_cast<size_t>(q) + 1] = d->agg_off[static_cast<size_t>(q)] + counts[static_cast<size_t>(q)];
  for (int q = 0; q < me; ++q) d->off += counts[static_cast<size_t>(q)];
  d->na = counts[static_cast<size_t>(me)];
  d->NL = int64_t(LA.size());
  d->own0 = int64_t(std::lower_bound(LA.begin(), LA.end(), d->off) - LA.begin());
  const int64_t na = d->na, own0 = d->own0, off = d->off;
  if (own0 + na > d->NL || LA[static_cast<size_t>(own0)] != off || LA[static_cast<size_t>(own0 + na - 1)] != off + na - 1)
    throw Fail{FCG_ERR_ARG, "coupled AMG: an owned aggregate is missing from P's columns"};
  auto owner = [&](int64_t gid) {
    return int(std::upper_bound(d->agg_off.begin(), d->agg_off.end(), gid) - d->agg_off.begin()) - 1;
  };
  d->c_lo = C.ptr_h[static_cast<size_t>(own0)];
  d->c_hi = C.ptr_h[static_cast<size_t>(own0 + na)];
  // 1. the partial rows of the other ranks' aggregates go to their owners: (row, column) pairs once
  std::vector<std::vector<double>> out(static_cast<size_t>(R));
  d->rows.scnt.assign(static_cast<size_t>(R), 0);
  for (int64_t r = 0; r < d->NL; ++r)
  {
    if (r >= own0 && r < own0 + na) continue;
    const int q = owner(LA[static_cast<size_t>(r)]);
    for (int64_t k = C.ptr_h[static_cast<size_t>(r)]; k < C.ptr_h[static_cast<size_t>(r) + 1]; ++k)
    {
      out[static_cast<size_t>(q)].push_back(double(LA[static_cast<size_t>(r)]));
      out[static_cast<size_t>(q)].push_back(double(LA[static_cast<size_t>(C.col_h[static_cast<size_t>(k)])]));
    }
    d->rows.scnt[static_cast<size_t>(q)] += C.ptr_h[static_cast<size_t>(r) + 1] - C.ptr_h[static_cast<size_t>(r)];
  }
  std::vector<std::vector<double>> in = host_exchange(tr, out, s);
  d->rows.rcnt.assign(static_cast<size_t>(R), 0);
  std::vector<std::vector<int64_t>> rowcols(static_cast<size_t>(na));
  for (int64_t i = 0; i < na; ++i)
  {
    rowcols[static_cast<size_t>(i)].push_back(off + i);  // the diagonal block
    for (int64_t k = C.ptr_h[static_cast<size_t>(own0 + i)]; k < C.ptr_h[static_cast<size_t>(own0 + i) + 1]; ++k)
      rowcols[static_cast<size_t>(i)].push_back(LA[static_cast<size_t>(C.col_h[static_cast<size_t>(k)])]);
  }
  for (int q = 0; q < R; ++q)
  {
    const auto& v = in[static_cast<size_t>(q)];
    d->rows.rcnt[static_cast<size_t>(q)] = int64_t(v.size() / 2);
    for (size_t k = 0; k + 1 < v.size(); k += 2)
    {
      const int64_t rg = int64_t(v[k]);
      if (rg < off || rg >= off + na) throw Fail{FCG_ERR_ARG, "coupled AMG: partial row sent to the wrong rank"};
      rowcols[static_cast<size_t>(rg - off)].push_back(int64_t(v[k + 1]));
    }
  }
  d->rows.finish();
  std::vector<int64_t> DA;
  for (auto& row : rowcols)
  {
    std::sort(row.begin(), row.end());
    row.erase(std::unique(row.begin(), row.end()), row.end());
    DA.insert(DA.end(), row.begin(), row.end());
  }
  std::sort(DA.begin(), DA.end());
  DA.erase(std::unique(DA.begin(), DA.end()), DA.end());
  d->NA = int64_t(DA.size());
  d->d0 = int64_t(std::lower_bound(DA.begin(), DA.end(), off) - DA.begin());
  auto da = [&](int64_t g) { return int32_t(std::lower_bound(DA.begin(), DA.end(), g) - DA.begin()); };
  std::vector<int64_t> aptr(static_cast<size_t>(na) + 1, 0);
  std::vector<int32_t> acol;
  for (int64_t i = 0; i < na; ++i)
  {
    for (int64_t g : rowcols[static_cast<size_t>(i)]) acol.push_back(da(g));
    aptr[static_cast<size_t>(i) + 1] = int64_t(acol.size());
  }
  make_bsr(h, d->A, aptr, acol, 6, 6, d->NA);
  auto block_of = [&](int64_t i, int32_t col) {
    const auto b = acol.begin() + aptr[static_cast<size_t>(i)], e = acol.begin() + aptr[static_cast<size_t>(i) + 1];
    const auto it = std::lower_bound(b, e, col);
    if (it == e || *it != col) throw Fail{FCG_ERR_ARG, "coupled AMG: level-1 block not in the pattern"};
    return int64_t(it - acol.begin());
  };
  {
    std::vector<int64_t> diag(static_cast<size_t>(na)), po(static_cast<size_t>(d->c_hi - d->c_lo)), pr(static_cast<size_t>(d->rows.nr));
    for (int64_t i = 0; i < na; ++i)
    {
      diag[static_cast<size_t>(i)] = block_of(i, int32_t(d->d0 + i));
      for (int64_t k = C.ptr_h[static_cast<size_t>(own0 + i)]; k < C.ptr_h[static_cast<size_t>(own0 + i) + 1]; ++k)
        po[static_cast<size_t>(k - d->c_lo)] = block_of(i, da(LA[static_cast<size_t>(C.col_h[static_cast<size_t>(k)])]));
    }
    int64_t o = 0;
    for (int q = 0; q < R; ++q)
    {
      const auto& v = in[static_cast<size_t>(q)];
      for (size_t k = 0; k + 1 < v.size(); k += 2)
        pr[static_cast<size_t>(o++)] = block_of(int64_t(v[k]) - off, da(int64_t(v[k + 1])));
    }
    d->diag = upload(h, diag);
    d->pos_own = upload(h, po);
    d->pos_recv = upload(h, pr);
  }
  d->dinv = dalloc<double>(h, 36 * na);
  d->rows_s = dalloc<double>(h, 36 * d->rows.ns);
  d->rows_r = dalloc<double>(h, 36 * d->rows.nr);
  // 2. the level-1 import: A's ghost columns (DA outside [d0, d0 + na)) from their owners
  {
    std::vector<std::vector<double>> req(static_cast<size_t>(R));
    d->imp.rcnt.assign(static_cast<size_t>(R), 0);
    for (int64_t j = 0; j < d->NA; ++j)
    {
      if (j >= d->d0 && j < d->d0 + na) continue;
      const int q = owner(DA[static_cast<size_t>(j)]);
      req[static_cast<size_t>(q)].push_back(double(DA[static_cast<size_t>(j)]));
      d->imp.rcnt[static_cast<size_t>(q)] += 1;
    }
    std::vector<std::vector<double>> want = host_exchange(tr, req, s);
    d->imp.scnt.assign(static_cast<size_t>(R), 0);
    std::vector<int32_t> idx;
    for (int q = 0; q < R; ++q)
    {
      d->imp.scnt[static_cast<size_t>(q)] = int64_t(want[static_cast<size_t>(q)].size());
      for (double g : want[static_cast<size_t>(q)])
      {
        const int64_t l = int64_t(g) - off;
        if (l < 0 || l >= na) throw Fail{FCG_ERR_ARG, "coupled AMG: import request for a foreign aggregate"};
        idx.push_back(int32_t(l));
      }
    }
    d->imp.finish();
    d->imp_idx = upload(h, idx);
    d->imp_idx_h = std::move(idx);
    d->imp_s = dalloc<double>(h, 6 * d->imp.ns);
    d->imp_r = dalloc<double>(h, 6 * d->imp.nr);
    d->xe = dalloc<double>(h, 6 * d->NA);
  }
  // 3. restriction / prolongation: LA's other-rank aggregates with their owners
  {
    std::vector<std::vector<double>> req(static_cast<size_t>(R));
    d->pex.scnt.assign(static_cast<size_t>(R), 0);
    for (int64_t r = 0; r < d->NL; ++r)
    {
      if (r >= own0 && r < own0 + na) continue;
      const int q = owner(LA[static_cast<size_t>(r)]);
      req[static_cast<size_t>(q)].push_back(double(LA[static_cast<size_t>(r)]));
      d->pex.scnt[static_cast<size_t>(q)] += 1;
    }
    std::vector<std::vector<double>> got = host_exchange(tr, req, s);
    d->pex.rcnt.assign(static_cast<size_t>(R), 0);
    std::vector<int32_t> idx;
    for (int q = 0; q < R; ++q)
    {
      d->pex.rcnt[static_cast<size_t>(q)] = int64_t(got[static_cast<size_t>(q)].size());
      for (double g : got[static_cast<size_t>(q)])
      {
        const int64_t l = int64_t(g) - off;
        if (l < 0 || l >= na) throw Fail{FCG_ERR_ARG, "coupled AMG: restriction entry for a foreign aggregate"};
        idx.push_back(int32_t(l));
      }
    }
    d->pex.finish();
    d->pex_idx = upload(h, idx);
    d->pex_s = dalloc<double>(h, 6 * d->pex.ns);
    d->pex_r = dalloc<double>(h, 6 * d->pex.nr);
    d->y = dalloc<double>(h, 6 * d->NL);
  }
  for (double** v : {&d->x, &d->b, &d->r, &d->dd, &d->z, &d->p, &d->q}) *v = dalloc<double>(h, 6 * na);
  // 4. level 2: a rank-local aggregation of A's owned block, its tentative prolongator T_1
  std::vector<int32_t> agg1(static_cast<size_t>(na), -1);
  std::vector<double> tent(static_cast<size_t>(na) * 36), ns2;
  {
    std::vector<int64_t> optr(static_cast<size_t>(na) + 1, 0);
    std::vector<int32_t> ocol;
    for (int64_t i = 0; i < na; ++i)
    {
      for (int64_t k = aptr[static_cast<size_t>(i)]; k < aptr[static_cast<size_t>(i) + 1]; ++k)
        if (acol[static_cast<size_t>(k)] >= d->d0 && acol[static_cast<size_t>(k)] < d->d0 + na) ocol.push_back(int32_t(acol[static_cast<size_t>(k)] - d->d0));
      optr[static_cast<size_t>(i) + 1] = int64_t(ocol.size());
    }
    d->n2 = fcg_amg_aggregate(na, optr.data(), ocol.data(), nullptr, agg1.data());
    if (d->n2 <= 0) throw Fail{FCG_ERR_ARG, "coupled AMG: level-1 aggregation failed"};
    ns2.assign(static_cast<size_t>(d->n2) * 36, 0.0);
    int64_t nd = 0;
    if (int64_t(ns.size()) != 36 * na) throw Fail{FCG_ERR_ARG, "coupled AMG: near-null space size"};
    ck(fcg_amg_tentative(na, 6, ns.data(), agg1.data(), d->n2, tent.data(), ns2.data(), &nd),
        "fcg_amg_tentative (distributed level)");
  }
  std::vector<int64_t> counts2(static_cast<size_t>(R), 0);
  int64_t min2 = 0;
  {
    std::vector<double> v(static_cast<size_t>(R), 0.0);
    v[static_cast<size_t>(me)] = double(d->n2);
    host_allsum(tr, v, s);
    min2 = int64_t(v[0]);
    for (int q = 0; q < R; ++q)
    {
      counts2[static_cast<size_t>(q)] = int64_t(v[static_cast<size_t>(q)]);
      if (q < me) d->off2 += counts2[static_cast<size_t>(q)];
      d->n2_tot += counts2[static_cast<size_t>(q)];
      min2 = std::min(min2, counts2[static_cast<size_t>(q)]);
    }
  }
  // the next level distributed too when it is still large (and coarser than this one)
  const int64_t n1_tot = d->agg_off.back();
  const bool next_dist = d->n2_tot < n1_tot && distribute_level(tr, level + 1, d->n2_tot, min2);
  // T_1,ext: A's column rows of T_1 (global level-2 ids), the ghost ones from their owners once
  std::vector<int64_t> eptr(static_cast<size_t>(d->NA) + 1, 0);
  std::vector<int32_t> ecol;
  std::vector<double> ev;
  {
    std::vector<std::vector<double>> rowsout(static_cast<size_t>(R));
    for (int q = 0, o = 0; q < R; ++q)
      for (int64_t k = 0; k < d->imp.scnt[static_cast<size_t>(q)]; ++k)
      {
        const int32_t l = d->imp_idx_h[static_cast<size_t>(o++)];
        const int32_t a = agg1[static_cast<size_t>(l)];
        rowsout[static_cast<size_t>(q)].push_back(a >= 0 ? double(d->off2 + a) : -1.0);
        for (int t = 0; t < 36; ++t) rowsout[static_cast<size_t>(q)].push_back(a >= 0 ? tent[static_cast<size_t>(36 * l + t)] : 0.0);
      }
    std::vector<std::vector<double>> rin = host_exchange(tr, rowsout, s);
    std::vector<double> gh;  // the ghost rows in DA order (ascending global id = rank order)
    for (int q = 0; q < R; ++q) gh.insert(gh.end(), rin[static_cast<size_t>(q)].begin(), rin[static_cast<size_t>(q)].end());
    if (int64_t(gh.size()) != 37 * d->imp.nr) throw Fail{FCG_ERR_ARG, "coupled AMG: T_1 ghost rows incomplete"};
    for (int64_t j = 0, gi = 0; j < d->NA; ++j)
    {
      if (j >= d->d0 && j < d->d0 + na)
      {
        const int64_t l = j - d->d0;
        if (agg1[static_cast<size_t>(l)] >= 0)
        {
          ecol.push_back(int32_t(d->off2 + agg1[static_cast<size_t>(l)]));
          ev.insert(ev.end(), tent.begin() + 36 * l, tent.begin() + 36 * (l + 1));
        }
      }
      else
      {
        const double* row = gh.data() + 37 * gi++;
        if (row[0] >= 0.0)
        {
          ecol.push_back(int32_t(row[0]));
          ev.insert(ev.end(), row + 1, row + 37);
        }
      }
      eptr[static_cast<size_t>(j) + 1] = int64_t(ecol.size());
    }
  }
  // P_1 = (I - w D^-1 A) T_1,ext on the pattern of A T_1,ext (smoothed with the distributed A_1:
  // its rows reach the neighbour ranks' level-2 aggregates), its transpose, and P_1,ext: the ghost
  // rows' patterns from their owners once (M1 column slots per row), their values per tangent
  std::vector<int64_t> a1p, tp, ep, ap1, c2p;
  std::vector<int32_t> a1c, tc, ec, ac1, c2c;
  symbolic(d->A, eptr, ecol, d->n2_tot, a1p, a1c);
  {
    std::vector<double> v(static_cast<size_t>(R), 0.0);
    int64_t w = 0;
    for (int64_t i = 0; i < na; ++i) w = std::max(w, a1p[static_cast<size_t>(i) + 1] - a1p[static_cast<size_t>(i)]);
    v[static_cast<size_t>(me)] = double(w);
    host_allsum(tr, v, s);
    for (double x : v) d->M1 = std::max(d->M1, int(x));
  }
  {
    std::vector<std::vector<double>> rowsout(static_cast<size_t>(R));
    for (int q = 0, o = 0; q < R; ++q)
      for (int64_t k = 0; k < d->imp.scnt[static_cast<size_t>(q)]; ++k)
      {
        const int32_t l = d->imp_idx_h[static_cast<size_t>(o++)];
        const int64_t b0 = a1p[static_cast<size_t>(l)], b1 = a1p[static_cast<size_t>(l) + 1];
        for (int64_t j = 0; j < d->M1; ++j)
          rowsout[static_cast<size_t>(q)].push_back(b0 + j < b1 ? double(a1c[static_cast<size_t>(b0 + j)]) : -1.0);
      }
    std::vector<std::vector<double>> rin = host_exchange(tr, rowsout, s);
    std::vector<double> gh;
    for (int q = 0; q < R; ++q) gh.insert(gh.end(), rin[static_cast<size_t>(q)].begin(), rin[static_cast<size_t>(q)].end());
    if (int64_t(gh.size()) != d->M1 * d->imp.nr) throw Fail{FCG_ERR_ARG, "coupled AMG: P_1 ghost rows incomplete"};
    ep.assign(static_cast<size_t>(d->NA) + 1, 0);
    for (int64_t j = 0, gi = 0; j < d->NA; ++j)
    {
      if (j >= d->d0 && j < d->d0 + na)
      {
        const int64_t l = j - d->d0;
        ec.insert(ec.end(), a1c.begin() + a1p[static_cast<size_t>(l)], a1c.begin() + a1p[static_cast<size_t>(l) + 1]);
      }
      else
      {
        for (int64_t k = 0; k < d->M1; ++k)
        {
          const double col = gh[static_cast<size_t>(d->M1 * gi + k)];
          if (col >= 0.0) ec.push_back(int32_t(col));
        }
        ++gi;
      }
      ep[static_cast<size_t>(j) + 1] = int64_t(ec.size());
    }
  }
  // the column space of P_1: the global level-2 ids (replicated next level), or the next level's
  // LA -- the level-2 ids P_1,ext reaches, ascending (P_1's own rows reach every owned aggregate)
  std::vector<int64_t> LA2;
  d->n2_cols = d->n2_tot;
  std::vector<int32_t> ag(static_cast<size_t>(na));
  for (int64_t i = 0; i < na; ++i)
    ag[static_cast<size_t>(i)] = agg1[static_cast<size_t>(i)] >= 0 ? int32_t(d->off2 + agg1[static_cast<size_t>(i)]) : -1;
  if (next_dist)
  {
    LA2.assign(ec.begin(), ec.end());
    std::sort(LA2.begin(), LA2.end());
    LA2.erase(std::unique(LA2.begin(), LA2.end()), LA2.end());
    auto g2l = [&](int32_t g) {
      const auto it = std::lower_bound(LA2.begin(), LA2.end(), int64_t(g));
      if (it == LA2.end() || *it != g) throw Fail{FCG_ERR_ARG, "coupled AMG: level-2 aggregate outside P_1,ext's columns"};
      return int32_t(it - LA2.begin());
    };
    for (auto* v : {&ecol, &a1c, &ec})
      for (auto& x : *v) x = g2l(x);
    for (auto& x : ag)
      if (x >= 0) x = g2l(x);
    d->n2_cols = int64_t(LA2.size());
  }
  d->agg1 = upload(h, ag);
  d->tent1 = upload(h, tent);
  make_bsr(h, d->T1ext, eptr, ecol, 6, 6, d->n2_cols);
  if (!ev.empty())
    ck(hipMemcpy(d->T1ext.vals, ev.data(), sizeof(double) * ev.size(), hipMemcpyHostToDevice), "hipMemcpy");
  make_bsr(h, d->AT1, a1p, a1c, 6, 6, d->n2_cols);
  make_bsr(h, d->P1, a1p, a1c, 6, 6, d->n2_cols);
  {
    tp.assign(static_cast<size_t>(d->n2_cols) + 1, 0);
    tc.assign(std::max<size_t>(1, a1c.size()), 0);
    std::vector<int64_t> perm(std::max<size_t>(1, a1c.size()));
    ck(fcg_bsr_transpose_pattern(na, d->n2_cols, a1p.data(), a1c.data(), tp.data(), tc.data(), perm.data()),
        "fcg_bsr_transpose_pattern (P_1)");
    tc.resize(a1c.size());
    perm.resize(a1c.size());
    make_bsr(h, d->P1t, tp, tc, 6, 6, na);
    d->p1_perm = upload(h, perm);
  }
  make_bsr(h, d->P1ext, ep, ec, 6, 6, d->n2_cols);
  d->p1_s = dalloc<double>(h, 36 * d->M1 * d->imp.ns);
  d->p1_r = dalloc<double>(h, 36 * d->M1 * d->imp.nr);
  // this rank's part of A_2 = P_1^T (A P_1,ext): rows of every level-2 aggregate its P_1 reaches
  symbolic(d->A, ep, ec, d->n2_cols, ap1, ac1);
  make_bsr(h, d->AP1, ap1, ac1, 6, 6, d->n2_cols);
  symbolic(d->P1t, ap1, ac1, d->n2_cols, c2p, c2c);
  make_bsr(h, d->C2, c2p, c2c, 6, 6, d->n2_cols);
  if (next_dist)
  {
    std::vector<double> ns_next(ns2.begin(), ns2.begin() + 36 * d->n2);
    d->next = build_dist(h, c, tr, counts2, LA2, d->C2, ns_next, level + 1, s);
  }
  else
  {
    std::vector<int64_t> gptr, pos;
    std::vector<int32_t> gcol;
    gather_replicated(c, tr, c2p, c2c, 0, d->n2_tot, s, gptr, gcol, pos);
    c->rep_part = &d->C2;
    c->rep_pos = upload(h, pos);
    std::vector<double> nsg(static_cast<size_t>(36 * d->n2_tot), 0.0);
    std::copy(ns2.begin(), ns2.end(), nsg.begin() + 36 * d->off2);
    host_allsum(tr, nsg, s);
    build_replicated(h, c, std::move(gptr), std::move(gcol), d->n2_tot, std::move(nsg));
  }
  return guard_d.release();
}

// y = A_1 x on the owned rows: x into the extended vector, its ghost entries imported
void dist_spmv(fcg_amg* h, Dist* d, const fcg_transport* tr, const double* x, double* y, hipStream_t s)
{
  Coupled* c = h->cpl;
  copy_dd(d->xe + 6 * d->d0, x, 6 * d->na, s);
  if (d->imp.ns > 0)
    hipLaunchKernelGGL(gather_items_kernel, dim3(blocks_for(6 * d->imp.ns)), dim3(kBlock), 0, s, d->imp.ns,
        d->imp_idx, x, d->imp_s);
  ck(hipGetLastError(), "gather_items_kernel");
  exchange_counted(c, tr, d->imp, 6, false, d->imp_s, d->imp_r, s, "transport exchange (level-1 import)");
  copy_dd(d->xe, d->imp_r, 6 * d->d0, s);
  copy_dd(d->xe + 6 * (d->d0 + d->na), d->imp_r + 6 * d->d0, 6 * (d->NA - d->d0 - d->na), s);
  ck(fcg_bsr_spmv(h->device, 6, 6, d->A.n, d->A.ptr, d->A.col, d->A.vals, d->xe, y, 1.0, 0, s), "fcg_bsr_spmv (level 1)");
}

void dist_dinv(fcg_amg* h, const Dist* d, const double* r, double* z, double scale, bool acc, hipStream_t s)
{
  ck(fcg_bsr_block_jacobi_apply(h->device, 6, d->na, d->dinv, r, z, scale, acc ? 1 : 0, s),
      "fcg_bsr_block_jacobi_apply (level 1)");
}

// numeric: A_1's owned rows from this rank's blocks and the partial rows of the other ranks, its
// block Jacobi and lambda_max, P_1 and this rank's part of A_2
void dist_setup(fcg_amg* h, Dist* d, const Bsr& C, const fcg_transport* tr, hipStream_t s)
{
  Coupled* c = h->cpl;
  ck(hipMemsetAsync(d->A.vals, 0, sizeof(double) * static_cast<size_t>(std::max<int64_t>(1, d->A.nnzb)) * 36, s), "memset");
  if (d->c_hi > d->c_lo)
    hipLaunchKernelGGL(add_blocks_kernel, dim3(blocks_for((d->c_hi - d->c_lo) * 36)), dim3(kBlock), 0, s,
        d->c_hi - d->c_lo, d->pos_own, C.vals + 36 * d->c_lo, d->A.vals);
  ck(hipGetLastError(), "add_blocks_kernel");
  copy_dd(d->rows_s, C.vals, 36 * d->c_lo, s);
  copy_dd(d->rows_s + 36 * d->c_lo, C.vals + 36 * d->c_hi, 36 * (C.nnzb - d->c_hi), s);
  exchange_counted(c, tr, d->rows, 36, false, d->rows_s, d->rows_r, s, "transport exchange (partial level-1 rows)");
  for (int q = 0, o = 0; q < d->R; ++q)
  {
    const int64_t n = d->rows.rcnt[static_cast<size_t>(q)];
    if (n > 0)
      hipLaunchKernelGGL(add_blocks_kernel, dim3(blocks_for(n * 36)), dim3(kBlock), 0, s, n, d->pos_recv + o,
          d->rows_r + 36 * o, d->A.vals);
    o += int(n);
  }
  ck(hipGetLastError(), "add_blocks_kernel");
  ck(fcg_bsr_block_jacobi_setup(h->device, 6, d->na, d->A.ptr, d->diag, d->A.vals, d->dinv, h->flag, s),
      d->level == 1 ? "coupled AMG level 1: singular diagonal block"
                    : "coupled AMG distributed level: singular diagonal block");
  Ops o{h, 1, nullptr, s, tr};
  o.dl = d;
  estimate_lmax(o);
  ck(fcg_bsr_spgemm(h->device, 6, 6, 6, d->A.n, d->A.ptr, d->A.col, d->A.vals, d->T1ext.ptr, d->T1ext.col,
         d->T1ext.vals, d->AT1.ptr, d->AT1.col, d->AT1.vals, s), "fcg_bsr_spgemm (A_1 T_1,ext)");
  ck(fcg_amg_smooth_prolongator(h->device, 6, d->na, d->P1.ptr, d->P1.col, d->agg1, d->tent1, d->dinv,
         d->AT1.vals, h->opt.omega / d->lmax, d->P1.vals, s), "fcg_amg_smooth_prolongator (level 1)");
  if (d->P1.nnzb > 0)
    ck(fcg_bsr_transpose_values(h->device, 6, 6, d->P1.nnzb, d->p1_perm, d->P1.vals, d->P1t.vals, s),
        "fcg_bsr_transpose_values (P_1)");
  copy_dd(d->P1ext.vals + 36 * d->P1ext.ptr_h[static_cast<size_t>(d->d0)], d->P1.vals, 36 * d->P1.nnzb, s);
  const int64_t w = 36 * int64_t(d->M1);
  if (d->imp.ns > 0)
    hipLaunchKernelGGL(pack_rows_kernel, dim3(blocks_for(w * d->imp.ns)), dim3(kBlock), 0, s, d->imp.ns, d->imp_idx,
        d->M1, d->P1.ptr, d->P1.vals, d->p1_s);
  ck(hipGetLastError(), "pack_rows_kernel");
  exchange_counted(c, tr, d->imp, int(w), false, d->p1_s, d->p1_r, s, "transport exchange (P_1 ghost rows)");
  if (d->imp.nr > 0)
    hipLaunchKernelGGL(unpack_rows_kernel, dim3(blocks_for(w * d->imp.nr)), dim3(kBlock), 0, s, d->imp.nr, d->d0,
        d->na, d->M1, d->P1ext.ptr, d->p1_r, d->P1ext.vals);
  ck(hipGetLastError(), "unpack_rows_kernel");
  ck(fcg_bsr_spgemm(h->device, 6, 6, 6, d->A.n, d->A.ptr, d->A.col, d->A.vals, d->P1ext.ptr, d->P1ext.col,
         d->P1ext.vals, d->AP1.ptr, d->AP1.col, d->AP1.vals, s), "fcg_bsr_spgemm (A_1 P_1,ext)");
  ck(fcg_bsr_spgemm(h->device, 6, 6, 6, d->P1t.n, d->P1t.ptr, d->P1t.col, d->P1t.vals, d->AP1.ptr,
         d->AP1.col, d->AP1.vals, d->C2.ptr, d->C2.col, d->C2.vals, s), "fcg_bsr_spgemm (P_1^T A_1 P_1)");
  if (d->next) dist_setup(h, d->next, d->C2, tr, s);
}

void dist_vcycle(fcg_amg* h, const fcg_transport* tr, Dist* d, const double* b, double* x, hipStream_t s);

// y (+)= P A_nd^-1 P^T x through the distributed level nd: the restriction by Pt into nd's LA (rows
// of the level above, bs-wide blocks), whose other-rank entries go to their owners and are added
// there (senders in rank order), nd's V-cycle, the reverse exchange, P back
void dist_coarse(fcg_amg* h, const fcg_transport* tr, Dist* nd, int bs, const Bsr& Pt, const Bsr& P,
    const double* x, double* y, int accumulate, hipStream_t s)
{
  Coupled* c = h->cpl;
  const int64_t na = nd->na, own0 = nd->own0, tail = nd->NL - own0 - na;
  ck(fcg_bsr_spmv(h->device, 6, bs, Pt.n, Pt.ptr, Pt.col, Pt.vals, x, nd->y, 1.0, 0, s), "restriction");
  copy_dd(nd->b, nd->y + 6 * own0, 6 * na, s);
  copy_dd(nd->pex_s, nd->y, 6 * own0, s);
  copy_dd(nd->pex_s + 6 * own0, nd->y + 6 * (own0 + na), 6 * tail, s);
  exchange_counted(c, tr, nd->pex, 6, false, nd->pex_s, nd->pex_r, s, "transport exchange (restriction)");
  for (int q = 0, o = 0; q < nd->R; ++q)
  {
    const int64_t n = nd->pex.rcnt[static_cast<size_t>(q)];
    if (n > 0)
      hipLaunchKernelGGL(add_items_kernel, dim3(blocks_for(6 * n)), dim3(kBlock), 0, s, n, nd->pex_idx + o,
          nd->pex_r + 6 * o, nd->b);
    o += int(n);
  }
  ck(hipGetLastError(), "add_items_kernel");
  dist_vcycle(h, tr, nd, nd->b, nd->x, s);
  if (nd->pex.nr > 0)
    hipLaunchKernelGGL(gather_items_kernel, dim3(blocks_for(6 * nd->pex.nr)), dim3(kBlock), 0, s, nd->pex.nr,
        nd->pex_idx, nd->x, nd->pex_r);
  ck(hipGetLastError(), "gather_items_kernel");
  exchange_counted(c, tr, nd->pex, 6, true, nd->pex_r, nd->pex_s, s, "transport exchange (prolongation)");
  copy_dd(nd->y + 6 * own0, nd->x, 6 * na, s);
  copy_dd(nd->y, nd->pex_s, 6 * own0, s);
  copy_dd(nd->y + 6 * (own0 + na), nd->pex_s + 6 * own0, 6 * tail, s);
  ck(fcg_bsr_spmv(h->device, bs, 6, P.n, P.ptr, P.col, P.vals, nd->y, y, 1.0, accumulate, s), "prolongation");
}

// one V-cycle of a distributed level: Chebyshev with its A, the residual restricted by P_1^T into
// the next level -- distributed in turn (dist_coarse), or replicated (each rank's partial sums,
// completed by the all-reduce, and the replicated hierarchy) -- P_1 back, Chebyshev again
void dist_vcycle(fcg_amg* h, const fcg_transport* tr, Dist* d, const double* b, double* x, hipStream_t s)
{
  Coupled* c = h->cpl;
  Ops o{h, 1, nullptr, s, tr};
  o.dl = d;
  cheb(h, o, b, x, true);
  o.spmv(x, d->r);
  const int64_t n = 6 * d->na;
  hipLaunchKernelGGL(rsub_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, b, d->r, n);
  if (d->next)
    dist_coarse(h, tr, d->next, 6, d->P1t, d->P1, d->r, x, 1, s);
  else
  {
    ck(fcg_bsr_spmv(h->device, 6, 6, d->P1t.n, d->P1t.ptr, d->P1t.col, d->P1t.vals, d->r, c->gb, 1.0, 0, s),
        "restriction (distributed level)");
    allreduce_counted(c, tr, c->gb, 6 * d->n2_tot, s, "transport all-reduce (replicated level)");
    vcycle(c->g, 1, nullptr, c->gb, c->ge, s);
    ck(fcg_bsr_spmv(h->device, 6, 6, d->P1.n, d->P1.ptr, d->P1.col, d->P1.vals, c->ge, x, 1.0, 1, s),
        "prolongation (distributed level)");
  }
  cheb(h, o, b, x, false);
}

// numeric part per tangent, after the local setup (T_0, the nodal block inverses)
void coupled_setup(fcg_amg* h, const double* K, const fcg_transport* tr, hipStream_t s)
{
  Coupled* c = h->cpl;
  c->ctr_ar = c->ctr_x = 0;
  const fcg::DeviceMesh& m = h->ctx->mesh;
  const Step& st0 = h->steps[0];
  const int64_t nb0 = h->nb0;
  ck(fcg_bsr_from_node_csr(h->device, nb0, m.rowptr, c->Afull.ptr, K, c->Afull.vals, s), "fcg_bsr_from_node_csr (full rows)");
  // lambda_max of the global D^-1 A (Lanczos over the ranks): the smoother's and P's
  estimate_lmax(Ops{h, 0, K, s, tr});
  ck(fcg_bsr_spgemm(h->device, 3, 3, 6, nb0, c->Afull.ptr, c->Afull.col, c->Afull.vals, c->Text.ptr,
         c->Text.col, c->Text.vals, c->AT.ptr, c->AT.col, c->AT.vals, s), "fcg_bsr_spgemm (A T_ext)");
  ck(fcg_amg_smooth_prolongator(h->device, 3, nb0, c->P.ptr, c->P.col, c->agg, st0.tent, h->A0_dinv,
         c->AT.vals, h->opt.omega / c->lmax0, c->P.vals, s), "fcg_amg_smooth_prolongator (global)");
  ck(fcg_bsr_transpose_values(h->device, 3, 6, c->P.nnzb, c->p_perm, c->P.vals, c->Pt.vals, s),
      "fcg_bsr_transpose_values");
  extend_values(h, c, c->P, c->Pext, c->M, tr, s);
  ck(fcg_bsr_spgemm(h->device, 3, 3, 6, nb0, c->Afull.ptr, c->Afull.col, c->Afull.vals, c->Pext.ptr,
         c->Pext.col, c->Pext.vals, c->AP.ptr, c->AP.col, c->AP.vals, s), "fcg_bsr_spgemm (A P_ext)");
  ck(fcg_bsr_spgemm(h->device, 6, 3, 6, c->Pt.n, c->Pt.ptr, c->Pt.col, c->Pt.vals, c->AP.ptr, c->AP.col,
         c->AP.vals, c->C.ptr, c->C.col, c->C.vals, s), "fcg_bsr_spgemm (P^T A P)");
  if (c->d) dist_setup(h, c->d, c->C, tr, s);
  // the replicated operator: every rank's blocks scattered into a zeroed buffer, summed
  fcg_amg* g = c->g;
  Level& L1 = g->levels[0];
  ck(hipMemsetAsync(L1.A.vals, 0, sizeof(double) * static_cast<size_t>(std::max<int64_t>(1, c->rep_nnzb)) * 36, s), "memset");
  if (c->rep_part->nnzb > 0)
    hipLaunchKernelGGL(scatter_blocks_kernel, dim3(blocks_for(c->rep_part->nnzb * 36)), dim3(kBlock), 0, s,
        c->rep_part->nnzb, c->rep_pos, c->rep_part->vals, L1.A.vals);
  ck(hipGetLastError(), "scatter_blocks_kernel");
  allreduce_counted(c, tr, L1.A.vals, c->rep_nnzb * 36, s, c->d ? "transport all-reduce (replicated coarse level)" : "transport all-reduce (A_1)");
  ck(fcg_bsr_block_jacobi_setup(g->device, 6, L1.A.n, L1.A.ptr, L1.diag, L1.A.vals, L1.dinv, g->flag, s),
      c->d ? "coupled AMG replicated level: singular diagonal block" : "coupled AMG level 1: singular diagonal block");
  if (g->steps.size() > 1) estimate_lmax(Ops{g, 1, nullptr, s});
  galerkin_from(g, 1, nullptr, s);
  c->ar_setup = c->ctr_ar;
  c->x_setup = c->ctr_x;
}

// Q x = P A_1^-1 P^T x over all ranks.  Replicated level 1: this rank's rows restricted into the
// global level-1 vector (every rank adds to the aggregates its rows reach), the all-reduce, the
// replicated hierarchy's V-cycle, prolongation into this rank's rows (overwrites y).  Distributed
// level 1: the restriction over LA, whose other-rank entries go to their owners and are added
// there (senders in rank order), the level-1 V-cycle, and the reverse exchange before P.
void coupled_coarse(fcg_amg* h, const fcg_transport* tr, const double* x, double* y, hipStream_t s)
{
  Coupled* c = h->cpl;
  Dist* d = c->d;
  if (!d)
  {
    ck(fcg_bsr_spmv(h->device, 6, 3, c->Pt.n, c->Pt.ptr, c->Pt.col, c->Pt.vals, x, c->gb, 1.0, 0, s), "restriction");
    allreduce_counted(c, tr, c->gb, 6 * c->n_agg_tot, s, "transport all-reduce (level 1)");
    vcycle(c->g, 1, nullptr, c->gb, c->ge, s);
    ck(fcg_bsr_spmv(h->device, 3, 6, c->P.n, c->P.ptr, c->P.col, c->P.vals, c->ge, y, 1.0, 0, s), "prolongation");
    return;
  }
  dist_coarse(h, tr, d, 3, c->Pt, c->P, x, y, 0, s);
}

// y = A x with the global operator: the import of x into the column map, the rank's SpMV
void coupled_spmv(fcg_amg* h, const double* K, const fcg_transport* tr, const double* x, double* y, hipStream_t s)
{
  Coupled* c = h->cpl;
  ck(tr->import_fn(tr->user, x, c->chan_col, s), "transport import");
  ck(fcg_spmv(h->ctx, K, c->chan_col, y, s), "fcg_spmv");
}

// One V-cycle of the global system: Chebyshev smoothing with the global operator (D = the owned
// nodal blocks, lambda_max of the global D^-1 A), the residual restricted by this rank's P_0 into
// level 1, the coarse levels there, prolongation, Chebyshev again -- the single-rank cycle, with
// P_0 from the rank-local aggregation.  (Tried before: a multiplicative cycle with rank-local
// smoothing, indefinite; the balancing form Q r + (I - Q A) M (I - A Q) r with M the rank-local
// V-cycle, 64 FCG iterations against 33 on one rank for the 2-rank test box.)
void coupled_apply(fcg_amg* h, const double* K, const fcg_transport* tr, const double* r, double* z,
    hipStream_t s)
{
  Coupled* c = h->cpl;
  c->ctr_ar = c->ctr_x = 0;
  const int64_t n = h->n0;
  const Ops o{h, 0, K, s, tr};
  cheb(h, o, r, z, true);
  coupled_spmv(h, K, tr, z, c->q, s);
  hipLaunchKernelGGL(rsub_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, r, c->q, n);
  coupled_coarse(h, tr, c->q, c->w, s);
  hipLaunchKernelGGL(axpby_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, 1.0, c->w, 1.0, z, n);
  cheb(h, o, r, z, false);
  c->ar_apply = c->ctr_ar;
  c->x_apply = c->ctr_x;
}

// bytes of a hierarchy's matrices (fcg_amg_coupled_stats)
int64_t hierarchy_bytes(const fcg_amg* g)
{
  int64_t b = 0;
  for (const Level& L : g->levels) b += L.A.nnzb * 36 * 8;
  for (const Step& st : g->steps)
    for (const Bsr* M : {&st.T, &st.P, &st.AT, &st.AP, &st.Pt}) b += M->nnzb * M->br * M->bc * 8;
  b += g->cn * g->cn * 8;
  return b;
}

// A transport whose every collective is preceded by a status all-reduce (one double: 0 on a rank
// still going).  The coupled build and numeric setup run over it, so a rank that throws between
// two collectives (a malformed pattern, a singular level-1 block found by dist_setup, a HIP error)
// joins the other ranks at their next collective with its status 1 instead of its payload
// (guard_fail below); every rank then stops there together and returns an error.  The status
// all-reduce is a host round trip per collective of the setup, never of the application.
struct Guard {
  const fcg_transport* in = nullptr;
  fcg_amg* h = nullptr;
  hipStream_t s = nullptr;
  bool remote = false;   // a checkpoint saw another rank's failure (this rank joined it)
  int64_t checkpoints = 0;
  int64_t fail_at = -1;  // test hook: throw on reaching this checkpoint (a failure inside the build)
};

// all-reduced status: true when some rank reported a failure
bool guard_checkpoint(Guard* g, double mine)
{
  if (!g->h->agree) g->h->agree = dalloc<double>(g->h, 2);
  const double v[2] = {mine, 0.0};
  double out[2] = {0.0, 0.0};
  ck(hipMemcpyAsync(g->h->agree, v, sizeof(v), hipMemcpyHostToDevice, g->s), "hipMemcpyAsync");
  ck(g->in->allreduce_fn(g->in->user, g->h->agree, 2, g->s), "transport all-reduce (status)");
  ck(hipMemcpyAsync(out, g->h->agree, sizeof(out), hipMemcpyDeviceToHost, g->s), "hipMemcpyAsync");
  ck(hipStreamSynchronize(g->s), "hipStreamSynchronize");
  ++g->checkpoints;
  return out[0] > 0.0;
}

int guard_enter(Guard* g)
{
  if (g->fail_at >= 0 && g->checkpoints >= g->fail_at)
  {
    g->fail_at = -1;
    throw Fail{FCG_ERR_ARG, "coupled AMG: injected failure inside the build (FCG_AMG_INJECT_BUILD_FAIL)"};
  }
  if (!guard_checkpoint(g, 0.0)) return FCG_OK;
  g->remote = true;
  return FCG_ERR_DEVICE;
}

int guard_allreduce(void* u, double* d, int64_t n, void* s)
{
  Guard* g = static_cast<Guard*>(u);
  const int rc = guard_enter(g);
  return rc != FCG_OK ? rc : g->in->allreduce_fn(g->in->user, d, n, s);
}

int guard_import(void* u, const double* x_row, double* x_col, void* s)
{
  Guard* g = static_cast<Guard*>(u);
  const int rc = guard_enter(g);
  return rc != FCG_OK ? rc : g->in->import_fn(g->in->user, x_row, x_col, s);
}

int guard_exchange(void* u, const double* sb, const int64_t* sc, double* rb, const int64_t* rc_, void* s)
{
  Guard* g = static_cast<Guard*>(u);
  const int rc = guard_enter(g);
  return rc != FCG_OK ? rc : g->in->exchange_fn(g->in->user, sb, sc, rb, rc_, s);
}

fcg_transport guarded(const fcg_transport* tr, Guard* g)
{
  fcg_transport t = *tr;
  t.user = g;
  t.allreduce_fn = guard_allreduce;
  t.import_fn = guard_import;
  t.exchange_fn = tr->exchange_fn ? guard_exchange : nullptr;
  return t;
}

}  // namespace fcg_amgs

extern "C" {

void fcg_amg_default_options(fcg_amg_options* opt)
{
  if (!opt) return;
  opt->nu = 2;
  opt->max_levels = 10;
  opt->coarse_max = 3000;
  opt->coarse_max_iter = 500;
  opt->coarse_rtol = 1e-2;
  opt->omega = 4.0 / 3.0;
  opt->ratio = 20.0;
  opt->boost = 1.1;
}

int fcg_amg_create(fcg_ctx* ctx, const int64_t* rowptr, const int32_t* col_lid,
    const double* node_x, int64_t n_dbc, const int32_t* dbc_rows, const fcg_amg_options* opt,
    fcg_amg** out)
{
  using namespace fcg_amgs;
  if (!ctx || !rowptr || !col_lid || !node_x || !out || n_dbc < 0 || (n_dbc > 0 && !dbc_rows))
    return FCG_ERR_ARG;
  *out = nullptr;
  const fcg::DeviceMesh& m = ctx->mesh;
  if (!m.owned_cols_first || m.n_rows % 3 != 0 || m.n_rows == 0)
  {
    ctx->last_error = "fcg_amg_create: 3 DOFs per owned node (rows 3b..3b+2), owned columns first";
    return FCG_ERR_ARG;
  }
  fcg_amg* h = new fcg_amg();
  h->ctx = ctx;
  h->device = ctx->device;
  h->local = !m.square_local;
  if (opt) h->opt = *opt;
  else fcg_amg_default_options(&h->opt);
  try
  {
    ck(hipSetDevice(h->device), "hipSetDevice");
    const int64_t n = m.n_rows, nb = n / 3;
    h->n0 = n;
    h->nb0 = nb;
    // level 0 block graph: block row b = rows 3b..3b+2 (one pattern of DOF triples)
    // (local: the owned block only -- owned column LIDs are < n and, the columns being sorted,
    // come before every ghost column)
    std::vector<int64_t> bptr(size_t(nb) + 1, 0);
    for (int64_t b = 0; b < nb; ++b)
    {
      const int64_t len = rowptr[3 * b + 1] - rowptr[3 * b];
      if (len % 3 != 0 || rowptr[3 * b + 2] - rowptr[3 * b + 1] != len || rowptr[3 * b + 3] - rowptr[3 * b + 2] != len)
        throw Fail{FCG_ERR_ARG, "fcg_amg_create: rows 3b..3b+2 must share one pattern of DOF triples"};
      int64_t own = 0;
      while (own < len / 3 && col_lid[rowptr[3 * b] + 3 * own] < n) ++own;
      for (int64_t k = own; k < len / 3; ++k)
        if (col_lid[rowptr[3 * b] + 3 * k] < n)
          throw Fail{FCG_ERR_ARG, "fcg_amg_create: row columns must be sorted (owned before ghosts)"};
      bptr[size_t(b) + 1] = bptr[size_t(b)] + own;
    }
    std::vector<int32_t> bcol(size_t(bptr.back()));
    for (int64_t b = 0; b < nb; ++b)
      for (int64_t k = 0; k < bptr[size_t(b) + 1] - bptr[size_t(b)]; ++k)
      {
        const int32_t c = col_lid[rowptr[3 * b] + 3 * k];
        if (c < 0 || c % 3 != 0 || c >= n) throw Fail{FCG_ERR_ARG, "fcg_amg_create: column triples must start at 3 c"};
        bcol[size_t(bptr[size_t(b)] + k)] = c / 3;
      }
    // single rank: level 0 in the Morton order of the node coordinates (21 bits per axis)
    std::vector<int32_t> new2old;
    if (!h->local && !env_off("FCG_AMG_REORDER") && nb > 1)
    {
      double lo[3] = {node_x[0], node_x[1], node_x[2]}, hi[3] = {node_x[0], node_x[1], node_x[2]};
      for (int64_t b = 0; b < nb; ++b)
        for (int d = 0; d < 3; ++d)
        {
          lo[d] = std::min(lo[d], node_x[3 * b + d]);
          hi[d] = std::max(hi[d], node_x[3 * b + d]);
        }
      std::vector<uint64_t> key(static_cast<size_t>(nb));
      for (int64_t b = 0; b < nb; ++b)
      {
        uint64_t m = 0;
        uint32_t q[3];
        for (int d = 0; d < 3; ++d)
        {
          const double ext = hi[d] - lo[d];
          const double f = ext > 0.0 ? (node_x[3 * b + d] - lo[d]) / ext : 0.0;
          q[d] = uint32_t(std::min(2097151.0, std::max(0.0, f * 2097151.0)));
        }
        for (int bit = 20; bit >= 0; --bit)
          for (int d = 0; d < 3; ++d) m = (m << 1) | ((q[d] >> bit) & 1u);
        key[size_t(b)] = m;
      }
      new2old.resize(size_t(nb));
      for (int64_t b = 0; b < nb; ++b) new2old[size_t(b)] = int32_t(b);
      std::stable_sort(new2old.begin(), new2old.end(),
          [&](int32_t a, int32_t c) { return key[size_t(a)] < key[size_t(c)]; });
      std::vector<int32_t> old2new(static_cast<size_t>(nb));
      for (int64_t p = 0; p < nb; ++p) old2new[size_t(new2old[size_t(p)])] = int32_t(p);
      std::vector<int64_t> pptr(size_t(nb) + 1, 0);
      std::vector<int32_t> pcol(bcol.size()), pk(bcol.size());
      std::vector<std::pair<int32_t, int32_t>> row;
      for (int64_t p = 0; p < nb; ++p)
      {
        const int64_t r = new2old[size_t(p)];
        row.clear();
        for (int64_t k = bptr[size_t(r)]; k < bptr[size_t(r) + 1]; ++k)
          row.emplace_back(old2new[size_t(bcol[size_t(k)])], int32_t(k - bptr[size_t(r)]));
        std::sort(row.begin(), row.end());
        pptr[size_t(p) + 1] = pptr[size_t(p)] + int64_t(row.size());
        for (size_t m = 0; m < row.size(); ++m)
        {
          pcol[size_t(pptr[size_t(p)]) + m] = row[m].first;
          pk[size_t(pptr[size_t(p)]) + m] = row[m].second;
        }
      }
      bptr.swap(pptr);
      bcol.swap(pcol);
      h->new2old = upload(h, new2old);
      h->old_k = upload(h, pk);
      h->pb = dalloc<double>(h, n);
      h->px = dalloc<double>(h, n);
    }
    make_bsr(h, h->A0, bptr, bcol, 3, 3, nb);
    if (h->local)
    {
      // the rank's whole rows (ghost column triples included), for the coarse level coupled
      // across ranks (A_1 = P_0^T A P_0 with the global operator): block column = column LID / 3
      if (m.n_cols % 3 != 0) throw Fail{FCG_ERR_ARG, "fcg_amg_create: 3 DOFs per column node"};
      h->full_ptr.assign(size_t(nb) + 1, 0);
      for (int64_t b = 0; b < nb; ++b) h->full_ptr[size_t(b) + 1] = h->full_ptr[size_t(b)] + (rowptr[3 * b + 1] - rowptr[3 * b]) / 3;
      h->full_col.resize(size_t(h->full_ptr.back()));
      for (int64_t b = 0; b < nb; ++b)
        for (int64_t k = 0; k < h->full_ptr[size_t(b) + 1] - h->full_ptr[size_t(b)]; ++k)
        {
          const int32_t c = col_lid[rowptr[3 * b] + 3 * k];
          if (c < 0 || c % 3 != 0 || c >= m.n_cols)
            throw Fail{FCG_ERR_ARG, "fcg_amg_create: column triples must start at 3 c"};
          h->full_col[size_t(h->full_ptr[size_t(b)] + k)] = c / 3;
        }
    }
    h->A0_diag = upload(h, diag_index(h->A0));
    h->A0_dinv = dalloc<double>(h, 9 * nb);
    h->ctx_dinv = dalloc<double>(h, 9 * nb);
    std::vector<uint8_t> dbc(size_t(n), 0);
    for (int64_t k = 0; k < n_dbc; ++k)
    {
      if (dbc_rows[k] < 0 || dbc_rows[k] >= n) throw Fail{FCG_ERR_ARG, "fcg_amg_create: Dirichlet row out of range"};
      dbc[size_t(dbc_rows[k])] = 1;
    }
    // level 0's order (identity without reordering)
    std::vector<double> xl;
    const double* X0 = node_x;
    if (!new2old.empty())
    {
      std::vector<uint8_t> dp(static_cast<size_t>(n));
      xl.resize(size_t(3 * nb));
      for (int64_t p = 0; p < nb; ++p)
        for (int d = 0; d < 3; ++d)
        {
          dp[size_t(3 * p + d)] = dbc[size_t(3 * int64_t(new2old[size_t(p)]) + d)];
          xl[size_t(3 * p + d)] = node_x[3 * int64_t(new2old[size_t(p)]) + d];
        }
      dbc.swap(dp);
      X0 = xl.data();
    }
    std::vector<double> mask(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) mask[size_t(i)] = dbc[size_t(i)] ? 0.0 : 1.0;
    h->mask0 = upload(h, mask);
    // near-null space: rigid-body modes about the centroid, Dirichlet rows zeroed
    double cen[3] = {0, 0, 0};
    for (int64_t b = 0; b < nb; ++b)
      for (int d = 0; d < 3; ++d) cen[d] += X0[3 * b + d] / double(nb);
    std::vector<double> ns(size_t(nb) * 18, 0.0);
    std::vector<uint8_t> skip(size_t(nb), 0);
    for (int64_t b = 0; b < nb; ++b)
    {
      const double x = X0[3 * b] - cen[0], y = X0[3 * b + 1] - cen[1], z = X0[3 * b + 2] - cen[2];
      double* B = ns.data() + 18 * b;  // [3][6]
      B[0 * 6 + 0] = B[1 * 6 + 1] = B[2 * 6 + 2] = 1.0;
      B[0 * 6 + 3] = -y; B[1 * 6 + 3] = x;
      B[1 * 6 + 4] = -z; B[2 * 6 + 4] = y;
      B[0 * 6 + 5] = z;  B[2 * 6 + 5] = -x;
      int nd = 0;
      for (int d = 0; d < 3; ++d)
        if (dbc[size_t(3 * b + d)])
        {
          ++nd;
          for (int j = 0; j < 6; ++j) B[d * 6 + j] = 0.0;
        }
      skip[size_t(b)] = nd == 3;
    }
    coarsen(h, &h->A0, 3, std::move(ns), skip.data());
    if (h->levels.empty()) throw Fail{FCG_ERR_ARG, "fcg_amg_create: no coarse level (aggregation did not coarsen)"};
    for (double** v : {&h->r0, &h->d0, &h->z0, &h->q0, &h->p0, &h->ro0, &h->fr, &h->fz, &h->fx})
      *v = dalloc<double>(h, n);
    h->partial = dalloc<double>(h, kMaxPartials);
    h->sc = dalloc<double>(h, 16);  // [0, 6) outer FCG, 6 host dots, [8, 13) coarsest CG
    h->flag = dalloc<int32_t>(h, 1);
  }
  catch (const Fail& f)
  {
    ctx->last_error = f.msg;
    fcg_amg_destroy(h);
    return f.code;
  }
  *out = h;
  return FCG_OK;
}

int fcg_amg_setup(fcg_amg* h, const double* d_K_vals, void* stream)
{
  using namespace fcg_amgs;
  if (!h || !d_K_vals) return FCG_ERR_ARG;
  try
  {
    ck(hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->ctx->stream;
    hipEvent_t e0, e1;
    ck(hipEventCreate(&e0), "hipEventCreate");
    ck(hipEventCreate(&e1), "hipEventCreate");
    ck(hipEventRecord(e0, s), "hipEventRecord");
    if (h->gexec)  // its kernel arguments hold the previous setup's lambda_max values
    {
      (void)hipGraphExecDestroy(h->gexec);
      h->gexec = nullptr;
    }
    setup(h, d_K_vals, s);
    ck(hipEventRecord(e1, s), "hipEventRecord");
    ck(hipEventSynchronize(e1), "hipEventSynchronize");
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    h->setup_ms = ms;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    h->ready = true;
    h->local_ready = true;
  }
  catch (const Fail& f)
  {
    h->ready = false;
    h->local_ready = false;
    h->last_error = f.msg;
    h->ctx->last_error = f.msg;
    return f.code;
  }
  return FCG_OK;
}

int fcg_amg_iterate(fcg_amg* h, const double* d_K_vals, const double* d_b_row, double* d_x_row,
    double rtol, int max_iter, int* iterations, double* rel_residual, void* stream)
{
  using namespace fcg_amgs;
  if (!h || !d_K_vals || !d_b_row || !d_x_row || !(rtol >= 0.0) || max_iter < 0) return FCG_ERR_ARG;
  if (h->local)
  {
    // a rank of a partition: level 0 is only the owned block, so iterating here would solve the
    // block-diagonal local system and report it converged -- the solve across ranks is
    // fcg_dfcg_solve (this handle then serves as its preconditioner through setup / apply)
    h->last_error = "fcg_amg_iterate: multi-rank context (ghost columns) -- solve with fcg_dfcg_solve";
    h->ctx->last_error = h->last_error;
    return FCG_ERR_ARG;
  }
  if (!h->ready || !h->local_ready)
  {
    h->last_error = "fcg_amg_iterate: no numeric setup of the handle's own hierarchy for this K (call fcg_amg_setup first)";
    return FCG_ERR_ARG;
  }
  int it = 0;
  double rel = 0.0;
  try
  {
    ck(hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->ctx->stream;
    run_fcg(h, d_K_vals, d_b_row, d_x_row, rtol, max_iter, &it, &rel, s);
  }
  catch (const Fail& f)
  {
    h->last_error = f.msg;
    h->ctx->last_error = f.msg;
    if (iterations) *iterations = it;
    if (rel_residual) *rel_residual = rel;
    return f.code;
  }
  if (iterations) *iterations = it;
  if (rel_residual) *rel_residual = rel;
  return FCG_OK;
}

int fcg_amg_solve(fcg_amg* h, const double* d_K_vals, const double* d_b_row, double* d_x_row,
    double rtol, int max_iter, int* iterations, double* rel_residual, void* stream)
{
  if (iterations) *iterations = 0;
  if (rel_residual) *rel_residual = 0.0;
  if (!h || !d_K_vals || !d_b_row || !d_x_row || !(rtol >= 0.0) || max_iter < 0) return FCG_ERR_ARG;
  if (h->local)
  {
    h->last_error = "fcg_amg_solve: multi-rank context (ghost columns) -- solve with fcg_dfcg_solve";
    h->ctx->last_error = h->last_error;
    return FCG_ERR_ARG;
  }
  const int rc = fcg_amg_setup(h, d_K_vals, stream);
  if (rc != FCG_OK) return rc;
  return fcg_amg_iterate(h, d_K_vals, d_b_row, d_x_row, rtol, max_iter, iterations, rel_residual, stream);
}

int fcg_amg_level_info(const fcg_amg* h, int level, int64_t* dofs, int64_t* blocks, double* lmax)
{
  if (!h || level < 0 || level > int(h->levels.size())) return FCG_ERR_ARG;
  if (level == 0)
  {
    if (dofs) *dofs = h->n0;
    if (blocks) *blocks = h->A0.nnzb;
    if (lmax) *lmax = h->lmax0;
    return FCG_OK;
  }
  const fcg_amgs::Level& c = h->levels[size_t(level - 1)];
  if (dofs) *dofs = c.A.n * 6;
  if (blocks) *blocks = c.A.nnzb;
  if (lmax) *lmax = c.lmax;
  return FCG_OK;
}

int fcg_amg_levels(const fcg_amg* h) { return h ? int(h->levels.size()) + 1 : 0; }

double fcg_amg_setup_ms(const fcg_amg* h) { return h ? h->setup_ms : -1.0; }

int fcg_amg_stats(const fcg_amg* h, int* coarse_dense, int* graph_launches)
{
  if (!h) return FCG_ERR_ARG;
  if (coarse_dense) *coarse_dense = h->cinv ? 1 : 0;
  if (graph_launches) *graph_launches = h->graph_launches;
  return FCG_OK;
}

const char* fcg_amg_last_error(const fcg_amg* h) { return h ? h->last_error.c_str() : ""; }

int fcg_amg_apply(fcg_amg* h, const double* d_K_vals, const double* d_r_row, double* d_z_row,
    void* stream)
{
  using namespace fcg_amgs;
  if (!h || !d_K_vals || !d_r_row || !d_z_row) return FCG_ERR_ARG;
  if (!h->ready || !h->local_ready)
  {
    // after fcg_dfcg_solve's coupled setup only the coupled application is valid on this handle
    h->last_error = "fcg_amg_apply: no numeric setup of the handle's own hierarchy for this K (call fcg_amg_setup first)";
    return FCG_ERR_ARG;
  }
  try
  {
    ck(hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->ctx->stream;
    if (h->new2old)
    {
      const dim3 g(blocks_for(h->n0)), bl(kBlock);
      hipLaunchKernelGGL(node_perm_kernel, g, bl, 0, s, h->nb0, h->new2old, d_r_row, h->pb, 0);
      vcycle(h, 0, d_K_vals, h->pb, h->px, s);
      hipLaunchKernelGGL(node_perm_kernel, g, bl, 0, s, h->nb0, h->new2old, h->px, d_z_row, 1);
      ck(hipGetLastError(), "node_perm_kernel");
    }
    else
      vcycle(h, 0, d_K_vals, d_r_row, d_z_row, s);
  }
  catch (const Fail& f)
  {
    h->last_error = f.msg;
    h->ctx->last_error = f.msg;
    return f.code;
  }
  return FCG_OK;
}

// fcg_dfcg_solve's preconditioner (internal, fcg_internal.hpp): the numeric setup and one
// application -- coupled across ranks when the handle is rank-local and the transport names more
// than one rank (the coupled levels are built on the first call), else the handle's own V-cycle
int fcg_amg_precond_setup(fcg_amg* h, const double* d_K, const fcg_transport* tr, void* stream)
{
  using namespace fcg_amgs;
  // test hook: FCG_AMG_INJECT_FAIL_RANK=r makes rank r's local setup fail (tests/test_multigpu.py)
  static const int inject = [] {
    const char* e = std::getenv("FCG_AMG_INJECT_FAIL_RANK");
    return e ? std::atoi(e) : -1;
  }();
  int rc = FCG_OK;
  if (tr && tr->nranks > 1 && h->local)
  {
    try
    {
      ck(hipSetDevice(h->device), "hipSetDevice");
      h->local_ready = false;  // only the block inverses follow this K
      setup_coupled_local(h, d_K, stream ? static_cast<hipStream_t>(stream) : h->ctx->stream);
      h->ready = true;
    }
    catch (const Fail& f)
    {
      h->ready = false;
      h->last_error = f.msg;
      h->ctx->last_error = f.msg;
      rc = f.code;
    }
  }
  else
    rc = fcg_amg_setup(h, d_K, stream);
  if (rc == FCG_OK && tr && tr->nranks > 1 && tr->rank == inject)
  {
    h->ready = false;
    h->last_error = "coupled AMG: injected setup failure (FCG_AMG_INJECT_FAIL_RANK)";
    rc = FCG_ERR_SINGULAR;
  }
  if (!tr || tr->nranks <= 1) return rc;
  // Every rank of the transport enters the coupled levels' chain of collectives (imports, the
  // A_1 all-reduce) or none does: a go/no-go all-reduce of {local setup failed, handle not
  // rank-local} first, a status all-reduce after the build and numeric setup.  A rank that fails
  // alone would otherwise leave the others waiting in their next collective.
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->ctx->stream;
  auto agree = [&](double bad, double nonlocal, double* out) -> int {
    try
    {
      if (!h->agree) h->agree = dalloc<double>(h, 2);
      const double v[2] = {bad, nonlocal};
      ck(hipMemcpyAsync(h->agree, v, sizeof(v), hipMemcpyHostToDevice, s), "hipMemcpyAsync");
      ck(tr->allreduce_fn(tr->user, h->agree, 2, s), "transport all-reduce (go/no-go)");
      ck(hipMemcpyAsync(out, h->agree, 2 * sizeof(double), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
      ck(hipStreamSynchronize(s), "hipStreamSynchronize");
    }
    catch (const Fail& f)
    {
      h->last_error = f.msg;
      h->ctx->last_error = f.msg;
      return f.code;
    }
    return FCG_OK;
  };
  double g[2] = {0.0, 0.0};
  const int ra = agree(rc != FCG_OK ? 1.0 : 0.0, h->local ? 0.0 : 1.0, g);
  if (ra != FCG_OK) return ra;
  auto others_failed = [&](int code) {
    h->ready = false;
    h->last_error = "coupled AMG: the setup failed on another rank of the transport";
    h->ctx->last_error = h->last_error;
    return code;
  };
  if (g[0] > 0.0) return rc != FCG_OK ? rc : others_failed(FCG_ERR_DEVICE);
  if (g[1] > 0.0 && g[1] < double(tr->nranks))
  {
    h->last_error = "coupled AMG: the ranks disagree on whether their handles are rank-local";
    h->ctx->last_error = h->last_error;
    h->ready = false;
    return FCG_ERR_ARG;
  }
  if (!h->local) return FCG_OK;  // no rank's handle is rank-local: each keeps its own V-cycle
  int code = FCG_OK;
  // the build and the numeric setup over the guarded transport: a rank failing inside them meets
  // the others at their next collective (or at the final status below) and all stop together
  Guard G;
  G.in = tr;
  G.h = h;
  G.s = s;
  const fcg_transport gt = guarded(tr, &G);
  // test hook: FCG_AMG_INJECT_BUILD_FAIL="r:k" makes rank r throw inside coupled_build when it
  // reaches its k-th guarded collective (tests/test_multigpu.py, tests/cxx/config3_native.cpp)
  static const std::pair<int, int64_t> inject_build = [] {
    const char* e = std::getenv("FCG_AMG_INJECT_BUILD_FAIL");
    const char* c = e ? std::strchr(e, ':') : nullptr;
    return e ? std::make_pair(std::atoi(e), c ? int64_t(std::atoll(c + 1)) : int64_t(0))
             : std::make_pair(-1, int64_t(0));
  }();
  try
  {
    ck(hipSetDevice(h->device), "hipSetDevice");
    if (tr->rank < 0 || tr->rank >= tr->nranks) throw Fail{FCG_ERR_ARG, "coupled AMG: transport rank out of range"};
    if (!h->cpl)
    {
      try
      {
        if (tr->rank == inject_build.first) G.fail_at = inject_build.second;
        coupled_build(h, &gt, s);
        G.fail_at = -1;
      }
      catch (const Fail&)
      {
        // a failed build leaves no half-built coupling behind (its device buffers stay listed
        // in the handle's allocations until fcg_amg_destroy)
        if (h->cpl) fcg_amg_destroy(h->cpl->g);
        delete h->cpl;
        h->cpl = nullptr;
        throw;
      }
    }
    else if (h->cpl->rank != tr->rank || h->cpl->nranks != tr->nranks)
      throw Fail{FCG_ERR_ARG, "coupled AMG: the transport's rank / rank count changed"};
    coupled_setup(h, d_K, &gt, s);
  }
  catch (const Fail& f)
  {
    h->ready = false;
    if (G.remote)
      return others_failed(FCG_ERR_DEVICE);  // met another rank's failure at a collective: done
    h->last_error = f.msg;
    h->ctx->last_error = f.msg;
    code = f.code;
  }
  // the final status: the ranks that finished and the ranks that failed on their own meet here (a
  // rank that failed is at the same count of checkpoints as the others' next one)
  bool any = false;
  try
  {
    any = guard_checkpoint(&G, code != FCG_OK ? 1.0 : 0.0);
  }
  catch (const Fail& f)
  {
    h->ready = false;
    h->last_error = f.msg;
    h->ctx->last_error = f.msg;
    return code != FCG_OK ? code : f.code;
  }
  if (code != FCG_OK) return code;
  if (any) return others_failed(FCG_ERR_DEVICE);
  return FCG_OK;
}

int fcg_amg_precond_apply(fcg_amg* h, const double* d_K, const fcg_transport* tr, const double* d_r,
    double* d_z, void* stream)
{
  using namespace fcg_amgs;
  if (!h->cpl || !tr || tr->nranks <= 1) return fcg_amg_apply(h, d_K, d_r, d_z, stream);
  try
  {
    ck(hipSetDevice(h->device), "hipSetDevice");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : h->ctx->stream;
    coupled_apply(h, d_K, tr, d_r, d_z, s);
  }
  catch (const Fail& f)
  {
    h->last_error = f.msg;
    h->ctx->last_error = f.msg;
    return f.code;
  }
  return FCG_OK;
}

int fcg_amg_coupled_levels(const fcg_amg* h)
{
  if (!h || !h->cpl || !h->cpl->g) return 0;
  int n = int(h->cpl->g->levels.size());
  for (const fcg_amgs::Dist* d = h->cpl->d; d; d = d->next) ++n;
  return n;
}

int fcg_amg_coupled_stats(const fcg_amg* h, int64_t* out, int n)
{
  if (!h || !out || n < 0) return FCG_ERR_ARG;
  const fcg_amgs::Coupled* c = h->cpl;
  int64_t v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (c && c->g)
  {
    for (const fcg_amgs::Dist* d = c->d; d; d = d->next) ++v[0];
    v[1] = c->d ? c->d->na : c->n_agg_tot;
    v[2] = c->n_agg_tot;
    v[3] = c->ar_setup;
    v[4] = c->ar_apply;
    v[5] = c->x_setup;
    v[6] = c->x_apply;
    v[7] = fcg_amgs::hierarchy_bytes(c->g);
    v[8] = c->rep_n;
  }
  const int k = std::min(n, 9);
  for (int i = 0; i < k; ++i) out[i] = v[i];
  return k;
}

int fcg_amg_destroy(fcg_amg* h)
{
  if (!h) return FCG_OK;
  if (h->cpl)
  {
    fcg_amg_destroy(h->cpl->g);
    delete h->cpl;
    h->cpl = nullptr;
  }
  (void)hipSetDevice(h->device);
  if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
  if (h->gs)
  {
    (void)hipStreamSynchronize(h->gs);
    (void)hipStreamDestroy(h->gs);
  }
  for (hipEvent_t e : h->gev)
    if (e) (void)hipEventDestroy(e);
  for (void* p : h->allocs) (void)hipFree(p);
  delete h;
  return FCG_OK;
}

}  // extern "C"
