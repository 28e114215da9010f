// fcg_solver.hip -- what the Newton step around the assembly needs on the device (SURVEY §8f
// rows 1-2): Dirichlet rows applied to the assembled tangent and residual, the CSR operator, and
// a Jacobi-preconditioned conjugate-gradient solve, all on the HBM-resident K of the context.
//
//  * fcg_dirichlet_apply: Solid::Dbc::apply_dirichlet_to_local_system
//    (4C_structure_new_dbc.cpp:221-262): residual entries of the DBC DOFs are set to zero
//    (LinAlg::apply_dirichlet_to_system with zeros) after they were extracted as reaction forces
//    (extract_freact), and the matrix rows become unit rows -- SparseMatrix::apply_dirichlet with
//    diagonalblock = true (4C_linalg_sparsematrix.cpp:978-1097; the in-place branch, which keeps
//    the graph, is what runs here; the explicit branch yields the same values).
//  * fcg_spmv: y_row = K x_col (Epetra_CrsMatrix::Multiply on the local rows).
//  * fcg_pcg_solve: K x = b for a single-rank system (column map = row map), x_0 = 0.  With unit
//    DBC rows and zero DBC right-hand sides every iterate keeps x_D = 0, so CG on the row-modified
//    matrix is CG on K_FF.  All reductions are block partials summed in a fixed order: the solve
//    is bitwise reproducible.  (4C hands this system to Belos/MueLu through NOX,
//    4C_solver_nonlin_nox_linearsystem.cpp:275-353; the preconditioner here is block Jacobi on
//    the 3 x 3 nodal diagonal blocks -- Ifpack's point-block relaxation with the DOF triples of a
//    node as blocks.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "fcg_internal.hpp"
#include "fcg_status.hpp"

namespace fcg {

namespace {

constexpr int kBlock = 256;

// deterministic block sum (wave butterfly, then the waves in order); result valid in thread 0
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

// y = K x by node rows: the 3 rows of an owned node share one column pattern made of DOF triples
// (checked by fcg_create), so LPN lanes walk the node's neighbour triples -- one column index,
// x[c..c+2] and the 3 x 3 block of the 3 rows per triple -- instead of one index per matrix entry.
// Row-major sums in a fixed lane order: deterministic.  Optionally
// partial[blockIdx] = sum over the block's rows of dotw[row] * y[row].  V = float: matrix values
// stored in FP32 (the multigrid smoother's copy of K), vectors and sums in FP64.
template <int LPN, typename V>
__global__ __launch_bounds__(kBlock) void spmv_node_kernel(const int64_t* __restrict__ rowptr,
    const int32_t* __restrict__ row0_of, const int32_t* __restrict__ col,
    const V* __restrict__ vals, const double* __restrict__ x, double* __restrict__ y,
    int64_t n_nodes, const double* __restrict__ dotw, double* partial)
{
  __shared__ double sbuf[kBlock / 64];
  const int lane = threadIdx.x % LPN;
  const int64_t step = int64_t(gridDim.x) * (kBlock / LPN);
  double mine = 0.0;
  // grid-stride over the nodes: a bounded number of blocks keeps the dot partials few
  for (int64_t node = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / LPN; node - (threadIdx.x / LPN) <
       n_nodes; node += step)
  {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    int32_t row0 = 0;
    if (node < n_nodes)
    {
      row0 = row0_of[node];
      const int64_t s = rowptr[row0];
      const int64_t len = rowptr[row0 + 1] - s;
      const V* v0 = vals + s;
      const V* v1 = v0 + len;
      const V* v2 = v1 + len;
      for (int64_t k = 3 * lane; k < len; k += 3 * LPN)
      {
        const int32_t c = col[s + k];
        const double x0 = x[c], x1 = x[c + 1], x2 = x[c + 2];
        a0 += double(v0[k]) * x0 + double(v0[k + 1]) * x1 + double(v0[k + 2]) * x2;
        a1 += double(v1[k]) * x0 + double(v1[k + 1]) * x1 + double(v1[k + 2]) * x2;
        a2 += double(v2[k]) * x0 + double(v2[k + 1]) * x1 + double(v2[k + 2]) * x2;
      }
    }
#pragma unroll
    for (int o = LPN / 2; o >= 1; o >>= 1)
    {
      a0 += __shfl_xor(a0, o, LPN);
      a1 += __shfl_xor(a1, o, LPN);
      a2 += __shfl_xor(a2, o, LPN);
    }
    if (node < n_nodes && lane == 0)
    {
      y[row0] = a0;
      y[row0 + 1] = a1;
      y[row0 + 2] = a2;
      if (dotw) mine += dotw[row0] * a0 + dotw[row0 + 1] * a1 + dotw[row0 + 2] * a2;
    }
  }
  if (partial)
  {
    const double t = block_sum(mine, sbuf);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
  }
}

// Single-block reduction of n partials (fixed order) into sc[slot]; then the scalar recurrences
// of the PCG step (op: 0 = store only, 1 = alpha = sc[RZ] / sum, 2 = beta = sum / sc[RZ], RZ = sum)
enum { SC_RZ = 0, SC_PQ = 1, SC_RR = 2, SC_RZN = 3, SC_RR0 = 4, SC_BETA = 5, SC_ALPHA = 6, SC_BAD = 7, SC_N = 8 };
__global__ __launch_bounds__(kBlock) void reduce_kernel(const double* __restrict__ partial,
    int64_t n, double* sc, int slot, int op, const double* __restrict__ partial2, int slot2)
{
  __shared__ double sbuf[kBlock / 64];
  double a = 0.0, b = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock)
  {
    a += partial[i];
    if (partial2) b += partial2[i];
  }
  const double ta = block_sum(a, sbuf);
  const double tb = partial2 ? block_sum(b, sbuf) : 0.0;
  if (threadIdx.x != 0) return;
  sc[slot] = ta;
  if (partial2) sc[slot2] = tb;
  if (op == 1)
  {
    // CG breakdown: p.Kp must be positive for an SPD operator (NaN fails the test too) unless the
    // iteration already converged exactly (r = 0 -> z = p = 0 within a burst)
    if (!(sc[SC_PQ] > 0.0) && sc[SC_RZ] != 0.0) sc[SC_BAD] = 1.0;
    sc[SC_ALPHA] = sc[SC_PQ] > 0.0 ? sc[SC_RZ] / sc[SC_PQ] : 0.0;
  }
  if (op == 2)
  {
    sc[SC_BETA] = sc[SC_RZ] != 0.0 ? sc[SC_RZN] / sc[SC_RZ] : 0.0;
    sc[SC_RZ] = sc[SC_RZN];
  }
  if (op == 3)
  {
    sc[SC_RZ] = ta;  // init: rz and rr (= rr0)
    sc[SC_RR0] = tb;
    sc[SC_BAD] = 0.0;
  }
}

// Block-Jacobi preconditioner: z_A = D_AA^-1 r_A with D_AA the 3 x 3 diagonal block of owned node
// A (its rows' entries in the node's own DOF columns).  A Dirichlet row of the block is a unit row,
// so z keeps zeros on constrained DOFs and the preconditioner restricted to the free DOFs is the
// symmetric positive definite free part of the block.  One thread per owned node.
__device__ inline void bj_apply(const double* __restrict__ Dinv, const double* r, double* z)
{
  z[0] = Dinv[0] * r[0] + Dinv[1] * r[1] + Dinv[2] * r[2];
  z[1] = Dinv[3] * r[0] + Dinv[4] * r[1] + Dinv[5] * r[2];
  z[2] = Dinv[6] * r[0] + Dinv[7] * r[1] + Dinv[8] * r[2];
}

// init: x = 0, r = b, z = D^-1 r, p = z; partials r.z, r.r
__global__ __launch_bounds__(kBlock) void pcg_init_kernel(const int32_t* __restrict__ row0_of,
    const double* __restrict__ b, const double* __restrict__ dinv, double* x, double* r, double* z,
    double* p, int64_t n_nodes, double* part_rz, double* part_rr)
{
  __shared__ double sbuf[kBlock / 64];
  double rz = 0.0, rr = 0.0;
  for (int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x; k < n_nodes;
       k += int64_t(gridDim.x) * kBlock)
  {
    const int32_t i = row0_of[k];
    double ri[3], zi[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) ri[d] = b[i + d];
    bj_apply(dinv + 9 * k, ri, zi);
#pragma unroll
    for (int d = 0; d < 3; ++d)
    {
      x[i + d] = 0.0;
      r[i + d] = ri[d];
      z[i + d] = zi[d];
      p[i + d] = zi[d];
      rz += ri[d] * zi[d];
      rr += ri[d] * ri[d];
    }
  }
  const double a = block_sum(rz, sbuf);
  const double c = block_sum(rr, sbuf);
  if (threadIdx.x == 0)
  {
    part_rz[blockIdx.x] = a;
    part_rr[blockIdx.x] = c;
  }
}

// x += alpha p, r -= alpha q, z = D^-1 r; partials r.z, r.r
__global__ __launch_bounds__(kBlock) void pcg_update_kernel(const int32_t* __restrict__ row0_of,
    const double* __restrict__ p, const double* __restrict__ q, const double* __restrict__ dinv,
    double* x, double* r, double* z, int64_t n_nodes, const double* sc, double* part_rz,
    double* part_rr)
{
  __shared__ double sbuf[kBlock / 64];
  const double alpha = sc[SC_ALPHA];
  double rz = 0.0, rr = 0.0;
  for (int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x; k < n_nodes;
       k += int64_t(gridDim.x) * kBlock)
  {
    const int32_t i = row0_of[k];
    double ri[3], zi[3];
#pragma unroll
    for (int d = 0; d < 3; ++d)
    {
      x[i + d] += alpha * p[i + d];
      ri[d] = r[i + d] - alpha * q[i + d];
    }
    bj_apply(dinv + 9 * k, ri, zi);
#pragma unroll
    for (int d = 0; d < 3; ++d)
    {
      r[i + d] = ri[d];
      z[i + d] = zi[d];
      rz += ri[d] * zi[d];
      rr += ri[d] * ri[d];
    }
  }
  const double a = block_sum(rz, sbuf);
  const double c = block_sum(rr, sbuf);
  if (threadIdx.x == 0)
  {
    part_rz[blockIdx.x] = a;
    part_rr[blockIdx.x] = c;
  }
}

__global__ __launch_bounds__(kBlock) void pcg_dir_kernel(const double* __restrict__ z, double* p,
    int64_t n, const double* sc)
{
  const double beta = sc[SC_BETA];
  const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) p[i] = z[i] + beta * p[i];
}

// D_AA^-1 per owned node: the block's row d sits in row row0 + d at the columns of the node's own
// DOF triple, which starts at the diagonal entry's position minus d
__global__ __launch_bounds__(kBlock) void block_jacobi_kernel(const int32_t* __restrict__ row0_of,
    const int64_t* __restrict__ diag_pos, const double* __restrict__ K, double* dinv,
    int64_t n_nodes, int32_t* bad)
{
  const int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= n_nodes) return;
  const int32_t i = row0_of[k];
  double m[9];  // column-major, as invert3x3 of the element kernels
  bool ok = true;
#pragma unroll
  for (int d = 0; d < 3; ++d)
  {
    const int64_t dp = diag_pos[i + d];
    ok = ok && dp >= 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) m[d + 3 * c] = dp >= 0 ? K[dp - d + c] : 0.0;
  }
  const double c00 = m[4] * m[8] - m[7] * m[5], c01 = m[7] * m[2] - m[1] * m[8],
               c02 = m[1] * m[5] - m[4] * m[2];
  const double det = m[0] * c00 + m[3] * c01 + m[6] * c02;
  double* o = dinv + 9 * k;  // row-major inverse
  if (!ok || det == 0.0 || !(det == det))
  {
    atomicMax(bad, 1);
#pragma unroll
    for (int q = 0; q < 9; ++q) o[q] = 0.0;
    return;
  }
  const double id = 1.0 / det;
  // inverse (row-major): inv(r, c) = cofactor(c, r) / det
  o[0] = c00 * id;
  o[1] = (m[6] * m[5] - m[3] * m[8]) * id;
  o[2] = (m[3] * m[7] - m[6] * m[4]) * id;
  o[3] = c01 * id;
  o[4] = (m[0] * m[8] - m[6] * m[2]) * id;
  o[5] = (m[6] * m[1] - m[0] * m[7]) * id;
  o[6] = c02 * id;
  o[7] = (m[3] * m[2] - m[0] * m[5]) * id;
  o[8] = (m[0] * m[4] - m[3] * m[1]) * id;
}

// Dirichlet rows: one wavefront per DBC row
__global__ __launch_bounds__(kBlock) void dirichlet_kernel(const int64_t* __restrict__ rowptr,
    const int64_t* __restrict__ diag_pos, const int32_t* __restrict__ rows, int64_t n_dbc,
    int64_t n_rows, double* K, double* rhs, double* freact, int32_t* bad)
{
  const int64_t k = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (k >= n_dbc) return;
  const int32_t row = rows[k];
  if (row < 0 || row >= n_rows)
  {
    if (lane == 0) atomicMax(bad, 2);
    return;
  }
  const int64_t dp = diag_pos[row];
  if (dp < 0)
  {
    if (lane == 0) atomicMax(bad, 1);
    return;
  }
  if (K)
    for (int64_t j = rowptr[row] + lane; j < rowptr[row + 1]; j += 64) K[j] = j == dp ? 1.0 : 0.0;
  if (lane == 0 && rhs)
  {
    if (freact) freact[row] = -rhs[row];  // extract_freact: freact().scale(-1.0), 4C_structure_new_dbc.cpp:389-394
    rhs[row] = 0.0;
  }
}

// z = scale D^-1 r (+ z if accumulate) per owned node: the smoother step of the multigrid
// preconditioner (4c_amd/multigrid.py)
__global__ __launch_bounds__(kBlock) void bj_apply_kernel(const int32_t* __restrict__ row0_of,
    const double* __restrict__ dinv, const double* __restrict__ r, double* z, int64_t n_nodes,
    double scale, int accumulate)
{
  const int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= n_nodes) return;
  const int32_t i = row0_of[k];
  double ri[3], zi[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) ri[d] = r[i + d];
  bj_apply(dinv + 9 * k, ri, zi);
#pragma unroll
  for (int d = 0; d < 3; ++d) z[i + d] = __fma_rn(scale, zi[d], accumulate ? z[i + d] : 0.0);
}

// fcg_chebyshev_step: the smoother update per node (fourc_gpu.h); d = c_d d first, then the
// block-Jacobi term added as in bj_apply_kernel, so the result equals the separate passes
__global__ __launch_bounds__(kBlock) void cheb_step_kernel(const int32_t* __restrict__ row0_of,
    const double* __restrict__ dinv, const double* __restrict__ b, const double* __restrict__ y, double* dv,
    double* x, int64_t n_nodes, double c_d, double c_r, int mode)
{
  const int64_t k = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= n_nodes) return;
  const int32_t i = row0_of[k];
  double ri[3], zi[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) ri[d] = mode == 2 ? b[i + d] : b[i + d] - y[i + d];
  bj_apply(dinv + 9 * k, ri, zi);
#pragma unroll
  for (int d = 0; d < 3; ++d)
  {
    // the rounded c_d d, then one fused multiply-add (as the accumulating bj_apply_kernel)
    const double dn = __fma_rn(c_r, zi[d], mode == 1 ? __dmul_rn(c_d, dv[i + d]) : 0.0);
    dv[i + d] = dn;
    x[i + d] = mode == 2 ? dn : x[i + d] + dn;
  }
}

// Node-block transfer between two discretizations of one box (multigrid prolongation and its
// transpose): y[dst_row0[o] + d] = (accumulate ? y : 0) + sum_j w[j] x[src_row0[j] + d] over
// j in [ptr[o], ptr[o+1]), d = 0..2.  Fixed summation order: deterministic.
__global__ __launch_bounds__(kBlock) void node_transfer_kernel(const int64_t* __restrict__ ptr,
    const int32_t* __restrict__ src_row0, const double* __restrict__ w,
    const int32_t* __restrict__ dst_row0, const double* __restrict__ x, double* y, int64_t n_out,
    int accumulate)
{
  const int64_t o = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (o >= n_out) return;
  const int32_t dr = dst_row0[o];
  if (dr < 0) return;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  for (int64_t j = ptr[o]; j < ptr[o + 1]; ++j)
  {
    const int32_t sr = src_row0[j];
    const double wj = w[j];
    a0 += wj * x[sr];
    a1 += wj * x[sr + 1];
    a2 += wj * x[sr + 2];
  }
  if (accumulate)
  {
    a0 += y[dr];
    a1 += y[dr + 1];
    a2 += y[dr + 2];
  }
  y[dr] = a0;
  y[dr + 1] = a1;
  y[dr + 2] = a2;
}

inline unsigned blocks_for(int64_t n, int per_block) { return unsigned((n + per_block - 1) / per_block); }
// grid-stride kernels with dot partials: at most this many blocks (16 per CU of a 256-CU part),
// so the single-block reductions of the partials stay short
constexpr int64_t kMaxBlocks = 4096;
inline unsigned capped_blocks(int64_t n, int per_block)
{
  return unsigned(std::min<int64_t>(kMaxBlocks, std::max<int64_t>(1, (n + per_block - 1) / per_block)));
}

// one node per LPN lanes; with dot partials the grid is capped (grid-stride) so they stay few
inline unsigned spmv_grid(const DeviceMesh& m, int lpn, bool partials)
{
  return partials ? capped_blocks(m.n_rownodes * lpn, kBlock) : blocks_for(m.n_rownodes * lpn, kBlock);
}

// y = K x on a GridGenerator hex8 box whose elements are all the same parallelepiped (the
// multigrid's rediscretised coarse levels): a 27-point stencil of 3 x 3 blocks per node class
// (low face / interior / high face along each axis: 27 classes), S[class][offset][3 x 3] summed
// from the one element matrix; rows of clamped nodes are unit rows (y = x).  One thread per node,
// its 27 neighbours' DOF triples read through the lattice's row table.
__global__ __launch_bounds__(kBlock) void box_stencil_kernel(int nx, int ny, int nz,
    const int32_t* __restrict__ row_of, const uint8_t* __restrict__ clamped,
    const double* __restrict__ S, const double* __restrict__ x, double* __restrict__ y)
{
  const int64_t n = int64_t(nx) * ny * nz;
  const int64_t id = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (id >= n) return;
  const int i = int(id % nx), j = int((id / nx) % ny), k = int(id / (int64_t(nx) * ny));
  const int32_t r0 = row_of[id];
  if (r0 < 0) return;
  if (clamped[id])
  {
    y[r0] = x[r0];
    y[r0 + 1] = x[r0 + 1];
    y[r0 + 2] = x[r0 + 2];
    return;
  }
  const int cls = (i == 0 ? 0 : (i == nx - 1 ? 2 : 1)) + 3 * (j == 0 ? 0 : (j == ny - 1 ? 2 : 1)) +
                  9 * (k == 0 ? 0 : (k == nz - 1 ? 2 : 1));
  const double* Sc = S + 243 * cls;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll 3
  for (int o = 0; o < 27; ++o)
  {
    const int di = o % 3 - 1, dj = (o / 3) % 3 - 1, dk = o / 9 - 1;
    const int ii = i + di, jj = j + dj, kk = k + dk;
    if (ii < 0 || ii >= nx || jj < 0 || jj >= ny || kk < 0 || kk >= nz) continue;
    const int32_t c = row_of[(int64_t(kk) * ny + jj) * nx + ii];
    const double x0 = x[c], x1 = x[c + 1], x2 = x[c + 2];
    const double* B = Sc + 9 * o;
    a0 += B[0] * x0 + B[1] * x1 + B[2] * x2;
    a1 += B[3] * x0 + B[4] * x1 + B[5] * x2;
    a2 += B[6] * x0 + B[7] * x1 + B[8] * x2;
  }
  y[r0] = a0;
  y[r0 + 1] = a1;
  y[r0 + 2] = a2;
}

// Multigrid transfer between a GridGenerator box lattice and its 2:1 coarsening (fine lattice
// 2 (n_c - 1) + 1 points per axis: hex27 -> hex8 on the same elements, hex8 n -> n / 2), weights
// implicit (1 on a coincident point, 1/2 to both neighbours of a midpoint, products over the
// axes) instead of read from tables.  mode 0, prolongation, one thread per fine node:
// y_f (+)= sum_c w x_c; mode 1, restriction (the transpose), one thread per coarse node:
// y_c = sum_f w x_f.  Rows whose node is flagged in zero_out are set to 0 (the level's Dirichlet
// mask).  Fixed summation order: deterministic.
__global__ __launch_bounds__(kBlock) void box_transfer_kernel(int mode, int fnx, int fny, int fnz,
    int cnx, int cny, int cnz, const int32_t* __restrict__ frow, const int32_t* __restrict__ crow,
    const uint8_t* __restrict__ zero_out, const double* __restrict__ x, double* __restrict__ y,
    int accumulate)
{
  const int64_t id = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (mode == 0)
  {
    if (id >= int64_t(fnx) * fny * fnz) return;
    const int i = int(id % fnx), j = int((id / fnx) % fny), k = int(id / (int64_t(fnx) * fny));
    const int32_t r = frow[id];
    if (r < 0) return;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    if (!zero_out[id])
    {
      const int ni = 1 + (i & 1), nj = 1 + (j & 1), nk = 1 + (k & 1);
      const double wi = (i & 1) ? 0.5 : 1.0, wj = (j & 1) ? 0.5 : 1.0, wk = (k & 1) ? 0.5 : 1.0;
      for (int c = 0; c < nk; ++c)
        for (int b = 0; b < nj; ++b)
          for (int a = 0; a < ni; ++a)
          {
            const int32_t s = crow[(int64_t((k >> 1) + c) * cny + (j >> 1) + b) * cnx + (i >> 1) + a];
            const double w = wi * wj * wk;
            a0 += w * x[s];
            a1 += w * x[s + 1];
            a2 += w * x[s + 2];
          }
      if (accumulate)
      {
        a0 += y[r];
        a1 += y[r + 1];
        a2 += y[r + 2];
      }
    }
    y[r] = a0;
    y[r + 1] = a1;
    y[r + 2] = a2;
    return;
  }
  if (id >= int64_t(cnx) * cny * cnz) return;
  const int I = int(id % cnx), J = int((id / cnx) % cny), K = int(id / (int64_t(cnx) * cny));
  const int32_t r = crow[id];
  if (r < 0) return;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  if (!zero_out[id])
    for (int dk = -1; dk <= 1; ++dk)
    {
      const int k = 2 * K + dk;
      if (k < 0 || k >= fnz) continue;
      for (int dj = -1; dj <= 1; ++dj)
      {
        const int j = 2 * J + dj;
        if (j < 0 || j >= fny) continue;
        for (int di = -1; di <= 1; ++di)
        {
          const int i = 2 * I + di;
          if (i < 0 || i >= fnx) continue;
          const int32_t s = frow[(int64_t(k) * fny + j) * fnx + i];
          if (s < 0) continue;
          const double w = (di ? 0.5 : 1.0) * (dj ? 0.5 : 1.0) * (dk ? 0.5 : 1.0);
          a0 += w * x[s];
          a1 += w * x[s + 1];
          a2 += w * x[s + 2];
        }
      }
    }
  y[r] = a0;
  y[r + 1] = a1;
  y[r + 2] = a2;
}

// partial[blockIdx] = sum over the block's rows of p . q (grid-stride, fixed assignment)
__global__ __launch_bounds__(kBlock) void dot_kernel(const double* __restrict__ p,
    const double* __restrict__ q, int64_t n, double* partial)
{
  __shared__ double sbuf[kBlock / 64];
  double t = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
    t += p[i] * q[i];
  const double b = block_sum(t, sbuf);
  if (threadIdx.x == 0) partial[blockIdx.x] = b;
}

template <typename V>
hipError_t launch_spmv(const DeviceMesh& m, const V* K, const double* x, double* y,
    const double* dotw, double* partial, hipStream_t s)
{
  if (m.n_rows == 0) return hipSuccess;
  // node rows (every owned row belongs to a node triple, fcg_create checks the pattern)
  if (m.npe == 27)
    hipLaunchKernelGGL((spmv_node_kernel<64, V>), dim3(spmv_grid(m, 64, partial != nullptr)),
        dim3(kBlock), 0, s, m.rowptr, m.rownode_row0, m.col_lid, K, x, y, m.n_rownodes, dotw,
        partial);
  else
    hipLaunchKernelGGL((spmv_node_kernel<16, V>), dim3(spmv_grid(m, 16, partial != nullptr)),
        dim3(kBlock), 0, s, m.rowptr, m.rownode_row0, m.col_lid, K, x, y, m.n_rownodes, dotw,
        partial);
  return hipGetLastError();
}


}  // namespace

}  // namespace fcg

extern "C" {

int fcg_spmv(fcg_ctx* ctx, const double* d_K_vals, const double* d_x_col, double* d_y_row,
    void* stream)
{
  if (!ctx || (ctx->mesh.n_rows > 0 && (!d_K_vals || !d_x_col || !d_y_row))) return FCG_ERR_ARG;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const hipError_t he = fcg::launch_spmv(ctx->mesh, d_K_vals, d_x_col, d_y_row, nullptr, nullptr, s);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  return FCG_OK;
}

int fcg_spmv_f32(fcg_ctx* ctx, const float* d_K32, const double* d_x_col, double* d_y_row,
    void* stream)
{
  if (!ctx || (ctx->mesh.n_rows > 0 && (!d_K32 || !d_x_col || !d_y_row))) return FCG_ERR_ARG;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  hipError_t he = fcg::launch_spmv(ctx->mesh, d_K32, d_x_col, d_y_row, nullptr, nullptr, s);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  return FCG_OK;
}

int fcg_tangent_apply(fcg_ctx* ctx, const double* d_u_col, const double* d_x_col, double* d_y_row,
    void* stream)
{
  if (!ctx) return FCG_ERR_ARG;
  fcg::DeviceMesh& m = ctx->mesh;
  if (m.npe != 27 || m.material != FCG_MAT_STVK || !m.inc_of || !m.inc_ptr || !m.rownode_row0)
  {
    ctx->last_error = "fcg_tangent_apply: hex27 St.Venant-Kirchhoff contexts only";
    return FCG_ERR_ARG;
  }
  if (m.n_rows > 0 && (!d_x_col || !d_y_row || (m.kinem != 0 && !d_u_col))) return FCG_ERR_ARG;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (!m.apply_ye && m.n_inc > 0)
  {
    const size_t bytes = size_t(m.n_inc + 1) * 3 * sizeof(double);  // + the spare triple
    const hipError_t he = hipMalloc(&m.apply_ye, bytes);
    if (he != hipSuccess)
    {
      m.apply_ye = nullptr;
      ctx->last_error = std::string("fcg_tangent_apply: hipMalloc: ") + hipGetErrorString(he);
      return fcg_device_error();
    }
    ctx->device_bytes += int64_t(bytes);
  }
  if (!m.apply_dof && m.n_ele > 0)
  {
    const size_t bytes = size_t(m.n_ele) * 27 * sizeof(int32_t);
    hipError_t he = hipMalloc(&m.apply_dof, bytes);
    if (he == hipSuccess) he = fcg::launch_h27_apply_plan(m, s);
    if (he != hipSuccess)
    {
      if (m.apply_dof) (void)hipFree(m.apply_dof);
      m.apply_dof = nullptr;
      ctx->last_error = std::string("fcg_tangent_apply: gather plan: ") + hipGetErrorString(he);
      return fcg_device_error();
    }
    ctx->device_bytes += int64_t(bytes);
  }
  const hipError_t he = fcg::launch_h27_apply(m, d_u_col, d_x_col, d_y_row, s);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  return FCG_OK;
}

int fcg_dirichlet_apply(fcg_ctx* ctx, int64_t n_dbc, const int32_t* d_rows, double* d_K_vals,
    double* d_rhs_row, double* d_freact_row, void* stream)
{
  if (!ctx || n_dbc < 0 || (n_dbc > 0 && !d_rows)) return FCG_ERR_ARG;
  if (n_dbc == 0) return FCG_OK;
  fcg::DeviceMesh& m = ctx->mesh;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const int32_t zero = 0;
  int32_t* flag = m.err + 2;  // the solver flag word: evaluate's sticky flags are left alone
  hipError_t he = hipMemcpyAsync(flag, &zero, sizeof(zero), hipMemcpyHostToDevice, s);
  if (he == hipSuccess)
  {
    hipLaunchKernelGGL(fcg::dirichlet_kernel, dim3(fcg::blocks_for(n_dbc * 64, fcg::kBlock)),
        dim3(fcg::kBlock), 0, s, m.rowptr, m.diag_pos, d_rows, n_dbc, m.n_rows, d_K_vals, d_rhs_row,
        d_freact_row, flag);
    he = hipGetLastError();
  }
  int32_t bad = 0;
  if (he == hipSuccess) he = hipMemcpyAsync(&bad, flag, sizeof(bad), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  if (bad)
  {
    ctx->last_error = bad == 2 ? "Dirichlet row LID out of range" : "Dirichlet row without a diagonal entry";
    return FCG_ERR_ARG;
  }
  return FCG_OK;
}

int fcg_pcg_solve(fcg_ctx* ctx, const double* d_K_vals, const double* d_b_row, double* d_x_row,
    double rtol, int max_iter, int* iterations, double* rel_residual, void* stream)
{
  if (!ctx || !(rtol >= 0.0) || max_iter < 0) return FCG_ERR_ARG;
  fcg::DeviceMesh& m = ctx->mesh;
  if (!m.square_local)
  {
    ctx->last_error = "fcg_pcg_solve needs a single-rank system (matrix column map = row map)";
    return FCG_ERR_ARG;
  }
  const int64_t n = m.n_rows;
  if (iterations) *iterations = 0;
  if (rel_residual) *rel_residual = 0.0;
  if (n == 0) return FCG_OK;
  if (!d_K_vals || !d_b_row || !d_x_row) return FCG_ERR_ARG;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  hipError_t he = hipSuccess;
  const int64_t nn = m.n_rownodes;
  if (3 * nn != n)
  {
    ctx->last_error = "fcg_pcg_solve: every owned row must belong to an owned node's DOF triple";
    return FCG_ERR_ARG;
  }
  const int64_t nb_vec = fcg::blocks_for(n, fcg::kBlock);
  const int64_t nb_node = fcg::capped_blocks(nn, fcg::kBlock);
  const int64_t nb_dot = fcg::capped_blocks(n, fcg::kBlock);
  const int64_t nb = std::max(nb_node, nb_dot);
  if (!m.pcg_work || m.pcg_n != n)
  {
    if (m.pcg_work) (void)hipFree(m.pcg_work);
    m.pcg_work = nullptr;
    he = hipMalloc(reinterpret_cast<void**>(&m.pcg_work), sizeof(double) * (7 * n + 3 * nb + fcg::SC_N));
    if (he != hipSuccess)
    {
      ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
      return fcg_device_error();
    }
    m.pcg_n = n;
  }
  double* r = m.pcg_work;
  double* z = r + n;
  double* p = z + n;
  double* q = p + n;
  double* dinv = q + n;
  double* pa = dinv + 3 * n;  // dinv: 9 doubles per owned node
  double* pb = pa + nb;
  double* pc = pb + nb;
  double* sc = pc + nb;
  const int32_t zero = 0;
  int32_t* flag = m.err + 2;  // the solver flag word: evaluate's sticky flags are left alone
  he = hipMemcpyAsync(flag, &zero, sizeof(zero), hipMemcpyHostToDevice, s);
  if (he == hipSuccess)
  {
    hipLaunchKernelGGL(fcg::block_jacobi_kernel, dim3(fcg::blocks_for(nn, fcg::kBlock)), dim3(fcg::kBlock), 0, s,
        m.rownode_row0, m.diag_pos, d_K_vals, dinv, nn, flag);
    hipLaunchKernelGGL(fcg::pcg_init_kernel, dim3(nb_node), dim3(fcg::kBlock), 0, s, m.rownode_row0,
        d_b_row, dinv, d_x_row, r, z, p, nn, pa, pb);
    hipLaunchKernelGGL(fcg::reduce_kernel, dim3(1), dim3(fcg::kBlock), 0, s, pa, nb_node, sc,
        int(fcg::SC_RZ), 3, pb, int(fcg::SC_RR));
    he = hipGetLastError();
  }
  double hsc[fcg::SC_N] = {0};
  int32_t bad = 0;
  if (he == hipSuccess) he = hipMemcpyAsync(hsc, sc, sizeof(hsc), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipMemcpyAsync(&bad, flag, sizeof(bad), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  if (bad)
  {
    ctx->last_error = "singular or missing diagonal node block (block-Jacobi preconditioner)";
    return FCG_ERR_SINGULAR;
  }
  const double rr0 = hsc[fcg::SC_RR0];
  if (!std::isfinite(rr0) || !std::isfinite(hsc[fcg::SC_RZ]))
  {
    ctx->last_error = "fcg_pcg_solve: non-finite right-hand side or preconditioned residual";
    return FCG_ERR_SINGULAR;
  }
  if (rr0 == 0.0) return FCG_OK;  // b = 0 -> x = 0
  const double target = rtol * rtol * rr0;
  int it = 0;
  double rr = rr0;
  const int check_every = 8;
  while (it < max_iter && rr > target)
  {
    const int burst = std::min(check_every, max_iter - it);
    for (int k = 0; k < burst; ++k)
    {
      // q = K p (full-width grid), then p . q over a capped grid of block partials
      he = fcg::launch_spmv(m, d_K_vals, p, q, nullptr, nullptr, s);
      if (he != hipSuccess) break;
      hipLaunchKernelGGL(fcg::dot_kernel, dim3(nb_dot), dim3(fcg::kBlock), 0, s, p, q, n, pa);
      hipLaunchKernelGGL(fcg::reduce_kernel, dim3(1), dim3(fcg::kBlock), 0, s, pa, nb_dot, sc,
          int(fcg::SC_PQ), 1, nullptr, 0);
      hipLaunchKernelGGL(fcg::pcg_update_kernel, dim3(nb_node), dim3(fcg::kBlock), 0, s,
          m.rownode_row0, p, q, dinv, d_x_row, r, z, nn, sc, pb, pc);
      hipLaunchKernelGGL(fcg::reduce_kernel, dim3(1), dim3(fcg::kBlock), 0, s, pb, nb_node, sc,
          int(fcg::SC_RZN), 2, pc, int(fcg::SC_RR));
      hipLaunchKernelGGL(fcg::pcg_dir_kernel, dim3(nb_vec), dim3(fcg::kBlock), 0, s, z, p, n, sc);
      he = hipGetLastError();
      if (he != hipSuccess) break;
    }
    if (he == hipSuccess) he = hipMemcpyAsync(hsc, sc, sizeof(hsc), hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    if (he != hipSuccess)
    {
      ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
      return fcg_device_error();
    }
    it += burst;
    rr = hsc[fcg::SC_RR];
    if (!std::isfinite(rr) || hsc[fcg::SC_BAD] != 0.0)
    {
      if (iterations) *iterations = it;
      if (rel_residual) *rel_residual = std::sqrt(rr / rr0);
      ctx->last_error = !std::isfinite(rr)
                            ? "fcg_pcg_solve: non-finite residual (diverged)"
                            : "fcg_pcg_solve: breakdown, p.Kp <= 0 (matrix not positive definite)";
      return FCG_ERR_SINGULAR;
    }
  }
  if (iterations) *iterations = it;
  if (rel_residual) *rel_residual = std::sqrt(rr / rr0);
  return FCG_OK;
}

int fcg_block_jacobi_setup(fcg_ctx* ctx, const double* d_K_vals, double* d_dinv, void* stream)
{
  if (!ctx || !d_K_vals || !d_dinv) return FCG_ERR_ARG;
  fcg::DeviceMesh& m = ctx->mesh;
  const int64_t nn = m.n_rownodes;
  if (3 * nn != m.n_rows)
  {
    ctx->last_error = "fcg_block_jacobi_setup: every owned row must belong to an owned node's DOF triple";
    return FCG_ERR_ARG;
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  const int32_t zero = 0;
  int32_t bad = 0;
  int32_t* flag = m.err + 2;  // the solver flag word: evaluate's sticky flags are left alone
  hipError_t he = hipMemcpyAsync(flag, &zero, sizeof(zero), hipMemcpyHostToDevice, s);
  if (he == hipSuccess && nn > 0)
  {
    hipLaunchKernelGGL(fcg::block_jacobi_kernel, dim3(fcg::blocks_for(nn, fcg::kBlock)), dim3(fcg::kBlock), 0, s,
        m.rownode_row0, m.diag_pos, d_K_vals, d_dinv, nn, flag);
    he = hipGetLastError();
  }
  if (he == hipSuccess) he = hipMemcpyAsync(&bad, flag, sizeof(bad), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  if (bad)
  {
    ctx->last_error = "singular or missing diagonal node block (block-Jacobi preconditioner)";
    return FCG_ERR_SINGULAR;
  }
  return FCG_OK;
}

int fcg_block_jacobi_apply(fcg_ctx* ctx, const double* d_dinv, const double* d_r_row, double* d_z_row,
    double scale, int accumulate, void* stream)
{
  if (!ctx || !d_dinv || !d_r_row || !d_z_row) return FCG_ERR_ARG;
  fcg::DeviceMesh& m = ctx->mesh;
  const int64_t nn = m.n_rownodes;
  if (nn == 0) return FCG_OK;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  hipLaunchKernelGGL(fcg::bj_apply_kernel, dim3(fcg::blocks_for(nn, fcg::kBlock)), dim3(fcg::kBlock), 0, s,
      m.rownode_row0, d_dinv, d_r_row, d_z_row, nn, scale, accumulate);
  const hipError_t he = hipGetLastError();
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  return FCG_OK;
}

int fcg_chebyshev_step(fcg_ctx* ctx, const double* d_dinv, const double* d_b_row, const double* d_y_row,
    double* d_d_row, double* d_x_row, double c_d, double c_r, int mode, void* stream)
{
  if (!ctx || !d_dinv || !d_b_row || (!d_y_row && mode != 2) || !d_d_row || !d_x_row || mode < 0 || mode > 2)
    return FCG_ERR_ARG;
  fcg::DeviceMesh& m = ctx->mesh;
  const int64_t nn = m.n_rownodes;
  if (nn == 0) return FCG_OK;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  hipLaunchKernelGGL(fcg::cheb_step_kernel, dim3(fcg::blocks_for(nn, fcg::kBlock)), dim3(fcg::kBlock), 0, s,
      m.rownode_row0, d_dinv, d_b_row, mode == 2 ? d_b_row : d_y_row, d_d_row, d_x_row, nn, c_d, c_r, mode);
  const hipError_t he = hipGetLastError();
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  return FCG_OK;
}

int fcg_node_transfer(int device, int64_t n_out, const int64_t* d_ptr, const int32_t* d_src_row0,
    const double* d_w, const int32_t* d_dst_row0, const double* d_x, double* d_y, int accumulate,
    void* stream)
{
  if (n_out < 0 || (n_out > 0 && (!d_ptr || !d_src_row0 || !d_w || !d_dst_row0 || !d_x || !d_y)))
    return FCG_ERR_ARG;
  if (n_out == 0) return FCG_OK;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(fcg::node_transfer_kernel, dim3(fcg::blocks_for(n_out, fcg::kBlock)), dim3(fcg::kBlock), 0, s,
      d_ptr, d_src_row0, d_w, d_dst_row0, d_x, d_y, n_out, accumulate);
  return hipGetLastError() == hipSuccess ? FCG_OK : fcg_device_error();
}

int fcg_box_transfer(int device, int mode, int fnx, int fny, int fnz, int cnx, int cny, int cnz,
    const int32_t* d_fine_row_of, const int32_t* d_coarse_row_of, const uint8_t* d_zero_out,
    const double* d_x, double* d_y, int accumulate, void* stream)
{
  if ((mode != 0 && mode != 1) || cnx < 2 || cny < 2 || cnz < 2 || fnx != 2 * cnx - 1 ||
      fny != 2 * cny - 1 || fnz != 2 * cnz - 1 || !d_fine_row_of || !d_coarse_row_of || !d_zero_out ||
      !d_x || !d_y)
    return FCG_ERR_ARG;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = mode == 0 ? int64_t(fnx) * fny * fnz : int64_t(cnx) * cny * cnz;
  hipLaunchKernelGGL(fcg::box_transfer_kernel, dim3(fcg::blocks_for(n, fcg::kBlock)), dim3(fcg::kBlock), 0, s,
      mode, fnx, fny, fnz, cnx, cny, cnz, d_fine_row_of, d_coarse_row_of, d_zero_out, d_x, d_y, accumulate);
  return hipGetLastError() == hipSuccess ? FCG_OK : fcg_device_error();
}

int fcg_box_stencil_apply(int device, int nx, int ny, int nz, const int32_t* d_row_of,
    const uint8_t* d_clamped, const double* d_S, const double* d_x, double* d_y, void* stream)
{
  const int64_t n = int64_t(nx) * ny * nz;
  if (nx < 2 || ny < 2 || nz < 2 || !d_row_of || !d_clamped || !d_S || !d_x || !d_y) return FCG_ERR_ARG;
  if (!fcg_use_device(device)) return fcg_device_error();
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(fcg::box_stencil_kernel, dim3(fcg::blocks_for(n, fcg::kBlock)), dim3(fcg::kBlock), 0, s,
      nx, ny, nz, d_row_of, d_clamped, d_S, d_x, d_y);
  return hipGetLastError() == hipSuccess ? FCG_OK : fcg_device_error();
}

}  // extern "C"
