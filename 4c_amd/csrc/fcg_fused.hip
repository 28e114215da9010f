// fcg_fused.hip -- fused hex8 element evaluation + global assembly for structured (GridGenerator)
// lattices: each workgroup owns a 4 x 4 column of row nodes over a z-segment of node planes and
// sweeps the element layers bottom to top.
//
// Per element layer ez (between node planes ez and ez+1):
//   1. the 5 x 5 elements touching the tile's node columns (owned tile + one halo layer on the
//      low x/y sides) are evaluated, 8 lanes per element (fcg_hex8_element.hpp);
//   2. every lane adds its pair blocks K_ab / K_ab^T and f_a into LDS row images of the two node
//      planes -- in four colour phases (ex & 1, ey & 1) so that no two elements of a phase share
//      a node: plain read-add-write, fixed order, bitwise reproducible, no atomics;
//   3. node plane ez is now complete (its rows receive contributions only from layers ez-1 and
//      ez): its 3 CSR rows per node are written once, coalesced (81 contiguous columns for an
//      interior node), then the plane buffer is recycled for plane ez+2.
// HBM traffic is therefore K and r written once plus X, u, connectivity read ~1.6 times
// (halo recompute), instead of the general path's per-incidence scratch round trip.
//
// Reference semantics kept: SparseMatrix::assemble's owned-rows-only sum (4C_linalg_sparsematrix.cpp:474)
// and its column positions (resolved per node row into nbr_pos by fcg_create), Vector assemble
// (4C_linalg_utils_sparse_algebra_assemble.cpp:72-92), element evaluation as in
// 4C_solid_3D_ele_calc.cpp:110-240.
#include <hip/hip_runtime.h>

#include "fcg_hex8_element.hpp"
#include "fcg_internal.hpp"

namespace fcg {

namespace {

constexpr int TX = 4, TY = 4;             // node columns per tile
constexpr int EXN = TX + 1, EYN = TY + 1;  // element columns per layer
constexpr int NSLOT = EXN * EYN;           // 25 elements per layer
constexpr int NCOL = TX * TY;              // 16 node columns
constexpr int ROWIMG = 27 * 9;             // 27 neighbour blocks of 3x3

// hex8 node offsets in 4C node order (4C_io_gridgenerator.cpp:371-379)
__constant__ int c_ox[8] = {0, 1, 1, 0, 0, 1, 1, 0};
__constant__ int c_oy[8] = {0, 0, 1, 1, 0, 0, 1, 1};
__constant__ int c_oz[8] = {0, 0, 0, 0, 1, 1, 1, 1};

struct FusedArgs {
  const int32_t* ele_nodes;
  const double* node_x;
  const int32_t* node_dof_col;
  const double* u_col;
  const int32_t* elem_at;
  const int32_t* rownode_at;
  const uint16_t* nbr_pos;
  const int32_t* rownode_row0;
  const int64_t* rowptr;
  const double* tables;
  double* K;
  double* fint;
  int32_t* err;
  StVK mat;
  int32_t tiles_x, tiles_y, seg_planes;
  int32_t I0, J0, K0, NI, NJ, NK;
  int32_t EX0, EY0, EZ0, EX, EY, EZ;
};

template <int KIN>
struct FusedShared {
  H8Slot<KIN> slot[NSLOT];
  double row[2][NCOL][ROWIMG];
  double frow[2][NCOL][3];
  int64_t rbase[2][NCOL];  // rowptr of the node's first DOF row
  int32_t rowlen[2][NCOL];
  int32_t rn[2][NCOL];     // row node id of column c in plane buffer, -1 = not ours
  int32_t row0[2][NCOL];
  double dN[8][8][3];
  double dNn[8][8][3];
  double w8[8];
  int bad[32];
};

template <int KIN, bool WANT_K, bool OVERWRITE>
__global__ __launch_bounds__(256) void fused_h8_kernel(FusedArgs A)
{
  __shared__ FusedShared<KIN> sh;
  const int tid = threadIdx.x;
  const int s = tid >> 3;  // element slot
  const int j = tid & 7;   // lane in element group
  const int tile = blockIdx.x;
  const int tx = tile % A.tiles_x;
  const int ty = (tile / A.tiles_x) % A.tiles_y;
  const int tz = tile / (A.tiles_x * A.tiles_y);
  const int i0 = A.I0 + TX * tx, j0 = A.J0 + TY * ty;
  const int kz0 = A.K0 + A.seg_planes * tz;
  const int kz1 = min(kz0 + A.seg_planes, A.K0 + A.NK);

  for (int v = tid; v < 192; v += 256)
  {
    (&sh.dN[0][0][0])[v] = A.tables[v];
    (&sh.dNn[0][0][0])[v] = A.tables[192 + v];
  }
  if (tid < 8) sh.w8[tid] = A.tables[384 + tid];
  for (int v = tid; v < 2 * NCOL * ROWIMG; v += 256) (&sh.row[0][0][0])[v] = 0.0;
  if (tid < 2 * NCOL * 3) (&sh.frow[0][0][0])[tid] = 0.0;

  // element slot geometry (fixed over the sweep)
  const int sx = s % EXN, sy = s / EXN;
  const int ex = i0 - 1 + sx, ey = j0 - 1 + sy;
  const int colour = (ex & 1) | ((ey & 1) << 1);
  const bool slot_used = s < NSLOT;
  const int ox = c_ox[j], oy = c_oy[j], oz = c_oz[j];
  // the node column of this lane's node a = j (for accumulation), or -1 if outside the tile
  const int ca_x = ex + ox - i0, ca_y = ey + oy - j0;
  const int col_a = (ca_x >= 0 && ca_x < TX && ca_y >= 0 && ca_y < TY) ? ca_x + TX * ca_y : -1;
  int lo = 0;  // plane buffer holding the lower node plane of the current layer

  for (int ez = kz0 - 1; ez < kz1; ++ez)
  {
    // plane bookkeeping: buffers lo (plane ez) and 1-lo (plane ez+1)
    if (tid < 2 * NCOL)
    {
      const int pl = tid / NCOL, c = tid % NCOL;
      const int k = ez + pl;
      const int i = i0 + c % TX, jj = j0 + c / TX;
      int r = -1;
      if (k >= kz0 && k < kz1 && i < A.I0 + A.NI && jj < A.J0 + A.NJ)
        r = A.rownode_at[(int64_t(k - A.K0) * A.NJ + (jj - A.J0)) * A.NI + (i - A.I0)];
      const int b = pl == 0 ? lo : 1 - lo;
      sh.rn[b][c] = r;
      if (r >= 0)
      {
        const int32_t r0 = A.rownode_row0[r];
        sh.row0[b][c] = r0;
        sh.rbase[b][c] = A.rowptr[r0];
        sh.rowlen[b][c] = int32_t(A.rowptr[r0 + 1] - A.rowptr[r0]);
      }
    }
    // element of this slot
    int e = -1;
    if (slot_used && ex >= A.EX0 && ex < A.EX0 + A.EX && ey >= A.EY0 && ey < A.EY0 + A.EY &&
        ez >= A.EZ0 && ez < A.EZ0 + A.EZ)
      e = A.elem_at[(int64_t(ez - A.EZ0) * A.EY + (ey - A.EY0)) * A.EX + (ex - A.EX0)];
    H8Slot<KIN>& es = sh.slot[slot_used ? s : 0];  // unused slots never touch it (e < 0)
    if (e >= 0)
    {
      const int node = A.ele_nodes[int64_t(e) * 8 + j];
      const int dof = A.node_dof_col[node];
#pragma unroll
      for (int d = 0; d < 3; ++d)
      {
        es.X[j][d] = A.node_x[3 * int64_t(node) + d];
        es.U[j][d] = A.u_col[dof + d];
      }
    }
    if (j == 0) sh.bad[s] = 0;
    __syncthreads();
    if (e >= 0)
    {
      const int b = h8_stage_a<KIN>(j, es, sh.dN, sh.dNn, sh.w8[j], A.mat);
      if (b) atomicMax(&sh.bad[s], b);
    }
    __syncthreads();
    double K[5][9], f[3];
    const bool ok = e >= 0 && sh.bad[s] == 0;
    if (ok) h8_stage_b<KIN>(j, es, A.mat, WANT_K, K, f);
    if (e >= 0 && j == 0 && sh.bad[s])
    {
      atomicMax(&A.err[0], sh.bad[s]);
      atomicMin(&A.err[1], e);
    }
    // accumulate into the plane row images, one colour at a time
    const int buf_a = oz == 0 ? lo : 1 - lo;
    const bool own_a = ok && col_a >= 0 && sh.rn[buf_a][col_a] >= 0;
#pragma unroll 1
    for (int c = 0; c < 4; ++c)
    {
      if (ok && colour == c)
      {
        if (own_a)
        {
          double* fr = sh.frow[buf_a][col_a];
          fr[0] += f[0];
          fr[1] += f[1];
          fr[2] += f[2];
        }
        if (WANT_K)
        {
          const int npair = h8_npair(j);
#pragma unroll
          for (int p = 0; p < 5; ++p)
          {
            if (p >= npair) break;
            const int b = (j + p) & 7;
            const int dx = c_ox[b] - ox, dy = c_oy[b] - oy, dz = c_oz[b] - oz;
            if (own_a)
            {
              double* blk = sh.row[buf_a][col_a] + 9 * ((dz + 1) * 9 + (dy + 1) * 3 + (dx + 1));
#pragma unroll
              for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int q = 0; q < 3; ++q) blk[3 * r + q] += K[p][r + 3 * q];
            }
            if (p > 0)
            {
              const int cb_x = ca_x + dx, cb_y = ca_y + dy;
              if (cb_x >= 0 && cb_x < TX && cb_y >= 0 && cb_y < TY)
              {
                const int col_b = cb_x + TX * cb_y;
                const int buf_b = c_oz[b] == 0 ? lo : 1 - lo;
                if (sh.rn[buf_b][col_b] >= 0)
                {
                  double* blk = sh.row[buf_b][col_b] + 9 * ((1 - dz) * 9 + (1 - dy) * 3 + (1 - dx));
#pragma unroll
                  for (int r = 0; r < 3; ++r)
#pragma unroll
                    for (int q = 0; q < 3; ++q) blk[3 * r + q] += K[p][q + 3 * r];
                }
              }
            }
          }
        }
      }
      __syncthreads();
    }
    // node plane ez is complete: write its rows once, then recycle the buffer
    if (ez >= kz0)
    {
      if (WANT_K)
      {
        for (int v = tid; v < NCOL * ROWIMG; v += 256)
        {
          const int c = v / ROWIMG;
          const int rem = v - ROWIMG * c;
          const int r = rem / 81;
          const int rem2 = rem - 81 * r;
          const int t = rem2 / 3;
          const int q = rem2 - 3 * t;
          const int node = sh.rn[lo][c];
          if (node < 0) continue;
          const uint16_t pos = A.nbr_pos[int64_t(node) * 27 + t];
          if (pos == 0xFFFF) continue;
          double* dst = A.K + sh.rbase[lo][c] + int64_t(r) * sh.rowlen[lo][c] + pos + q;
          const double val = sh.row[lo][c][9 * t + 3 * r + q];
          if (OVERWRITE)
            *dst = val;
          else
            *dst += val;
        }
      }
      if (tid < NCOL * 3)
      {
        const int c = tid / 3, r = tid - 3 * (tid / 3);
        const int node = sh.rn[lo][c];
        if (node >= 0)
        {
          double* dst = A.fint + sh.row0[lo][c] + r;
          if (OVERWRITE)
            *dst = sh.frow[lo][c][r];
          else
            *dst += sh.frow[lo][c][r];
        }
      }
    }
    __syncthreads();
    for (int v = tid; v < NCOL * ROWIMG; v += 256) (&sh.row[lo][0][0])[v] = 0.0;
    if (tid < NCOL * 3) (&sh.frow[lo][0][0])[tid] = 0.0;
    lo = 1 - lo;
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_fused_h8(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream)
{
  const int64_t ntiles = int64_t(m.tiles_x) * m.tiles_y * m.tiles_z;
  if (ntiles == 0) return hipSuccess;
  FusedArgs a;
  a.ele_nodes = m.ele_nodes;
  a.node_x = m.node_x;
  a.node_dof_col = m.node_dof_col;
  a.u_col = d_u_col;
  a.elem_at = m.elem_at;
  a.rownode_at = m.rownode_at;
  a.nbr_pos = m.nbr_pos;
  a.rownode_row0 = m.rownode_row0;
  a.rowptr = m.rowptr;
  a.tables = m.tables;
  a.K = d_K;
  a.fint = d_fint;
  a.err = m.err;
  a.mat = StVK{m.lambda, m.mu, m.cdiag};
  a.tiles_x = m.tiles_x;
  a.tiles_y = m.tiles_y;
  a.seg_planes = m.seg_planes;
  a.I0 = m.I0; a.J0 = m.J0; a.K0 = m.K0; a.NI = m.NI; a.NJ = m.NJ; a.NK = m.NK;
  a.EX0 = m.EX0; a.EY0 = m.EY0; a.EZ0 = m.EZ0; a.EX = m.EX; a.EY = m.EY; a.EZ = m.EZ;
  const dim3 grid{static_cast<unsigned>(ntiles), 1, 1};
  const dim3 block{256, 1, 1};
#define FCG_FUSED(KIN)                                                                             \
  if (want_k && overwrite)                                                                         \
    hipLaunchKernelGGL((fused_h8_kernel<KIN, true, true>), grid, block, 0, stream, a);             \
  else if (want_k)                                                                                 \
    hipLaunchKernelGGL((fused_h8_kernel<KIN, true, false>), grid, block, 0, stream, a);            \
  else if (overwrite)                                                                              \
    hipLaunchKernelGGL((fused_h8_kernel<KIN, false, true>), grid, block, 0, stream, a);            \
  else                                                                                             \
    hipLaunchKernelGGL((fused_h8_kernel<KIN, false, false>), grid, block, 0, stream, a);
  if (m.kinem == 0)
  {
    FCG_FUSED(0)
  }
  else
  {
    FCG_FUSED(1)
  }
#undef FCG_FUSED
  return hipGetLastError();
}

}  // namespace fcg
