// fcg_fused.hip -- fused hex8 element evaluation + global assembly for structured (GridGenerator)
// lattices: each workgroup owns a 4 x 4 column of row nodes over a z-segment of node planes and
// sweeps the element layers bottom to top.
//
// Per element layer ez (between node planes ez and ez+1):
//   1. the 5 x 5 elements touching the tile's node columns (owned tile + one halo layer on the
//      low x/y sides) are evaluated, 8 lanes per element (fcg_hex8_element.hpp); each element's
//      36 pair blocks and 8 nodal forces are left in its (by then dead) LDS slot;
//   2. owner-computes gather: every lane owns row-image entries (node column, plane, neighbour
//      block, component) of the two node planes and adds the 1, 2 or 4 element contributions of
//      this layer in a fixed element order -- no atomics, no colouring, bitwise reproducible;
//   3. node plane ez is now complete (its rows receive contributions only from layers ez-1 and
//      ez): its 3 CSR rows per node are written once, coalesced (81 contiguous columns for an
//      interior node), then the plane image is recycled for plane ez+2.
// Latency hiding at one workgroup per CU: the next layer's node coordinates/displacements and the
// row bookkeeping of plane ez+2 (one 1152-byte record per tile and plane) are loaded into
// registers while the current layer computes, and committed to LDS at the next layer boundary.
// HBM traffic is therefore K and r written once plus X, u read ~1.6 times (halo recompute) and
// ~37 bytes of plane bookkeeping per row node, instead of the general path's scratch round trip.
//
// Reference semantics kept: SparseMatrix::assemble's owned-rows-only sum (4C_linalg_sparsematrix.cpp:474)
// and its column positions (resolved per node row by fcg_create), Vector assemble
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
// plane record (uint32 words): row0[16] | rowlen[16] | rbase[16] (int64) | npos[16][27] (uint16)
constexpr int PR_ROW0 = 0, PR_LEN = 16, PR_BASE = 32, PR_NPOS = 64;

// hex8 node offsets in 4C node order (4C_io_gridgenerator.cpp:371-379) and the inverse map
__constant__ int c_ox[8] = {0, 1, 1, 0, 0, 1, 1, 0};
__constant__ int c_oy[8] = {0, 0, 1, 1, 0, 0, 1, 1};
__constant__ int c_oz[8] = {0, 0, 0, 0, 1, 1, 1, 1};
__device__ inline int local_node(int ox, int oy, int oz)
{
  return 4 * oz + (oy ? (ox ? 2 : 3) : (ox ? 1 : 0));
}

struct FusedArgs {
  const double* u_col;
  const double* lat_x;       // [LZ][LY][LX][3] node coordinates on the column-node lattice
  const int32_t* lat_dof;    // [LZ][LY][LX] column LID of the first DOF, -1 = no node
  const int32_t* elem_at;    // [EZ][EY][EX] column element or -1
  const uint32_t* plane_rec; // [tiles_y][tiles_x][NK][PLANE_REC_WORDS]
  const double* tables;
  double* K;
  double* fint;
  int32_t* err;
  unsigned long long* stamps;  // diagnostic phase timers (NULL = off, the production setting)
  StVK mat;
  int32_t tiles_x, tiles_y, seg_planes;
  int32_t I0, J0, K0, NI, NJ, NK;
  int32_t EX0, EY0, EZ0, EX, EY, EZ;  // element box; the node lattice box is EX+1 x EY+1 x EZ+1
};

// LDS slot of one element: stage A/B working set, then (aliased) the stage B results
template <int KIN>
struct FusedSlot {
  union {
    H8Slot<KIN> s;
    double Kp[8][5][9];  // lane a's pair blocks (a, (a+p)&7), column-major 3x3
  } u;
  double fe[8][3];
};

template <int KIN>
struct FusedShared {
  FusedSlot<KIN> slot[NSLOT];
  double row[2][NCOL][ROWIMG];
  double frow[2][NCOL][3];
  uint32_t prec[3][PLANE_REC_WORDS];  // ring of plane records, plane p -> prec[ring(p)]
  double dN[8][8][3];
  double dNn[8][8][3];
  double w8[8];
  int bad[32];
  int ok[NSLOT];
};

__device__ inline int ring(int p) { return (p % 3 + 3) % 3; }

// Diagnostic phase stamps: thread 0 of each workgroup adds the cycles of every phase (including
// the barrier wait that ends it) into A.stamps[phase]; off (uniform branch, no s_memtime) when
// A.stamps is NULL.
#define FCG_STAMP(i)                                                                               \
  if (A.stamps && tid == 0)                                                                        \
  {                                                                                                \
    const unsigned long long now = __builtin_amdgcn_s_memtime();                                  \
    st_acc[i] += now - st_last;                                                                    \
    st_last = now;                                                                                 \
  }

template <int KIN, bool WANT_K, bool OVERWRITE, int ACC>
__global__ __launch_bounds__(256) void fused_h8_kernel(FusedArgs A)
{
  __shared__ FusedShared<KIN> sh;
  const int tid = threadIdx.x;
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long st_last = A.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
  const int s = tid >> 3;  // element slot
  const int j = tid & 7;   // lane in element group
  const int tile = blockIdx.x;
  const int tx = tile % A.tiles_x;
  const int ty = (tile / A.tiles_x) % A.tiles_y;
  const int tz = tile / (A.tiles_x * A.tiles_y);
  const int i0 = A.I0 + TX * tx, j0 = A.J0 + TY * ty;
  const int kz0 = A.K0 + A.seg_planes * tz;
  const int kz1 = min(kz0 + A.seg_planes, A.K0 + A.NK);
  const uint32_t* prec_tile = A.plane_rec + (int64_t(ty) * A.tiles_x + tx) * A.NK * PLANE_REC_WORDS;
  const int64_t LX = A.EX + 1, LY = A.EY + 1;

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
  const bool slot_used = s < NSLOT;
  const int ox = c_ox[j], oy = c_oy[j], oz = c_oz[j];
  const bool exy_in = slot_used && ex >= A.EX0 && ex < A.EX0 + A.EX && ey >= A.EY0 && ey < A.EY0 + A.EY;
  const int64_t lat_xy = exy_in ? (int64_t(ey - A.EY0 + oy) * LX + (ex - A.EX0 + ox)) : 0;
  // colour-phase accumulation (ACC 0): element colour and the tile column of this lane's node a
  const int colour = (ex & 1) | ((ey & 1) << 1);
  const int ca_x = ex + ox - i0, ca_y = ey + oy - j0;
  const int col_a = (ca_x >= 0 && ca_x < TX && ca_y >= 0 && ca_y < TY) ? ca_x + TX * ca_y : -1;

  // --- loaders (issue only; values land in registers)
  auto load_elem = [&](int lz, int& e, double* X, int& dof) {
    e = -1;
    dof = -1;
    if (exy_in && lz >= A.EZ0 && lz < A.EZ0 + A.EZ)
    {
      e = A.elem_at[(int64_t(lz - A.EZ0) * A.EY + (ey - A.EY0)) * A.EX + (ex - A.EX0)];
      const int64_t li = int64_t(lz - A.EZ0 + oz) * LX * LY + lat_xy;
      dof = A.lat_dof[li];
#pragma unroll
      for (int d = 0; d < 3; ++d) X[d] = A.lat_x[3 * li + d];
    }
  };
  auto load_rec = [&](int p, uint32_t* w) {
    const bool in = p >= kz0 && p < kz1;
    const uint32_t* src = prec_tile + int64_t(in ? p - A.K0 : 0) * PLANE_REC_WORDS;
#pragma unroll
    for (int k = 0; k < 2; ++k)
    {
      const int v = tid + 256 * k;
      if (v < PLANE_REC_WORDS) w[k] = in ? src[v] : (v < PR_LEN ? 0xFFFFFFFFu : 0u);
    }
  };
  auto store_rec = [&](int p, const uint32_t* w) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
    {
      const int v = tid + 256 * k;
      if (v < PLANE_REC_WORDS) sh.prec[ring(p)][v] = w[k];
    }
  };

  // --- prologue: plane records of kz0-1 (empty) and kz0, elements of layer kz0-1
  {
    uint32_t w[2];
    load_rec(kz0 - 1, w);
    store_rec(kz0 - 1, w);
    load_rec(kz0, w);
    store_rec(kz0, w);
  }
  int e_cur, dof_cur;
  double X_cur[3] = {0, 0, 0}, U_cur[3] = {0, 0, 0};
  load_elem(kz0 - 1, e_cur, X_cur, dof_cur);
  if (e_cur >= 0)
#pragma unroll
    for (int d = 0; d < 3; ++d) U_cur[d] = A.u_col[dof_cur + d];
  int lo = 0;  // row-image buffer of the lower node plane

  for (int ez = kz0 - 1; ez < kz1; ++ez)
  {
    // 1. commit this layer's element data
    FusedSlot<KIN>& fs = sh.slot[slot_used ? s : 0];  // unused slots never touch it (e < 0)
    H8Slot<KIN>& es = fs.u.s;
    const int e = e_cur;
    if (e >= 0)
    {
#pragma unroll
      for (int d = 0; d < 3; ++d)
      {
        es.X[j][d] = X_cur[d];
        es.U[j][d] = U_cur[d];
      }
    }
    if (j == 0) sh.bad[s] = 0;
    __syncthreads();
    FCG_STAMP(0);
    // 2. prefetch: next layer's elements and plane ez+2's record
    int e_nxt, dof_nxt;
    double X_nxt[3] = {0, 0, 0}, U_nxt[3] = {0, 0, 0};
    load_elem(ez + 1, e_nxt, X_nxt, dof_nxt);
    uint32_t rec_nxt[2];
    load_rec(ez + 2, rec_nxt);
    // 3. Gauss-point stage
    if (e >= 0)
    {
      const int b = h8_stage_a<KIN>(j, es, sh.dN, sh.dNn, sh.w8[j], A.mat);
      if (b) atomicMax(&sh.bad[s], b);
    }
    __syncthreads();
    FCG_STAMP(1);
    if (e_nxt >= 0)
#pragma unroll
      for (int d = 0; d < 3; ++d) U_nxt[d] = A.u_col[dof_nxt + d];
    // 4./5. node-row stage and accumulation into the plane row images
    if (ACC == 0)
    {
      double K[5][9], f[3];
      const bool ok = e >= 0 && sh.bad[s] == 0;
      if (ok) h8_stage_b<KIN>(j, es, A.mat, WANT_K, K, f);
      if (e >= 0 && j == 0 && sh.bad[s])
      {
        atomicMax(&A.err[0], sh.bad[s]);
        atomicMin(&A.err[1], e);
      }
      FCG_STAMP(2);
      const uint32_t* rec_lo = sh.prec[ring(ez)];
      const uint32_t* rec_hi = sh.prec[ring(ez + 1)];
      const int buf_a = oz == 0 ? lo : 1 - lo;
      const uint32_t* rec_a = oz == 0 ? rec_lo : rec_hi;
      const bool own_a = ok && col_a >= 0 && int32_t(rec_a[PR_ROW0 + col_a]) >= 0;
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
                  const uint32_t* rec_b = c_oz[b] == 0 ? rec_lo : rec_hi;
                  if (int32_t(rec_b[PR_ROW0 + col_b]) >= 0)
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
    }
    else
    {
    // 4. node-row stage; results into the slot (aliases the dead stage-A data of this element)
    {
      const bool ok = e >= 0 && sh.bad[s] == 0;
      if (ok)
      {
        double K[5][9], f[3];
        h8_stage_b<KIN>(j, es, A.mat, WANT_K, K, f);
        // all 8 lanes of this element are in one wavefront and finished reading the slot
        __builtin_amdgcn_wave_barrier();
        fs.fe[j][0] = f[0];
        fs.fe[j][1] = f[1];
        fs.fe[j][2] = f[2];
        if (WANT_K)
        {
#pragma unroll
          for (int p = 0; p < 5; ++p)
#pragma unroll
            for (int k = 0; k < 9; ++k) fs.u.Kp[j][p][k] = K[p][k];
        }
      }
      if (slot_used && j == 0) sh.ok[s] = ok ? 1 : 0;
      if (e >= 0 && j == 0 && sh.bad[s])
      {
        atomicMax(&A.err[0], sh.bad[s]);
        atomicMin(&A.err[1], e);
      }
    }
      __syncthreads();
      FCG_STAMP(2);
    // 5. owner-computes gather into the row images of planes ez (p = 0) and ez+1 (p = 1)
    {
      const uint32_t* rec_pl[2] = {sh.prec[ring(ez)], sh.prec[ring(ez + 1)]};
      const int buf_pl[2] = {lo, 1 - lo};
      // residual entries: 2 planes x 16 columns x 3
      if (tid < 2 * NCOL * 3)
      {
        const int p = tid / (NCOL * 3);
        const int rem = tid - p * NCOL * 3;
        const int c = rem / 3, r = rem - 3 * (rem / 3);
        if (int32_t(rec_pl[p][PR_ROW0 + c]) >= 0)
        {
          const int cx = c % TX, cy = c / TX;
          double acc = 0.0;
#pragma unroll
          for (int k = 0; k < 4; ++k)
          {
            const int bx = k & 1, by = k >> 1;  // element (cx-1+bx, cy-1+by) in tile columns
            const int sl = (cx + bx) + EXN * (cy + by);
            if (sh.ok[sl]) acc += sh.slot[sl].fe[local_node(1 - bx, 1 - by, p)][r];
          }
          sh.frow[buf_pl[p]][c][r] += acc;
        }
      }
      if (WANT_K)
      {
        // K entries: (p, c, t, k) with the neighbour in this layer's planes
        for (int v = tid; v < 2 * NCOL * ROWIMG; v += 256)
        {
          const int p = v / (NCOL * ROWIMG);
          const int rem = v - p * NCOL * ROWIMG;
          const int c = rem / ROWIMG;
          const int rem2 = rem - c * ROWIMG;
          const int t = rem2 / 9;
          const int kk = rem2 - 9 * t;
          const int dz = t / 9 - 1;
          const int pz = p + dz;
          if (pz < 0 || pz > 1) continue;
          if (int32_t(rec_pl[p][PR_ROW0 + c]) < 0) continue;
          const int dy = (t / 3) % 3 - 1, dx = t % 3 - 1;
          const int r = kk / 3, q = kk - 3 * (kk / 3);
          const int cx = c % TX, cy = c / TX;
          double acc = 0.0;
          // elements of the layer holding node (cx, cy) and its neighbour (cx+dx, cy+dy):
          // x offset bx in {0,1} relative to column cx-1 with both nodes inside
#pragma unroll
          for (int k = 0; k < 4; ++k)
          {
            const int bx = k & 1, by = k >> 1;
            // element x index (tile-relative, column cx-1+bx): node at local ox = 1-bx,
            // neighbour at ox + dx must be 0 or 1
            const int oxa = 1 - bx, oya = 1 - by;
            const int oxb = oxa + dx, oyb = oya + dy;
            if (oxb < 0 || oxb > 1 || oyb < 0 || oyb > 1) continue;
            const int sl = (cx + bx) + EXN * (cy + by);
            if (!sh.ok[sl]) continue;
            const int a = local_node(oxa, oya, p);
            const int b = local_node(oxb, oyb, pz);
            const int pp = (b - a) & 7;
            if (pp <= 3 || (pp == 4 && a < 4))
              acc += sh.slot[sl].u.Kp[a][pp][r + 3 * q];
            else
              acc += sh.slot[sl].u.Kp[b][(a - b) & 7][q + 3 * r];
          }
          sh.row[buf_pl[p]][c][9 * t + kk] += acc;
        }
      }
    }
    __syncthreads();
    }
    FCG_STAMP(3);
    // 6. node plane ez is complete: write its rows once and clear the image
    if (ez >= kz0)
    {
      const uint32_t* rec_lo = sh.prec[ring(ez)];
      const uint16_t* npos = reinterpret_cast<const uint16_t*>(rec_lo + PR_NPOS);
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
          double& img = sh.row[lo][c][9 * t + 3 * r + q];
          const double val = img;
          img = 0.0;
          if (int32_t(rec_lo[PR_ROW0 + c]) < 0) continue;
          const uint16_t pos = npos[27 * c + t];
          if (pos == 0xFFFF) continue;
          const int64_t base = int64_t(rec_lo[PR_BASE + 2 * c]) | (int64_t(rec_lo[PR_BASE + 2 * c + 1]) << 32);
          double* dst = A.K + base + int64_t(r) * int32_t(rec_lo[PR_LEN + c]) + pos + q;
          if (OVERWRITE)
            *dst = val;
          else
            *dst += val;
        }
      }
      if (tid < NCOL * 3)
      {
        const int c = tid / 3, r = tid - 3 * (tid / 3);
        const int32_t r0 = int32_t(rec_lo[PR_ROW0 + c]);
        const double val = sh.frow[lo][c][r];
        sh.frow[lo][c][r] = 0.0;
        if (r0 >= 0)
        {
          double* dst = A.fint + r0 + r;
          if (OVERWRITE)
            *dst = val;
          else
            *dst += val;
        }
      }
    }
    else
    {
      for (int v = tid; v < NCOL * ROWIMG; v += 256) (&sh.row[lo][0][0])[v] = 0.0;
      if (tid < NCOL * 3) (&sh.frow[lo][0][0])[tid] = 0.0;
    }
    // 7. commit plane ez+2's record (its ring slot held plane ez-1), roll registers
    store_rec(ez + 2, rec_nxt);
    e_cur = e_nxt;
    dof_cur = dof_nxt;
#pragma unroll
    for (int d = 0; d < 3; ++d)
    {
      X_cur[d] = X_nxt[d];
      U_cur[d] = U_nxt[d];
    }
    lo = 1 - lo;
    __syncthreads();
    FCG_STAMP(4);
  }
  if (A.stamps && tid == 0)
  {
    for (int i = 0; i < 5; ++i) atomicAdd(&A.stamps[i], st_acc[i]);
    atomicAdd(&A.stamps[5], 1ull);
  }
}

}  // namespace

hipError_t launch_fused_h8(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream)
{
  const int64_t ntiles = int64_t(m.tiles_x) * m.tiles_y * m.tiles_z;
  if (ntiles == 0) return hipSuccess;
  FusedArgs a;
  a.u_col = d_u_col;
  a.lat_x = m.lat_x;
  a.lat_dof = m.lat_dof;
  a.elem_at = m.elem_at;
  a.plane_rec = m.plane_rec;
  a.tables = m.tables;
  a.K = d_K;
  a.fint = d_fint;
  a.err = m.err;
  a.stamps = m.stamps;
  a.mat = StVK{m.lambda, m.mu, m.cdiag};
  a.tiles_x = m.tiles_x;
  a.tiles_y = m.tiles_y;
  a.seg_planes = m.seg_planes;
  a.I0 = m.I0; a.J0 = m.J0; a.K0 = m.K0; a.NI = m.NI; a.NJ = m.NJ; a.NK = m.NK;
  a.EX0 = m.EX0; a.EY0 = m.EY0; a.EZ0 = m.EZ0; a.EX = m.EX; a.EY = m.EY; a.EZ = m.EZ;
  const dim3 grid{static_cast<unsigned>(ntiles), 1, 1};
  const dim3 block{256, 1, 1};
#define FCG_FUSED3(KIN, ACC)                                                                       \
  if (want_k && overwrite)                                                                         \
    hipLaunchKernelGGL((fused_h8_kernel<KIN, true, true, ACC>), grid, block, 0, stream, a);        \
  else if (want_k)                                                                                 \
    hipLaunchKernelGGL((fused_h8_kernel<KIN, true, false, ACC>), grid, block, 0, stream, a);       \
  else if (overwrite)                                                                              \
    hipLaunchKernelGGL((fused_h8_kernel<KIN, false, true, ACC>), grid, block, 0, stream, a);       \
  else                                                                                             \
    hipLaunchKernelGGL((fused_h8_kernel<KIN, false, false, ACC>), grid, block, 0, stream, a);
#define FCG_FUSED(KIN)                                                                             \
  if (m.fused_acc == 0)                                                                            \
  {                                                                                                \
    FCG_FUSED3(KIN, 0)                                                                             \
  }                                                                                                \
  else                                                                                             \
  {                                                                                                \
    FCG_FUSED3(KIN, 1)                                                                             \
  }
  if (m.kinem == 0)
  {
    FCG_FUSED(0)
  }
  else
  {
    FCG_FUSED(1)
  }
#undef FCG_FUSED3
#undef FCG_FUSED
  return hipGetLastError();
}

}  // namespace fcg
