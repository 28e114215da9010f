// fcg_gather.hip -- hex8 element evaluation + assembly for unstructured meshes (FCG_PATH_GATHER):
// one wavefront per owned row node, no scratch, no atomics.
//
// The plan (fcg_create) lists, per owned row node A, "records" of up to 8 column elements holding
// A (its incidences, in element order), and keeps every element's node coordinates and DOF column
// LIDs contiguous (ele_x, ele_dof).  A wavefront walks a contiguous range of records; per record
// (lane = slot j x {element node | Gauss point} q):
//   1. lane (j, q): the trilinear coefficients c_q = sum_n sigma_q(n) x_n of the slot's element
//      (x = 1/8 sum_k c_k {1, xi, eta, zeta, xi eta, eta zeta, xi zeta, xi eta zeta}), so that a
//      Jacobian costs 27 FMA instead of the 72 of dN . X;
//   2. lane (j, g): J, J^-1, fac at Gauss point g (4C_solid_3D_ele_calc_lib.hpp:380-448), the nodal
//      det J > 0 check at corner g (calc_lib.hpp:475-496, same coefficients at xi = +-1), N_XYZ of
//      the 8 nodes; TotLag also F (hex8: from current coordinates, calc_lib.hpp:579-595, here as
//      J_cur J^-1), E, StVK S (4C_mat_stvenantkirchhoff.cpp:169-177) and the Gauss point's part of
//      f_A = sum_g fac F S N_XYZ_A (calc_lib.hpp:851-860);
//   3. lane (j, b): the 3 x 3 block K_ab of A's local node a with element node b over the Gauss
//      points,
//        linear  K_ab = sum_g fac [lambda a b^T + mu b a^T + mu (a.b) I]
//        TotLag  K_ab = sum_g fac [lambda (Fa)(Fb)^T + mu (Fb)(Fa)^T + mu (a.b) F F^T + (a.S.b) I]
//      (= B_a^T C B_b + K_geo of calc_lib.hpp:872-927 for the isotropic C of fill_cmat); linear
//      f_A part K_ab u_b (f_int = K u exactly);
//   4. the 64 blocks are summed per target entry of A's three CSR rows: lane v takes row entries
//      v, v+64, ... and adds the blocks aimed at that column triple in slot (= element) order, from a
//      per-record table fcg_create built from the positions of SparseMatrix::assemble's stride
//      fast path (4C_linalg_sparsematrix.cpp:497-543): per triple, the element node of each slot
//      that lands there (or none).  A node with one record
//      (<= 8 elements) writes its rows straight from there as one contiguous, coalesced run; a node
//      with more records sums them in an LDS image first.  Fixed summation order: bitwise
//      reproducible.
// Loads are software-pipelined: while record i computes, record i+1's element data and record i+2's
// slot lists are in flight.  An element is visited once per row node it holds, but only the blocks of
// that row (1/8 of its matrix) are formed there; only stages 1-2 (the Jacobians) repeat.
// Workgroups (one wave each) map to XCDs by blockIdx % 8; each XCD takes a contiguous range of row
// nodes, so the elements that neighbouring nodes share are re-read from the XCD's L2.
#include <hip/hip_runtime.h>

#include "fcg_hex8_element.hpp"
#include "fcg_internal.hpp"

namespace fcg {

namespace {

constexpr int kMaxRow = 81;  // hex8 node rows: 27 neighbour triples (fcg_create's limit)

// LDS of one wave.  The regions are reused across the stages of a record (one wave per workgroup:
// its LDS accesses are processed in program order, no barrier between a region's last read and
// the next write):
//   xa: X (and x_cur) in stage 1 -> per-Gauss-point data in stages 2-3
//   nb: N_XYZ in stages 2-3 -> the 64 blocks in stage 4
// Strides are chosen so that every access pattern of the stages is free of bank conflicts within
// each 32-lane group (ds_read_b64 / ds_write_b64, bank = (address / 4) mod 64): per slot 24 or 200
// doubles, per Gauss point 3 or 25, per node 3.
template <int KIN>
struct GatherShared {
  static constexpr int kNs = KIN ? 2 : 1;
  static constexpr int kGp = KIN ? 25 : 3;    // per (slot, GP): fac F a | fac S a | F | F F^T | fac a
  static constexpr int kGpSlot = KIN ? 200 : 24;
  union {
    double X[kNs][8][24];            // [x | x_cur][slot][3 node + d]
    double GP[8][kGpSlot];           // [slot][kGp g + k]
  } xa;
  double C[kNs][8][24];              // trilinear coefficients [x | x_cur][slot][3 k + d]
  union {
    double NX[8][200];               // N_XYZ [slot][25 g + 3 node + d]
    double blk[64][9];               // lane (slot, b): K_ab (column-major)
  } nb;
  double row[3 * kMaxRow];           // image of the node's rows (nodes with > 8 elements)
  double gp[8][4];                   // Gauss point coordinates | weight
  uint32_t tmap[32];                 // triple t: element node b of slot s in nibble s, 8 = none
};

struct GatherArgs {
  int64_t n_rownodes;
  const int64_t* rec_ptr;    // [n_rownodes + 1] records of each row node
  const int32_t* rec_row0;   // [n_rec] first row LID of the record's node
  const int32_t* rec_meta;   // [n_rec] nslot | first << 4 | last << 5
  const int32_t* rec_ele;    // [n_rec][8] element (-1 = empty slot)
  const uint8_t* rec_a;      // [n_rec][8] local node of the row node in the slot's element
  const uint32_t* rec_tmap;  // [n_rec][32] per column triple of the rows: slot s's node in nibble s
  const double* ele_x;       // [n_ele][8][3]
  const int32_t* ele_dof;    // [n_ele][8] column LID of each node's first DOF
  const int64_t* rowptr;
  const double* u_col;
  const double* gp;          // Gauss points [8][4]: xi, eta, zeta, weight
  double* K;
  double* fint;
  int32_t* err;
  StVK mat;
};

// hex8 corner n in 4C order: parametric coordinate signs
__host__ __device__ constexpr double h8_sx(int n) { return ((n & 3) == 1 || (n & 3) == 2) ? 1.0 : -1.0; }
__host__ __device__ constexpr double h8_sy(int n) { return (n & 3) >= 2 ? 1.0 : -1.0; }
__host__ __device__ constexpr double h8_sz(int n) { return n >= 4 ? 1.0 : -1.0; }

// column-major Jacobian J[dir + 3 comp] = d x_comp / d xi_dir at (x, y, z) from the coefficients
__device__ inline void h8_jac(const double* c, double x, double y, double z, double* J)
{
  const double yz = y * z, xz = x * z, xy = x * y;
#pragma unroll
  for (int d = 0; d < 3; ++d)
  {
    J[0 + 3 * d] = 0.125 * (c[3 + d] + y * c[12 + d] + z * c[18 + d] + yz * c[21 + d]);
    J[1 + 3 * d] = 0.125 * (c[6 + d] + x * c[12 + d] + z * c[15 + d] + xz * c[21 + d]);
    J[2 + 3 * d] = 0.125 * (c[9 + d] + y * c[15 + d] + x * c[18 + d] + xy * c[21 + d]);
  }
}

__device__ inline double h8_det(const double* m)
{
  return m[0] * (m[4] * m[8] - m[5] * m[7]) + m[3] * (m[2] * m[7] - m[1] * m[8]) +
         m[6] * (m[1] * m[5] - m[2] * m[4]);
}

struct RecRegs {
  int32_t row0, meta, ele;  // ele, a: slot j's
  int32_t a;
  uint32_t tm;              // tmap word (lane & 31) of the record
};

template <int KIN, bool WANT_K, bool OVERWRITE>
__global__ __launch_bounds__(64, KIN ? 1 : 2) void gather_h8_kernel(GatherArgs A)
{
  __shared__ GatherShared<KIN> sh;
  const int lane = threadIdx.x;
  const int j = lane >> 3, q = lane & 7;  // slot, element node / Gauss point
  if (lane < 32) (&sh.gp[0][0])[lane] = A.gp[lane];
  // XCD-contiguous node ranges: workgroup b runs on XCD b % 8 (round-robin dispatch); within the
  // XCD's range every workgroup takes one contiguous block of row nodes
  const int64_t nwg = gridDim.x;
  const int xcd = int(blockIdx.x & 7u);
  const int64_t per_xcd = (nwg + 7 - xcd) / 8;
  const int64_t rank = blockIdx.x >> 3;
  const int64_t chunk = (A.n_rownodes + 7) / 8;
  const int64_t x0 = min(A.n_rownodes, int64_t(xcd) * chunk), x1 = min(A.n_rownodes, x0 + chunk);
  const int64_t sub = (x1 - x0 + per_xcd - 1) / per_xcd;
  const int64_t n0 = min(x1, x0 + rank * sub), n1 = min(x1, n0 + sub);
  const int64_t R0 = A.rec_ptr[n0], R1 = A.rec_ptr[n1];

  auto load_rec = [&](int64_t i) -> RecRegs {
    RecRegs r{0, 0, -1, 0, 0u};
    if (i < R1)
    {
      r.row0 = A.rec_row0[i];
      r.meta = A.rec_meta[i];
      r.ele = A.rec_ele[i * 8 + j];
      r.a = A.rec_a[i * 8 + j];
      r.tm = A.rec_tmap[i * 32 + (lane & 31)];
    }
    return r;
  };
  // element data of node q of slot j
  auto load_x = [&](const RecRegs& r, double* x, int32_t& dof) {
    if (r.ele >= 0)
    {
      const double* p = A.ele_x + (int64_t(r.ele) * 8 + q) * 3;
      x[0] = p[0];
      x[1] = p[1];
      x[2] = p[2];
      dof = A.ele_dof[int64_t(r.ele) * 8 + q];
    }
    else
    {
      x[0] = x[1] = x[2] = 0.0;
      dof = -1;
    }
  };
  // sign pattern of coefficient q over the nodes: bit n set = -x_n
  const bool ux = q == 1 || q == 4 || q == 6 || q == 7;
  const bool uy = q == 2 || q == 4 || q == 5 || q == 7;
  const bool uz = q == 3 || q == 5 || q == 6 || q == 7;
  uint32_t negmask = 0;
#pragma unroll
  for (int n = 0; n < 8; ++n)
  {
    const bool neg = (ux && h8_sx(n) < 0) ^ (uy && h8_sy(n) < 0) ^ (uz && h8_sz(n) < 0);
    negmask |= uint32_t(neg) << n;
  }

  RecRegs cur = load_rec(R0), nxt = load_rec(R0 + 1);
  double xc[3];
  int32_t dofc;
  load_x(cur, xc, dofc);
  double fA0 = 0.0, fA1 = 0.0, fA2 = 0.0;
  __syncthreads();
  const double gx = sh.gp[q][0], gy = sh.gp[q][1], gz = sh.gp[q][2], gw = sh.gp[q][3];
  for (int64_t i = R0; i < R1; ++i)
  {
    // in flight while this record computes: its displacements, the next record's element data,
    // the record after that
    double uc[3] = {0.0, 0.0, 0.0};
    if (dofc >= 0)
    {
      uc[0] = A.u_col[dofc];
      uc[1] = A.u_col[dofc + 1];
      uc[2] = A.u_col[dofc + 2];
    }
    double xn[3];
    int32_t dofn;
    load_x(nxt, xn, dofn);
    const RecRegs nn = load_rec(i + 2);

    const bool first = (cur.meta >> 4) & 1, last = (cur.meta >> 5) & 1;
    const bool single = first && last;
    const int64_t base = A.rowptr[cur.row0];
    const int len = int(A.rowptr[cur.row0 + 1] - base);
    if (first)
    {
      fA0 = fA1 = fA2 = 0.0;
      if (!single)
        for (int v = lane; v < 3 * len; v += 64) sh.row[v] = 0.0;
    }
    const int32_t e = cur.ele;
    const int a = cur.a;
    sh.xa.X[0][j][3 * q + 0] = xc[0];
    sh.xa.X[0][j][3 * q + 1] = xc[1];
    sh.xa.X[0][j][3 * q + 2] = xc[2];
    if (KIN == 1)
    {
      sh.xa.X[KIN][j][3 * q + 0] = xc[0] + uc[0];
      sh.xa.X[KIN][j][3 * q + 1] = xc[1] + uc[1];
      sh.xa.X[KIN][j][3 * q + 2] = xc[2] + uc[2];
    }
    if (lane < 32) sh.tmap[lane] = cur.tm;
    __syncthreads();
    // 1. trilinear coefficient q of slot j
    if (e >= 0)
    {
#pragma unroll
      for (int s = 0; s < (KIN ? 2 : 1); ++s)
      {
        double c0 = 0.0, c1 = 0.0, c2 = 0.0;
#pragma unroll
        for (int n = 0; n < 8; ++n)
        {
          const double sg = (negmask >> n) & 1u ? -1.0 : 1.0;
          c0 += sg * sh.xa.X[s][j][3 * n + 0];
          c1 += sg * sh.xa.X[s][j][3 * n + 1];
          c2 += sg * sh.xa.X[s][j][3 * n + 2];
        }
        sh.C[s][j][3 * q + 0] = c0;
        sh.C[s][j][3 * q + 1] = c1;
        sh.C[s][j][3 * q + 2] = c2;
      }
    }
    __syncthreads();
    // 2. Gauss point q of slot j
    double fp0 = 0.0, fp1 = 0.0, fp2 = 0.0;
    if (e >= 0)
    {
      int bad = 0;
      double J[9];
      // nodal check at corner q (det J(corner) has the sign of the edge-vector determinant)
      h8_jac(sh.C[0][j], ((q & 3) == 1 || (q & 3) == 2) ? 1.0 : -1.0, (q & 3) >= 2 ? 1.0 : -1.0,
          q >= 4 ? 1.0 : -1.0, J);
      const double detn = h8_det(J);
      if (detn == 0.0) bad = 2;
      else if (!(detn > 0)) bad = 1;
      h8_jac(sh.C[0][j], gx, gy, gz, J);
      const double det = h8_invert3x3(J);
      if (det == 0.0) bad = 2;
      const double fac = det * gw;
      // dN_n/dxi = sx (1 + sy eta)(1 + sz zeta) / 8, ...
      const double xp = 1.0 + gx, xm = 1.0 - gx, yp = 1.0 + gy, ym = 1.0 - gy, zp = 1.0 + gz,
                   zm = 1.0 - gz;
      double na[3] = {0.0, 0.0, 0.0};
#pragma unroll
      for (int n = 0; n < 8; ++n)
      {
        const double fx = h8_sx(n) > 0 ? xp : xm, fy = h8_sy(n) > 0 ? yp : ym, fz = h8_sz(n) > 0 ? zp : zm;
        const double d0 = 0.125 * h8_sx(n) * (fy * fz);
        const double d1 = 0.125 * h8_sy(n) * (fx * fz);
        const double d2 = 0.125 * h8_sz(n) * (fx * fy);
        const double n0 = J[0] * d0 + J[3] * d1 + J[6] * d2;
        const double n1 = J[1] * d0 + J[4] * d1 + J[7] * d2;
        const double n2 = J[2] * d0 + J[5] * d1 + J[8] * d2;
        sh.nb.NX[j][25 * q + 3 * n + 0] = n0;
        sh.nb.NX[j][25 * q + 3 * n + 1] = n1;
        sh.nb.NX[j][25 * q + 3 * n + 2] = n2;
      }
      // N_XYZ_a back from the lane's own stores (in order within the wave)
      na[0] = sh.nb.NX[j][25 * q + 3 * a + 0];
      na[1] = sh.nb.NX[j][25 * q + 3 * a + 1];
      na[2] = sh.nb.NX[j][25 * q + 3 * a + 2];
      double* P = &sh.xa.GP[j][GatherShared<KIN>::kGp * q];
      if (KIN == 0)
      {
        P[0] = fac * na[0];
        P[1] = fac * na[1];
        P[2] = fac * na[2];
      }
      else
      {
        // F = J_cur J^-1 (column-major F[i + 3 j] = d x_i / d X_j)
        double Jc[9];
        h8_jac(sh.C[KIN][j], gx, gy, gz, Jc);
        double F[9];
#pragma unroll
        for (int ii = 0; ii < 3; ++ii)
#pragma unroll
          for (int jj = 0; jj < 3; ++jj)
            F[ii + 3 * jj] = Jc[0 + 3 * ii] * J[jj + 0] + Jc[1 + 3 * ii] * J[jj + 3] + Jc[2 + 3 * ii] * J[jj + 6];
        if (h8_det(F) == 0.0) bad = 2;
        const double C0 = F[0] * F[0] + F[1] * F[1] + F[2] * F[2];
        const double C4 = F[3] * F[3] + F[4] * F[4] + F[5] * F[5];
        const double C8 = F[6] * F[6] + F[7] * F[7] + F[8] * F[8];
        const double C3 = F[0] * F[3] + F[1] * F[4] + F[2] * F[5];
        const double C7 = F[3] * F[6] + F[4] * F[7] + F[5] * F[8];
        const double C2 = F[6] * F[0] + F[7] * F[1] + F[8] * F[2];
        const double E0 = 0.5 * (C0 - 1.0), E1 = 0.5 * (C4 - 1.0), E2 = 0.5 * (C8 - 1.0);
        const StVK& m = A.mat;
        const double S0 = m.cdiag * E0 + m.lambda * E1 + m.lambda * E2;
        const double S1 = m.lambda * E0 + m.cdiag * E1 + m.lambda * E2;
        const double S2 = m.lambda * E0 + m.lambda * E1 + m.cdiag * E2;
        const double S3 = m.mu * C3, S4 = m.mu * C7, S5 = m.mu * C2;
        const double sa0 = S0 * na[0] + S3 * na[1] + S5 * na[2];
        const double sa1 = S3 * na[0] + S1 * na[1] + S4 * na[2];
        const double sa2 = S5 * na[0] + S4 * na[1] + S2 * na[2];
        // f_A part: fac F S N_XYZ_A
        fp0 = fac * (F[0] * sa0 + F[3] * sa1 + F[6] * sa2);
        fp1 = fac * (F[1] * sa0 + F[4] * sa1 + F[7] * sa2);
        fp2 = fac * (F[2] * sa0 + F[5] * sa1 + F[8] * sa2);
        // fac F a | fac S a | F | F F^T
        P[0] = fac * (F[0] * na[0] + F[3] * na[1] + F[6] * na[2]);
        P[1] = fac * (F[1] * na[0] + F[4] * na[1] + F[7] * na[2]);
        P[2] = fac * (F[2] * na[0] + F[5] * na[1] + F[8] * na[2]);
        P[3] = fac * sa0;
        P[4] = fac * sa1;
        P[5] = fac * sa2;
#pragma unroll
        for (int k = 0; k < 9; ++k) P[6 + k] = F[k];
        P[15] = F[0] * F[0] + F[3] * F[3] + F[6] * F[6];
        P[16] = F[1] * F[1] + F[4] * F[4] + F[7] * F[7];
        P[17] = F[2] * F[2] + F[5] * F[5] + F[8] * F[8];
        P[18] = F[0] * F[1] + F[3] * F[4] + F[6] * F[7];
        P[19] = F[1] * F[2] + F[4] * F[5] + F[7] * F[8];
        P[20] = F[2] * F[0] + F[5] * F[3] + F[8] * F[6];
        P[21] = fac * na[0];
        P[22] = fac * na[1];
        P[23] = fac * na[2];
      }
      if (bad)
      {
        atomicMax(&A.err[0], bad);
        atomicMin(&A.err[1], e);
      }
    }
    __syncthreads();
    // 3. block (a, b = q) of slot j
    double Kb[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) Kb[k] = 0.0;
    if (e >= 0 && (WANT_K || KIN == 0))
    {
      double G[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      double H[KIN ? 6 : 1], geo = 0.0;
      if (KIN == 1)
#pragma unroll
        for (int k = 0; k < 6; ++k) H[k] = 0.0;
#pragma unroll 4
      for (int g = 0; g < 8; ++g)
      {
        const double* B = &sh.nb.NX[j][25 * g + 3 * q];
        const double b0 = B[0], b1 = B[1], b2 = B[2];
        const double* P = &sh.xa.GP[j][GatherShared<KIN>::kGp * g];
        if (KIN == 0)
        {
          const double fa0 = P[0], fa1 = P[1], fa2 = P[2];
          G[0] += fa0 * b0; G[1] += fa0 * b1; G[2] += fa0 * b2;
          G[3] += fa1 * b0; G[4] += fa1 * b1; G[5] += fa1 * b2;
          G[6] += fa2 * b0; G[7] += fa2 * b1; G[8] += fa2 * b2;
        }
        else
        {
          const double fpa0 = P[0], fpa1 = P[1], fpa2 = P[2];
          const double pb0 = P[6] * b0 + P[9] * b1 + P[12] * b2;
          const double pb1 = P[7] * b0 + P[10] * b1 + P[13] * b2;
          const double pb2 = P[8] * b0 + P[11] * b1 + P[14] * b2;
          G[0] += fpa0 * pb0; G[1] += fpa0 * pb1; G[2] += fpa0 * pb2;
          G[3] += fpa1 * pb0; G[4] += fpa1 * pb1; G[5] += fpa1 * pb2;
          G[6] += fpa2 * pb0; G[7] += fpa2 * pb1; G[8] += fpa2 * pb2;
          const double t = P[21] * b0 + P[22] * b1 + P[23] * b2;
#pragma unroll
          for (int k = 0; k < 6; ++k) H[k] += t * P[15 + k];
          geo += P[3] * b0 + P[4] * b1 + P[5] * b2;
        }
      }
      // G[3 r + c] = sum_g fac (.)_r (.)_c -> K_ab[r + 3 c] = lambda G_rc + mu G_cr (+ I terms)
      const double lam = A.mat.lambda, mu = A.mat.mu;
#pragma unroll
      for (int rr = 0; rr < 3; ++rr)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) Kb[rr + 3 * cc] = lam * G[3 * rr + cc] + mu * G[3 * cc + rr];
      if (KIN == 0)
      {
        const double tr = mu * (G[0] + G[4] + G[8]);
        Kb[0] += tr;
        Kb[4] += tr;
        Kb[8] += tr;
        // f_A part: K_ab u_b
        fp0 = Kb[0] * uc[0] + Kb[3] * uc[1] + Kb[6] * uc[2];
        fp1 = Kb[1] * uc[0] + Kb[4] * uc[1] + Kb[7] * uc[2];
        fp2 = Kb[2] * uc[0] + Kb[5] * uc[1] + Kb[8] * uc[2];
      }
      else
      {
        Kb[0] += mu * H[0] + geo;
        Kb[4] += mu * H[1] + geo;
        Kb[8] += mu * H[2] + geo;
        Kb[1] += mu * H[3]; Kb[3] += mu * H[3];
        Kb[5] += mu * H[4]; Kb[7] += mu * H[4];
        Kb[2] += mu * H[5]; Kb[6] += mu * H[5];
      }
    }
    // the record's part of f_A: a fixed butterfly over the wave
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
    {
      fp0 += __shfl_xor(fp0, o);
      fp1 += __shfl_xor(fp1, o);
      fp2 += __shfl_xor(fp2, o);
    }
    fA0 += fp0;
    fA1 += fp1;
    fA2 += fp2;
    // 4. sum the blocks per row entry in slot order
    if (WANT_K)
    {
      __syncthreads();  // NX -> blk
#pragma unroll
      for (int k = 0; k < 9; ++k) sh.nb.blk[lane][k] = Kb[k];
      __syncthreads();
      double* dst = A.K + base;
      // lane (triple t, half h): entries c = 2 e + h (column-major in the 3 x 3 block) of the
      // triple's block, each summed over the slots in order
      const int t = lane >> 1, h = lane & 1;
      if (t < len / 3)
      {
        const uint32_t tm = sh.tmap[t];
        int off[8];
        bool ok[8];
#pragma unroll
        for (int sl = 0; sl < 8; ++sl)
        {
          const uint32_t b = (tm >> (4 * sl)) & 15u;
          ok[sl] = b < 8u;
          off[sl] = 9 * (8 * sl + int(b & 7u));
        }
        const double* blk = &sh.nb.blk[0][0];
#pragma unroll
        for (int e = 0; e < 5; ++e)
        {
          const int c = h ? 2 * e + 1 : 2 * e;
          if (c < 9)
          {
            double s = 0.0;
#pragma unroll
            for (int sl = 0; sl < 8; ++sl)
            {
              const double x = blk[off[sl] + c];
              s += ok[sl] ? x : 0.0;
            }
            const int rr = h ? (2 * e + 1) % 3 : (2 * e) % 3;
            const int cc = h ? (2 * e + 1) / 3 : (2 * e) / 3;
            const int v = rr * len + 3 * t + cc;
            if (single)
            {
              if (OVERWRITE)
                __builtin_nontemporal_store(s, dst + v);
              else
                dst[v] += s;
            }
            else
              sh.row[v] += s;
          }
        }
      }
      // after the node's last record its image leaves contiguously
      if (last && !single)
      {
        __syncthreads();
        for (int v = lane; v < 3 * len; v += 64)
        {
          if (OVERWRITE)
            __builtin_nontemporal_store(sh.row[v], dst + v);
          else
            dst[v] += sh.row[v];
        }
      }
    }
    if (last && lane == 0)
    {
      if (OVERWRITE)
      {
        A.fint[cur.row0] = fA0;
        A.fint[cur.row0 + 1] = fA1;
        A.fint[cur.row0 + 2] = fA2;
      }
      else
      {
        A.fint[cur.row0] += fA0;
        A.fint[cur.row0 + 1] += fA1;
        A.fint[cur.row0 + 2] += fA2;
      }
    }
    __syncthreads();
    cur = nxt;
    nxt = nn;
    xc[0] = xn[0];
    xc[1] = xn[1];
    xc[2] = xn[2];
    dofc = dofn;
  }
}

}  // namespace

hipError_t launch_gather_h8(const DeviceMesh& m, const double* d_u_col, bool want_k, bool overwrite,
    double* d_K, double* d_fint, hipStream_t stream)
{
  if (m.n_rownodes == 0) return hipSuccess;
  GatherArgs a{};
  a.n_rownodes = m.n_rownodes;
  a.rec_ptr = m.rec_ptr;
  a.rec_row0 = m.rec_row0;
  a.rec_meta = m.rec_meta;
  a.rec_ele = m.rec_ele;
  a.rec_a = m.rec_a;
  a.rec_tmap = m.rec_tmap;
  a.ele_x = m.ele_x;
  a.ele_dof = m.ele_dof;
  a.rowptr = m.rowptr;
  a.u_col = d_u_col;
  a.gp = m.tables;
  a.K = d_K;
  a.fint = d_fint;
  a.err = m.err;
  a.mat = StVK{m.lambda, m.mu, m.cdiag};
  // one-wave workgroups, a few per SIMD on every CU, a multiple of the 8 XCDs, each a contiguous
  // block of row nodes
  const int64_t want = int64_t(256) * (m.kinem ? 5 : 8);  // LDS-resident workgroups per CU
  const int64_t wg = std::max<int64_t>(8, std::min<int64_t>(want, (m.n_rownodes + 7) / 8 * 8));
  const dim3 grid{static_cast<unsigned>(wg), 1, 1};
  const dim3 block{64, 1, 1};
#define FCG_GATHER(KIN)                                                                            \
  if (want_k && overwrite)                                                                         \
    hipLaunchKernelGGL((gather_h8_kernel<KIN, true, true>), grid, block, 0, stream, a);            \
  else if (want_k)                                                                                 \
    hipLaunchKernelGGL((gather_h8_kernel<KIN, true, false>), grid, block, 0, stream, a);           \
  else if (overwrite)                                                                              \
    hipLaunchKernelGGL((gather_h8_kernel<KIN, false, true>), grid, block, 0, stream, a);           \
  else                                                                                             \
    hipLaunchKernelGGL((gather_h8_kernel<KIN, false, false>), grid, block, 0, stream, a);
  if (m.kinem == 0)
  {
    FCG_GATHER(0)
  }
  else
  {
    FCG_GATHER(1)
  }
#undef FCG_GATHER
  return hipGetLastError();
}

}  // namespace fcg
