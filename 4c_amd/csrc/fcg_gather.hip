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

// LDS of one wave, one flat array with stage-dependent views (one wave per workgroup: its LDS
// accesses are processed in program order, so a region is reused without a barrier between its
// last read and the next write):
//   linear:  [X | GP] (192) | C (192) | [NX (1600) | blk (650) + row (243) at 656]
//   TotLag:  [X (384) + C (384) at 384 | GP (1728) | blk (650) + row (243) at 656]
// (TotLag forms its stage-3 terms from dN_b(xi_g) directly, with the Gauss point's J^-1 folded into
// per-point 3 x 3 factors, instead of keeping NX: 13 KB instead of 31 KB.)  A node with more records (MULTI) keeps its row image in its own array.
// Strides make every access pattern of the stages free of bank conflicts within each 32-lane group
// (ds_read_b64 / ds_write_b64, bank = (address / 4) mod 64): per slot 24 (X, C), 200 (NX), 24 or
// 216 (GP); per Gauss point 25 (NX), 3 or 26 (GP); per node 3; per block 10 (blk).
// TotLag's GP records and the blocks are 16-byte aligned, so that the compiler reads them as
// ds_read_b128 (4 LDS cycles per 16 bytes) instead of pairing two entries into a ds_read2_b64 (8
// cycles): renumbered 1M hex8 TotLag -4 %, linear -2.4 % (profiles/r06/r06_gather_lds_align_ab.txt).
// GP stride 26 / slot stride 216 keep the b128 reads (8 lanes of a slot broadcast, 4 slots per lane
// group at banks 0 / 48 / 32 / 16) and the stage-2 b128 stores (one slot's 8 points) conflict-free.
template <int KIN, bool MULTI>
struct GatherShared {
  static constexpr int kNs = KIN ? 2 : 1;
#ifdef FCG_GATHER_TL_ODD
  static constexpr int kGp = KIN ? 25 : 3;  // A/B probe: the round-5 strides (ds_read2_b64 pairs)
  static constexpr int kGpSlot = KIN ? 200 : 24;
#else
  static constexpr int kGp = KIN ? 26 : 3;  // per (slot, GP): fac a | TotLag: fac F a, J^-T fac S a, F J^-T, F F^T, J^-T fac a
  static constexpr int kGpSlot = KIN ? 216 : 24;
#endif
  static constexpr int kX = 0, kC = KIN ? 384 : 192, kGpOff = 0;
  static constexpr int kNX = KIN ? 0 : 384, kBlk = KIN ? 0 : 384, kRow = kBlk + 600;
  static constexpr int kSize = KIN ? 8 * kGpSlot : 384 + 1600;
  alignas(16) double u[kSize];
  double row_m[MULTI ? 3 * kMaxRow : 1];  // MULTI: the row image lives across records
  alignas(16) double gp[8][4];            // Gauss point coordinates | weight
  uint32_t tmap[32];                      // triple t: element node b of slot s in nibble s, 8 = none
  __device__ double* X(int s, int j) { return u + kX + 192 * s + 24 * j; }
  // C one double in (TotLag): the Jacobian reads c[3..23] then start 16-byte aligned and pair as
  // ds_read_b128 instead of ds_read2_b64 (c[0], never read, moves into the pad; FCG_GATHER_C0 = A/B)
#ifdef FCG_GATHER_C0
  static constexpr int kCo = 0;
#else
  static constexpr int kCo = KIN ? 1 : 0;
#endif
  __device__ double* C(int s, int j) { return u + kC + 192 * s + 24 * j + kCo; }
  __device__ double* GP(int j, int g) { return u + kGpOff + kGpSlot * j + kGp * g; }
  __device__ double* NX(int j, int g) { return u + kNX + 200 * j + 25 * g; }  // linear only
#ifdef FCG_GATHER_BLK9
  static constexpr int kBs = 9;  // A/B probe: the round-5 block stride (ds_read2_b64 pairs)
#else
  static constexpr int kBs = 10;  // block stride: entry pairs (2p, 2p + 1) 16-byte aligned
#endif
  __device__ double* blk(int l) { return u + kBlk + kBs * l; }
  __device__ double* row() { return MULTI ? row_m : u + kRow + (kBs - 9) * 56; }
};

struct GatherArgs {
  int64_t n_single;          // records [0, n_single): nodes with <= 8 elements, one record each
  int64_t n_multi;           // nodes with more elements; their records follow
  const int64_t* multi_ptr;  // [n_multi + 1] record range of each such node
  const int32_t* rec_row0;   // [n_rec] first row LID of the record's node
  const int32_t* rec_meta;   // [n_rec] nslot | first << 4 | last << 5 | row length << 8
  const int64_t* rec_base;   // [n_rec] CSR offset of the node's first row
  const int32_t* rec_ele;    // [n_rec][8] element (-1 = empty slot)
  const uint8_t* rec_a;      // [n_rec][8] local node of the row node in the slot's element
  const uint32_t* rec_tmap;  // [n_rec][32] per column triple of the rows: slot s's node in nibble s
  const int32_t* ele_orig;   // [n_ele] column element index of each storage slot (error report)
  const double* ele_x;       // [n_ele][8][3]
  const double* ele_gp;      // [n_ele][8][10] per Gauss point (gather_gp_kernel, once per context)
  const int32_t* ele_dof;    // [n_ele][8] column LID of each node's first DOF
  const double* u_col;
  const double* gp;          // Gauss points [8][4]: xi, eta, zeta, weight
  double* K;
  double* fint;
  int32_t* err;
  double* dummy;             // [3] target of the stores of a row without columns
  StVK mat;
};

// hex8 corner n in 4C order: parametric coordinate signs
__host__ __device__ constexpr double h8_sx(int n) { return ((n & 3) == 1 || (n & 3) == 2) ? 1.0 : -1.0; }
__host__ __device__ constexpr double h8_sy(int n) { return (n & 3) >= 2 ? 1.0 : -1.0; }
__host__ __device__ constexpr double h8_sz(int n) { return n >= 4 ? 1.0 : -1.0; }

// column-major Jacobian J[dir + 3 comp] = d x_comp / d xi_dir at (x, y, z) from the coefficients
// (stored as c_k / 8)
__device__ inline void h8_jac(const double* c, double x, double y, double z, double* J)
{
  const double yz = y * z, xz = x * z, xy = x * y;
#pragma unroll
  for (int d = 0; d < 3; ++d)
  {
    J[0 + 3 * d] = c[3 + d] + y * c[12 + d] + z * c[18 + d] + yz * c[21 + d];
    J[1 + 3 * d] = c[6 + d] + x * c[12 + d] + z * c[15 + d] + xz * c[21 + d];
    J[2 + 3 * d] = c[9 + d] + y * c[15 + d] + x * c[18 + d] + xy * c[21 + d];
  }
}

__device__ inline double h8_det(const double* m)
{
  return m[0] * (m[4] * m[8] - m[5] * m[7]) + m[3] * (m[2] * m[7] - m[1] * m[8]) +
         m[6] * (m[1] * m[5] - m[2] * m[4]);
}

struct RecRegs {
  int32_t row0, meta;       // first row LID; nslot | first << 4 | last << 5 | row length << 8
  int64_t base;             // CSR offset of the first row
  int32_t ele, a;           // slot j's element (-1 = empty) and local node of the row node
  uint32_t tm;              // tmap word (lane & 31) of the record
};

// sum over the 16 lanes of each DPP row (every lane of the row gets it): xor 1, xor 2, rotate 4, 8
template <int CTRL>
__device__ inline double dpp_mov(double v)
{
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ inline double row_sum(double v)
{
  v += dpp_mov<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x124>(v);  // row_ror 4
  v += dpp_mov<0x128>(v);  // row_ror 8
  return v;
}
// wave sum in a fixed order (rows 0 + 16 + 32 + 48), uniform
__device__ inline double wave_sum(double v)
{
  v = row_sum(v);
  double r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    r[k] = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 16 * k),
        __builtin_amdgcn_readlane(__double2loint(v), 16 * k));
  return ((r[0] + r[1]) + r[2]) + r[3];
}

template <int KIN, bool WANT_K, bool OVERWRITE, bool MULTI>
__global__ __launch_bounds__(64, 2) void gather_h8_kernel(GatherArgs A)
{
  using Sh = GatherShared<KIN, MULTI>;
  __shared__ Sh sh;
  const int lane = threadIdx.x;
  const int j = lane >> 3, q = lane & 7;  // slot, element node / Gauss point
  if (lane < 32) (&sh.gp[0][0])[lane] = A.gp[lane];
  // XCD-contiguous ranges: workgroup b runs on XCD b % 8 (round-robin dispatch); within the XCD's
  // range every workgroup takes one contiguous block -- of records (one per node) for nodes with
  // <= 8 elements, of nodes for the others (MULTI)
  const int64_t nwork = MULTI ? A.n_multi : A.n_single;
  const int64_t nwg = gridDim.x;
  const int xcd = int(blockIdx.x & 7u);
  const int64_t per_xcd = (nwg + 7 - xcd) / 8;
  const int64_t rank = blockIdx.x >> 3;
  const int64_t chunk = (nwork + 7) / 8;
  const int64_t x0 = min(nwork, int64_t(xcd) * chunk), x1 = min(nwork, x0 + chunk);
  // nodes with <= 8 elements: the XCD's workgroups take its records round robin (workgroup k
  // records x0 + k, x0 + k + per_xcd, ...), so that at any time they work on neighbouring row nodes
  // (Morton order) and share the elements' data in the XCD's L2 -- with a contiguous block each,
  // 256 workgroups streamed 256 separate regions through 4 MB of L2 and re-fetched every element's
  // Gauss-point factors for each of its row nodes.  Nodes with more records (MULTI) keep one
  // contiguous block of nodes each.
  const int64_t sub = (x1 - x0 + per_xcd - 1) / per_xcd;
#ifdef FCG_GATHER_CONTIGUOUS
  constexpr bool RR = false;  // A/B probe: one contiguous block of records per workgroup
#else
  constexpr bool RR = !MULTI;
#endif
  const int64_t n0 = RR ? x0 + rank : min(x1, x0 + rank * sub);
  const int64_t n1 = RR ? x1 : min(x1, n0 + sub);
  const int64_t step = RR ? per_xcd : 1;
  const int64_t R0 = MULTI ? A.multi_ptr[n0] : n0, R1 = MULTI ? A.multi_ptr[n1] : n1;
  if (R0 >= R1) return;

  // Loads are branch-free (indices clamped into range; an empty slot reads element 0, a record
  // past the range re-reads the last one) and every record issues the same stores, so that the
  // wait counts stay static: record i's words arrive three records ahead, its element data two,
  // its displacements one, and no wait covers the stores of the record before.
  auto load_rec = [&](int64_t i) -> RecRegs {
    const int64_t k = min(i, R1 - 1);  // past the end: re-reads a valid record, unused
    RecRegs r;
    r.row0 = A.rec_row0[k];
    r.meta = A.rec_meta[k];
    r.base = A.rec_base[k];
    r.ele = A.rec_ele[k * 8 + j];
    r.a = A.rec_a[k * 8 + j];
    r.tm = A.rec_tmap[k * 32 + (lane & 31)];
    return r;
  };
  // element data of node q of slot j (TotLag: its reference coordinates; linear: none) and its
  // DOF; the Gauss point q's geometric factors come one record ahead (load_g)
  auto load_x = [&](const RecRegs& r, double* x, int32_t& dof) {
    const int64_t el = max(r.ele, 0);
    if (KIN == 1)
    {
      const double* p = A.ele_x + (el * 8 + q) * 3;
      x[0] = p[0];
      x[1] = p[1];
      x[2] = p[2];
    }
    dof = A.ele_dof[el * 8 + q];
  };
  auto load_g = [&](const RecRegs& r, double* gv) {
    const int64_t el = max(r.ele, 0);
    const double2* p = reinterpret_cast<const double2*>(A.ele_gp + (el * 8 + q) * 10);
#pragma unroll
    for (int k = 0; k < 5; ++k)
    {
      const double2 v = p[k];
      gv[2 * k] = v.x;
      gv[2 * k + 1] = v.y;
    }
  };
  auto load_u = [&](int32_t dof, double* u) {
    u[0] = A.u_col[dof];
    u[1] = A.u_col[dof + 1];
    u[2] = A.u_col[dof + 2];
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

  RecRegs cur = load_rec(R0), nx1 = load_rec(R0 + step), nx2 = load_rec(R0 + 2 * step);
  double xc[3], xn1[3], uc[3], gc[10];
  int32_t dofc, dof1;
  load_x(cur, xc, dofc);
  load_x(nx1, xn1, dof1);
  load_u(dofc, uc);
  load_g(cur, gc);
  double fA0 = 0.0, fA1 = 0.0, fA2 = 0.0;
  int bad_code = 0, bad_ele = 0x7FFFFFFF;
  // the prologue's loads have landed before the loop: the loop header then carries only the
  // previous record's stores, and the waits inside stay at their static counts
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const double gx = sh.gp[q][0], gy = sh.gp[q][1], gz = sh.gp[q][2];
  // element node b = q: parametric signs (TotLag stage 3)
  const double bsx = h8_sx(q & 3), bsy = (q & 3) >= 2 ? 1.0 : -1.0, bsz = q >= 4 ? 1.0 : -1.0;
  const double bsx8 = 0.125 * bsx, bsy8 = 0.125 * bsy, bsz8 = 0.125 * bsz;
  for (int64_t i = R0; i < R1; i += step)
  {
    // in flight while this record computes: the next record's displacements, the element data of
    // the one after, the words of the third
    const RecRegs nx3 = load_rec(i + 3 * step);
    double xn2[3], u1[3], g1[10];
    int32_t dof2;
    load_x(nx2, xn2, dof2);
    load_u(dof1, u1);
    load_g(nx1, g1);

    const bool first = (cur.meta >> 4) & 1, last = (cur.meta >> 5) & 1;
    const int64_t base = cur.base;
    const int len = cur.meta >> 8;
    if (MULTI && first)
    {
      fA0 = fA1 = fA2 = 0.0;
      for (int v = lane; v < 3 * len; v += 64) sh.row()[v] = 0.0;
    }
    const int32_t e = cur.ele;
    const int a = cur.a;
    if (KIN == 1)
    {
      sh.X(1, j)[3 * q + 0] = xc[0] + uc[0];
      sh.X(1, j)[3 * q + 1] = xc[1] + uc[1];
      sh.X(1, j)[3 * q + 2] = xc[2] + uc[2];
    }
    if (lane < 32) sh.tmap[lane] = cur.tm;
    __syncthreads();
    // 1. trilinear coefficient q of slot j (TotLag: of the current coordinates; the reference
    // Jacobians come precomputed)
    if (KIN == 1 && e >= 0)
    {
#pragma unroll
      for (int s = 1; s < 2; ++s)
      {
        double c0 = 0.0, c1 = 0.0, c2 = 0.0;
#pragma unroll
        for (int n = 0; n < 8; ++n)
        {
          const double sg = (negmask >> n) & 1u ? -1.0 : 1.0;
          c0 += sg * sh.X(s, j)[3 * n + 0];
          c1 += sg * sh.X(s, j)[3 * n + 1];
          c2 += sg * sh.X(s, j)[3 * n + 2];
        }
        sh.C(s, j)[3 * q + 0] = 0.125 * c0;
        sh.C(s, j)[3 * q + 1] = 0.125 * c1;
        sh.C(s, j)[3 * q + 2] = 0.125 * c2;
      }
    }
    __syncthreads();
    // 2. Gauss point q of slot j
    double fp0 = 0.0, fp1 = 0.0, fp2 = 0.0;
    if (e >= 0)
    {
      int bad = 0;
      // the Gauss point's reference Jacobian, inverted (and the nodal det J check) once per
      // context by gather_gp_kernel: linear sqrt|fac| J^-1 | sign(fac), TotLag J^-1 | fac
      double J[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) J[k] = gc[k];
      double Jc[9];
      if (KIN == 1) h8_jac(sh.C(1, j), gx, gy, gz, Jc);  // before GP (aliasing C) is written
      const double fac = gc[9];
      // dN_n/dxi = sx (1 + sy eta)(1 + sz zeta) / 8, ...
      // the 12 distinct products (1 +- eta)(1 +- zeta) / 8, ...; the node's sign is a negation
      const double xp = 1.0 + gx, xm = 1.0 - gx, yp = 1.0 + gy, ym = 1.0 - gy, zp = 1.0 + gz,
                   zm = 1.0 - gz;
      const double hyp = 0.125 * yp, hym = 0.125 * ym, hxp = 0.125 * xp, hxm = 0.125 * xm;
      const double pyz[2][2] = {{hym * zm, hym * zp}, {hyp * zm, hyp * zp}};
      const double pxz[2][2] = {{hxm * zm, hxm * zp}, {hxp * zm, hxp * zp}};
      const double pxy[2][2] = {{hxm * ym, hxm * yp}, {hxp * ym, hxp * yp}};
      double na[3];
      if (KIN == 0)
      {
#pragma unroll
        for (int n = 0; n < 8; ++n)
        {
          const int ix = h8_sx(n) > 0, iy = h8_sy(n) > 0, iz = h8_sz(n) > 0;
          const double d0 = ix ? pyz[iy][iz] : -pyz[iy][iz];
          const double d1 = iy ? pxz[ix][iz] : -pxz[ix][iz];
          const double d2 = iz ? pxy[ix][iy] : -pxy[ix][iy];
          double* nx = sh.NX(j, q) + 3 * n;
          nx[0] = J[0] * d0 + J[3] * d1 + J[6] * d2;
          nx[1] = J[1] * d0 + J[4] * d1 + J[7] * d2;
          nx[2] = J[2] * d0 + J[5] * d1 + J[8] * d2;
        }
        // N_XYZ_a back from the lane's own stores (in order within the wave)
        na[0] = sh.NX(j, q)[3 * a + 0];
        na[1] = sh.NX(j, q)[3 * a + 1];
        na[2] = sh.NX(j, q)[3 * a + 2];
      }
      else
      {
        // N_XYZ of node a only (stage 3 rebuilds the others from J^-1); a is a runtime index, so
        // the factors are selected, not looked up (an indexed private array lives in scratch)
        const bool ix = ((a & 3) == 1 || (a & 3) == 2), iy = (a & 3) >= 2, iz = a >= 4;
        const double ex = ix ? xp : xm, ey = iy ? yp : ym, ez = iz ? zp : zm;
        const double d0 = (ix ? 0.125 : -0.125) * ey * ez;
        const double d1 = (iy ? 0.125 : -0.125) * ex * ez;
        const double d2 = (iz ? 0.125 : -0.125) * ex * ey;
        na[0] = J[0] * d0 + J[3] * d1 + J[6] * d2;
        na[1] = J[1] * d0 + J[4] * d1 + J[7] * d2;
        na[2] = J[2] * d0 + J[5] * d1 + J[8] * d2;
      }
      double* P = sh.GP(j, q);
      if (KIN == 0)
      {
        // NX holds sqrt|fac| N_XYZ: sign(fac) sqrt|fac| N_XYZ_a . sqrt|fac| N_XYZ_b = fac a b^T
        P[0] = fac * na[0];
        P[1] = fac * na[1];
        P[2] = fac * na[2];
      }
      else
      {
        // F = J_cur J^-1 (column-major F[i + 3 j] = d x_i / d X_j)
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
        // stage 3 needs, for N_XYZ_b = J^-T dN_b (b_j = sum_dir J[j + 3 dir] d_dir):
        //   fac F a | J^-T-folded fac S a | Q = F J^-T (Q[i + 3 dir]) | F F^T | J^-T-folded fac a
        const double fs0 = fac * sa0, fs1 = fac * sa1, fs2 = fac * sa2;
        const double fa0 = fac * na[0], fa1 = fac * na[1], fa2 = fac * na[2];
        P[0] = F[0] * fa0 + F[3] * fa1 + F[6] * fa2;
        P[1] = F[1] * fa0 + F[4] * fa1 + F[7] * fa2;
        P[2] = F[2] * fa0 + F[5] * fa1 + F[8] * fa2;
#pragma unroll
        for (int dir = 0; dir < 3; ++dir)
        {
          const double j0 = J[0 + 3 * dir], j1 = J[1 + 3 * dir], j2 = J[2 + 3 * dir];
          P[3 + dir] = fs0 * j0 + fs1 * j1 + fs2 * j2;
          P[21 + dir] = fa0 * j0 + fa1 * j1 + fa2 * j2;
#pragma unroll
          for (int ii = 0; ii < 3; ++ii) P[6 + ii + 3 * dir] = F[ii] * j0 + F[ii + 3] * j1 + F[ii + 6] * j2;
        }
        P[15] = F[0] * F[0] + F[3] * F[3] + F[6] * F[6];
        P[16] = F[1] * F[1] + F[4] * F[4] + F[7] * F[7];
        P[17] = F[2] * F[2] + F[5] * F[5] + F[8] * F[8];
        P[18] = F[0] * F[1] + F[3] * F[4] + F[6] * F[7];
        P[19] = F[1] * F[2] + F[4] * F[5] + F[7] * F[8];
        P[20] = F[2] * F[0] + F[5] * F[3] + F[8] * F[6];
      }
      if (bad)
      {
        bad_code = max(bad_code, bad);
        bad_ele = min(bad_ele, A.ele_orig[e]);  // the column element index (4C's loop order)
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
      // the 8 Gauss points fully unrolled (was 4: renumbered 1M box linear -1.8 %, TotLag -8 %, the
      // same two waves per SIMD and no spills; profiles/r06/r06_gather_g_unroll_ab.txt)
#ifndef FCG_GATHER_G_UNROLL
#define FCG_GATHER_G_UNROLL 8
#endif
#pragma unroll FCG_GATHER_G_UNROLL
      for (int g = 0; g < 8; ++g)
      {
        const double* P = sh.GP(j, g);
        if (KIN == 0)
        {
          const double* B = sh.NX(j, g) + 3 * q;
          const double b0 = B[0], b1 = B[1], b2 = B[2];
          const double fa0 = P[0], fa1 = P[1], fa2 = P[2];
          G[0] += fa0 * b0; G[1] += fa0 * b1; G[2] += fa0 * b2;
          G[3] += fa1 * b0; G[4] += fa1 * b1; G[5] += fa1 * b2;
          G[6] += fa2 * b0; G[7] += fa2 * b1; G[8] += fa2 * b2;
        }
        else
        {
          // dN_b(xi_g): dN_b/dxi = sx (1 + sy eta)(1 + sz zeta) / 8, ...; N_XYZ_b = J^-T dN_b
          // enters only through the folded factors: F N_XYZ_b = Q dN_b, a.b = (J^-1 fac a).dN_b
          const double fx = fma(bsx, sh.gp[g][0], 1.0), fy = fma(bsy, sh.gp[g][1], 1.0),
                       fz = fma(bsz, sh.gp[g][2], 1.0);
          const double d0 = (bsx8 * fy) * fz, d1 = (bsy8 * fx) * fz, d2 = (bsz8 * fx) * fy;
          const double fpa0 = P[0], fpa1 = P[1], fpa2 = P[2];
          const double pb0 = P[6] * d0 + P[9] * d1 + P[12] * d2;
          const double pb1 = P[7] * d0 + P[10] * d1 + P[13] * d2;
          const double pb2 = P[8] * d0 + P[11] * d1 + P[14] * d2;
          G[0] += fpa0 * pb0; G[1] += fpa0 * pb1; G[2] += fpa0 * pb2;
          G[3] += fpa1 * pb0; G[4] += fpa1 * pb1; G[5] += fpa1 * pb2;
          G[6] += fpa2 * pb0; G[7] += fpa2 * pb1; G[8] += fpa2 * pb2;
          const double t = P[21] * d0 + P[22] * d1 + P[23] * d2;
#pragma unroll
          for (int k = 0; k < 6; ++k) H[k] += t * P[15 + k];
          geo += P[3] * d0 + P[4] * d1 + P[5] * d2;
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
    // the record's part of f_A: a fixed-order reduction over the wave
    const double r0 = wave_sum(fp0), r1 = wave_sum(fp1), r2 = wave_sum(fp2);
    if (MULTI)
    {
      fA0 += r0;
      fA1 += r1;
      fA2 += r2;
    }
    else
    {
      fA0 = r0;
      fA1 = r1;
      fA2 = r2;
    }
    // 4. sum the blocks per row entry in slot order
    // a node whose rows hold no column (len 0) stores into a dummy triple instead of branching
    double* dst = len ? A.K + base : A.dummy;
    if (WANT_K)
    {
      __syncthreads();  // NX / GP -> blk
#pragma unroll
      for (int k = 0; k < 9; ++k) sh.blk(lane)[k] = Kb[k];
      if (lane < 9) sh.blk(64)[lane] = 0.0;
      __syncthreads();
      // lane (triple t, half h): entries c = 2 e + h (column-major in the 3 x 3 block) of the
      // triple's block, each summed over the slots in order into the LDS image of the rows (lanes
      // past the row's triples redo the last triple and the ninth entry stands in for the missing
      // tenth: the same value to the same address, no branch).
      const int ntrip = len / 3;
      const int t = max(0, min(lane >> 1, ntrip - 1)), h = lane & 1;
      const bool active = (lane >> 1) < ntrip;
      {
        const uint32_t tm = sh.tmap[t];
        int off[8];  // block of slot sl aimed at triple t, or the zero row
#pragma unroll
        for (int sl = 0; sl < 8; ++sl)
        {
          const uint32_t b = (tm >> (4 * sl)) & 15u;
          off[sl] = Sh::kBs * (b < 8u ? 8 * sl + int(b) : 64);
        }
        const double* blk = sh.blk(0);
#ifndef FCG_GATHER_BLK9
        // h = 0: entries 0, 1, 4, 5, 8; h = 1: entries 2, 3, 6, 7, 8 (both lanes write entry 8: the
        // same value to the same address).  Each pair (2p, 2p + 1) is one 16-byte LDS read per slot
        // instead of two entries 2 apart, which the compiler paired into a ds_read2_b64 (8 LDS cycles
        // per 16 bytes against 4 for a ds_read_b128)
        double xs[5];
#pragma unroll
        for (int p = 0; p < 2; ++p)
        {
          const int c0 = 4 * p + 2 * h;
          double2 v = *reinterpret_cast<const double2*>(blk + off[0] + c0);
          double x0 = v.x, x1 = v.y;
#pragma unroll
          for (int sl = 1; sl < 8; ++sl)
          {
            v = *reinterpret_cast<const double2*>(blk + off[sl] + c0);
            x0 += v.x;
            x1 += v.y;
          }
          xs[2 * p] = x0;
          xs[2 * p + 1] = x1;
        }
        {
          double x = blk[off[0] + 8];
#pragma unroll
          for (int sl = 1; sl < 8; ++sl) x += blk[off[sl] + 8];
          xs[4] = x;
        }
#endif
#pragma unroll
        for (int e5 = 0; e5 < 5; ++e5)
        {
#ifdef FCG_GATHER_BLK9
          const int c = h ? min(2 * e5 + 1, 7) : 2 * e5;  // h = 1: entries 1, 3, 5, 7, 7
          double x = blk[off[0] + c];
#pragma unroll
          for (int sl = 1; sl < 8; ++sl) x += blk[off[sl] + c];
#else
          const int c = e5 == 4 ? 8 : 4 * (e5 >> 1) + 2 * h + (e5 & 1);
          const double x = xs[e5];
#endif
          const int rr = c % 3, cc = c / 3;
          const int v = rr * len + 3 * t + cc;
          if (MULTI)
          {
            if (active && !(h && e5 == 4)) sh.row()[v] += x;
          }
          else
            sh.row()[v] = x;
        }
      }
      // one record per node: the rows leave as contiguous runs of 64 (OVERWRITE: four stores per
      // lane, lanes past the end repeating the last entry)
      if (!MULTI)
      {
        const int n3 = 3 * len;
#pragma unroll
        for (int k = 0; k < 4; ++k)
        {
          const int v = max(0, min(lane + 64 * k, n3 - 1));
          if (OVERWRITE)
            __builtin_nontemporal_store(sh.row()[v], dst + v);
          else if (lane + 64 * k < n3)
            dst[v] += sh.row()[v];
        }
      }
      // a node with more records: its image leaves after the last one
      if (MULTI && last)
      {
        __syncthreads();
        for (int v = lane; v < 3 * len; v += 64)
        {
          if (OVERWRITE)
            __builtin_nontemporal_store(sh.row()[v], dst + v);
          else
            dst[v] += sh.row()[v];
        }
      }
    }
    // f_A: lanes 0..2 (OVERWRITE without MULTI: every lane, lanes >= 2 all storing component 2)
    {
      const int comp = min(lane, 2);
      const double fv = comp == 0 ? fA0 : (comp == 1 ? fA1 : fA2);
      if (!MULTI && OVERWRITE)
        A.fint[cur.row0 + comp] = fv;
      else if ((!MULTI || last) && lane < 3)
      {
        if (OVERWRITE)
          A.fint[cur.row0 + comp] = fv;
        else
          A.fint[cur.row0 + comp] += fv;
      }
    }
    __syncthreads();
    cur = nx1;
    nx1 = nx2;
    nx2 = nx3;
#pragma unroll
    for (int k = 0; k < 3; ++k)
    {
      xc[k] = xn1[k];
      xn1[k] = xn2[k];
      uc[k] = u1[k];
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) gc[k] = g1[k];
    dofc = dof1;
    dof1 = dof2;
  }
  if (bad_code)
  {
    atomicMax(&A.err[0], bad_code);
    atomicMin(&A.err[1], bad_ele);
  }
}

// The Gauss points' geometric factors of every element, from its reference coordinates (fixed for
// the context's lifetime), one thread per (element, Gauss point): J at the point and its inverse
// (4C_solid_3D_ele_calc_lib.hpp:380-448), fac = det J w, the nodal det J > 0 check at corner g
// (calc_lib.hpp:475-496).  Linear kinematics store sqrt|fac| J^-1 and sign(fac) (N_XYZ then comes
// out scaled by sqrt|fac|), TotLag J^-1 and fac.  Failures go to err[0] (max code) / err[1] (min
// column element).
template <int KIN>
__global__ __launch_bounds__(256) void gather_gp_kernel(int64_t n_ele, const double* __restrict__ ele_x,
    const int32_t* __restrict__ ele_orig, const double* __restrict__ gp, double* ele_gp, int32_t* err)
{
  const int64_t t = int64_t(blockIdx.x) * 256 + threadIdx.x;
  const int64_t e = t >> 3;
  const int g = int(t & 7);
  if (e >= n_ele) return;
  double x[8][3];
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int d = 0; d < 3; ++d) x[n][d] = ele_x[e * 24 + 3 * n + d];
  auto jac = [&](double px, double py, double pz, double* J) {
    const H8dN dn = h8_dn_products(px, py, pz);
#pragma unroll
    for (int k = 0; k < 9; ++k) J[k] = 0.0;
#pragma unroll
    for (int n = 0; n < 8; ++n)
    {
      double d0, d1, d2;
      h8_dn(dn, n, d0, d1, d2);
#pragma unroll
      for (int d = 0; d < 3; ++d)
      {
        J[0 + 3 * d] += d0 * x[n][d];
        J[1 + 3 * d] += d1 * x[n][d];
        J[2 + 3 * d] += d2 * x[n][d];
      }
    }
  };
  int bad = 0;
  double J[9];
  jac(((g & 3) == 1 || (g & 3) == 2) ? 1.0 : -1.0, (g & 3) >= 2 ? 1.0 : -1.0, g >= 4 ? 1.0 : -1.0, J);
  const double detn = h8_det(J);
  if (detn == 0.0) bad = 2;
  else if (!(detn > 0)) bad = 1;
  jac(gp[4 * g], gp[4 * g + 1], gp[4 * g + 2], J);
  const double det = h8_invert3x3(J);
  if (det == 0.0) bad = 2;
  const double fac = det * gp[4 * g + 3];
  double* o = ele_gp + (e * 8 + g) * 10;
  if (KIN == 0)
  {
    const double sq = sqrt(fabs(fac));
#pragma unroll
    for (int k = 0; k < 9; ++k) o[k] = sq * J[k];
    o[9] = fac < 0.0 ? -1.0 : 1.0;
  }
  else
  {
#pragma unroll
    for (int k = 0; k < 9; ++k) o[k] = J[k];
    o[9] = fac;
  }
  if (bad)
  {
    atomicMax(&err[0], bad);
    atomicMin(&err[1], ele_orig[e]);
  }
}

__global__ void fold_err_kernel(int32_t* err, int code, int ele)
{
  atomicMax(&err[0], code);
  atomicMin(&err[1], ele);
}

}  // namespace

hipError_t gather_precompute(DeviceMesh& m, int64_t n_ele, hipStream_t stream)
{
  if (n_ele == 0) return hipSuccess;
  int32_t* d_err = nullptr;
  hipError_t e = hipMalloc(&d_err, 2 * sizeof(int32_t));
  if (e != hipSuccess) return e;
  const int32_t init[2] = {0, 0x7FFFFFFF};
  e = hipMemcpyAsync(d_err, init, sizeof(init), hipMemcpyHostToDevice, stream);
  const dim3 grid{static_cast<unsigned>((n_ele * 8 + 255) / 256), 1, 1}, block{256, 1, 1};
  if (e == hipSuccess)
  {
    if (m.kinem == 0)
      hipLaunchKernelGGL((gather_gp_kernel<0>), grid, block, 0, stream, n_ele, m.ele_x, m.ele_orig, m.tables, m.ele_gp, d_err);
    else
      hipLaunchKernelGGL((gather_gp_kernel<1>), grid, block, 0, stream, n_ele, m.ele_x, m.ele_orig, m.tables, m.ele_gp, d_err);
    e = hipGetLastError();
  }
  int32_t h[2] = {0, 0};
  if (e == hipSuccess) e = hipMemcpyAsync(h, d_err, sizeof(h), hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  (void)hipFree(d_err);
  m.gp_bad_code = h[0];
  m.gp_bad_ele = h[1];
  return e;
}

hipError_t launch_gather_h8(const DeviceMesh& m, const double* d_u_col, bool want_k, bool overwrite,
    double* d_K, double* d_fint, hipStream_t stream)
{
  // a nodal / Gauss-point Jacobian failure found when the geometric factors were made is reported
  // by every evaluate, as 4C's element throws on every call
  if (m.gp_bad_code) hipLaunchKernelGGL(fold_err_kernel, dim3(1), dim3(1), 0, stream, m.err, m.gp_bad_code, m.gp_bad_ele);
  GatherArgs a{};
  a.n_single = m.n_rec_single;
  a.n_multi = m.n_multi;
  a.multi_ptr = m.multi_ptr;
  a.rec_row0 = m.rec_row0;
  a.rec_meta = m.rec_meta;
  a.rec_base = m.rec_base;
  a.rec_ele = m.rec_ele;
  a.rec_a = m.rec_a;
  a.rec_tmap = m.rec_tmap;
  a.ele_orig = m.ele_orig;
  a.ele_x = m.ele_x;
  a.ele_gp = m.ele_gp;
  a.ele_dof = m.ele_dof;
  a.u_col = d_u_col;
  a.gp = m.tables;
  a.K = d_K;
  a.fint = d_fint;
  a.err = m.err;
  a.dummy = m.gather_dummy;
  a.mat = StVK{m.lambda, m.mu, m.cdiag};
  // one-wave workgroups, as many as the LDS keeps resident on every CU, a multiple of the 8 XCDs,
  // each a contiguous block of records / nodes
  // workgroups per CU: two waves per SIMD.  (Linear kinematics would fit nine by LDS and registers
  // since the Gauss-point factors are precomputed -- measured 10 % slower: more streams in L2.)
#ifndef FCG_GATHER_WPC_LINEAR
#define FCG_GATHER_WPC_LINEAR 8
#endif
  const int64_t want = int64_t(256) * (m.kinem == 0 ? FCG_GATHER_WPC_LINEAR : 8);
  const dim3 block{64, 1, 1};
  auto grid_of = [&](int64_t work) {
    return dim3{static_cast<unsigned>(std::max<int64_t>(8, std::min<int64_t>(want, (work + 7) / 8 * 8))), 1, 1};
  };
#define FCG_GATHER(KIN, MULTI, WORK)                                                               \
  if ((WORK) > 0)                                                                                  \
  {                                                                                                \
    const dim3 grid = grid_of(WORK);                                                               \
    if (want_k && overwrite)                                                                       \
      hipLaunchKernelGGL((gather_h8_kernel<KIN, true, true, MULTI>), grid, block, 0, stream, a);   \
    else if (want_k)                                                                               \
      hipLaunchKernelGGL((gather_h8_kernel<KIN, true, false, MULTI>), grid, block, 0, stream, a);  \
    else if (overwrite)                                                                            \
      hipLaunchKernelGGL((gather_h8_kernel<KIN, false, true, MULTI>), grid, block, 0, stream, a);  \
    else                                                                                           \
      hipLaunchKernelGGL((gather_h8_kernel<KIN, false, false, MULTI>), grid, block, 0, stream, a); \
  }
  if (m.kinem == 0)
  {
    FCG_GATHER(0, false, m.n_rec_single)
    FCG_GATHER(0, true, m.n_multi)
  }
  else
  {
    FCG_GATHER(1, false, m.n_rec_single)
    FCG_GATHER(1, true, m.n_multi)
  }
#undef FCG_GATHER
  return hipGetLastError();
}

}  // namespace fcg
