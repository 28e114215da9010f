// fcg_sweep.hip -- fused hex8 element evaluation + global assembly on structured (GridGenerator)
// lattices: the row-block sweep.
//
// A workgroup owns a 4 x 4 column of row nodes over a z-segment of node planes and sweeps the
// element layers bottom to top.  Per layer L (the elements between node planes L and L+1):
//   A. one lane per (element, Gauss point) of the 5 x 5 elements touching the tile's node
//      columns: J, J^-1, det J (and det J > 0 at node g), N_XYZ, strain or F, StVK stress
//      (4C_solid_3D_ele_calc_lib.hpp:380-496, 579-676, 682-799; 4C_mat_stvenantkirchhoff.cpp:169-177).
//      Into LDS go sqrt|fac| N_XYZ of the 8 nodes and the stress (with F for TotLag);
//   B. sixteen lanes per node column, four element visits each (fcg_visit_table.h): a lane sums
//      over the elements holding both nodes of its blocks (A, B) and all Gauss points
//        linear: G = sum fac a b^T,                 K_AB = lambda G + mu G^T + mu tr(G) I
//        TotLag: G = sum fac (Fa)(Fb)^T, H = sum fac (a.b) F F^T, geo = sum fac a.S.b,
//                K_AB = lambda G + mu G^T + mu H + geo I
//      (= B_a^T C B_b + K_geo of calc_lib.hpp:872-927 for the isotropic C of fill_cmat) and
//      writes the 3 x 3 block straight into its 3 CSR rows -- or keeps the lower-layer part of
//      an in-plane block (dz = 0) in registers until the next layer adds the upper part.
//      The residual rows f_A = sum fac F S N_XYZ_A (calc_lib.hpp:851-860) are summed the same way,
//      16 lanes per column.
// Every entry of an owned row is written exactly once, by one lane, in a fixed summation order:
// no atomics, no row image in LDS, bitwise reproducible.  Owned-rows-only assembly and column
// positions follow SparseMatrix::assemble (4C_linalg_sparsematrix.cpp:474-543, positions resolved
// per node row by fcg_create), the residual LinAlg::assemble (4C_linalg_utils_sparse_algebra_assemble.cpp:72-92).
//
// Linear kinematics: f_int = K u exactly (E = B u, f = sum fac B^T C B u), so the residual rows are
// summed from the finished blocks, f_A += K_AB u_B, and stage A needs neither strains nor stresses.
//
// Latency hiding: two workgroups per CU for linear kinematics (LDS 59 KB), one for TotLag
// (85 KB), plus, inside a workgroup, register prefetch of the next node plane (coordinates,
// displacements) and plane record while the current layer computes.
#include <hip/hip_runtime.h>

#include "fcg_hex8_element.hpp"
#include "fcg_internal.hpp"
#include "fcg_visit_table.h"

namespace fcg {

namespace {

constexpr int TX = 4, TY = 4;              // node columns per tile
constexpr int EXN = TX + 1, EYN = TY + 1;  // element columns per layer
constexpr int NSLOT = EXN * EYN;           // 25 elements per layer
constexpr int NXN = TX + 2;                // node columns per row of the node grid (6 x 6)
constexpr int NNODE = NXN * (TY + 2);
// plane record (uint32 words): row0[16] | rowlen[16] | rbase[16] (int64) | npos[16][27] (uint16)
constexpr int PR_ROW0 = 0, PR_LEN = 16, PR_BASE = 32, PR_NPOS = 64;
// LDS image of sqrt|fac| N_XYZ: [dim][Gauss-point pair p][slot][node ^ swizzle][2], the two
// Gauss points 2p, 2p+1 of a node side by side so that one ds_read_b128 fetches both.  The node
// swizzle (p + 4 (slot & 1)) spreads the stage-A stores of an element's 8 lanes (and of the
// 2 elements of a 16-lane store group) over distinct banks.
__device__ constexpr int nx_sw(int p, int slot) { return (p + 4 * (slot & 1)) & 7; }
__device__ constexpr int nx2i(int d, int p, int slot, int n)
{
  return (((d * 4 + p) * NSLOT + slot) * 8 + (n ^ nx_sw(p, slot))) * 2;
}

// hex8 node offsets in 4C node order (4C_io_gridgenerator.cpp:371-379)
__device__ constexpr int node_ox(int n) { return ((n & 3) == 1 || (n & 3) == 2) ? 1 : 0; }
__device__ constexpr int node_oy(int n) { return (n & 3) >= 2 ? 1 : 0; }
__device__ constexpr int node_oz(int n) { return n >> 2; }

struct SweepArgs {
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
  // fused TSI blocks (TSI instantiation only): v, T by column LID (thermo LID = structural / 3),
  // shape values at the Gauss points [8][8], the k_ST / k_TS / k_TT values and f_T by row LID
  const double* v_col;
  const double* T_col;
  const double* Ngp;
  double* Kst;
  double* Kts;
  double* Ktt;
  double* fT;
  double tsi_m, tsi_T0, tsi_k, tsi_kts;  // m, T_0, Fourier k, -timefac timefac_d
  int32_t tiles_x, tiles_y, seg_planes;
  int32_t I0, J0, K0, NI, NJ, NK;
  int32_t EX0, EY0, EZ0, EX, EY, EZ;  // element box; the node lattice box is EX+1 x EY+1 x EZ+1
};

// node data per lattice column: X | u, and for TSI v | T
template <bool TSI>
constexpr int node_comps() { return TSI ? 10 : 6; }

// Record strides (doubles) of the per-(Gauss point, slot) arrays gp and tg below.  Stage A's lane
// (slot s, Gauss point g) stores record 25 g + s; with 16 doubles (32 dwords) every record began on
// bank 0 (mod 32), so a 16-lane ds_write_b64 group was a 16-way conflict and the visit loads at one
// Gauss point saw two distinct banks.  18 (36 dwords) starts record r on bank 4 (g + s) mod 32
// for the stores and 36 s mod 64 for the loads, 16-byte aligned for ds_*_b128 (1M hex8 TotLag
// 2.76 -> 2.40 ms, profiles/r05/r05_gp_stride_ab.txt).  tg (TSI) at 6 instead of 4 measured the
// same (4.31-4.40 vs 4.31-4.35 ms fused), so it stays at 4.
#ifndef FCG_GP_STRIDE
#define FCG_GP_STRIDE 18
#endif
#ifndef FCG_TG_STRIDE
#define FCG_TG_STRIDE 4
#endif

template <int KIN, bool TSI, bool TH = false, bool DEFER = false>
struct SweepShared {
  alignas(16) double nx[3 * 4 * NSLOT * 8 * 2];  // sqrt|fac| N_XYZ, see nx2i()
  // TotLag: F (column-major) | S (Voigt) | c = fac / sqrt|fac| | pad  (linear kinematics: unused)
  alignas(16) double gp[KIN ? 8 : 1][KIN ? NSLOT : 1][KIN ? FCG_GP_STRIDE : 16];
  // TSI: c = fac / sqrt|fac| | T_g | m c sqrt|fac| tr(B_L v)_g = m fac tr(e')_g | pad
  alignas(16) double tg[TSI ? 8 : 1][TSI ? NSLOT : 1][TSI ? FCG_TG_STRIDE : 4];
  double node[3][NNODE][node_comps<TSI>()];  // node columns of the 6 x 6 grid, ring by plane mod 3
  uint32_t prec[3][PLANE_REC_WORDS];  // plane records, ring by plane mod 3
  double gxi[8][4];  // Gauss point coordinates (stage A forms the shape derivatives from them)
  double Ng[TSI ? 8 : 1][8];  // TSI: shape values N_n at Gauss point g
  // the same, node-major rows of 10 (16-byte aligned): the thermal pass's visit reads a node's
  // values at Gauss points (2p, 2p + 1) as one ds_read_b128
  alignas(16) double NgT[TSI ? 8 : 1][10];
  double w8[8];
  uint32_t neg[NSLOT];  // bit g set: fac < 0 at Gauss point g
  // lower-layer parts of the in-plane blocks (dz = 0) of node plane L+1: written by the D-side
  // lane k + 8, read by the U-side lane k of the next layer in the same instruction that precedes
  // the next write (LDS operations of a wavefront complete in order): one buffer suffices.
  // [column][in-plane neighbour (dy+1)*3 + dx+1][3x3 | TSI: k_ST 3 | k_TS 3 | k_TT 1]
  // (TSI rows padded to 18 doubles: with 16 every (column, t) record started on the same bank;
  // thermal-only pass TH: k_ST 3 | k_TS 3 | k_TT 1, padded to 9)
#ifdef FCG_PROBE_WG3
  double hold[1][9][TSI ? (TH ? 9 : 18) : 9];  // timing probe only: one column's buffer for all
#else
  // structural rows 10 apart (16-byte aligned: the 9 held entries as 4 ds_read_b128 + 1
  // ds_read_b64 and 4 ds_write_b128 + 1 ds_write_b64 instead of ds_read2_b64 / ds_write2_b64
  // pairs): headline -0.1 to -0.6 %, TotLag -0.9 % (profiles/r06/r06_sweep_hold10_ab.txt);
  // FCG_HOLD9 = the round-5 rows (A/B)
#if defined(FCG_HOLD9)
  static constexpr int kHs = 9;
#else
  static constexpr int kHs = 10;
#endif
  // (the thermal pass's 7 held values keep rows of 9: aligned rows of 10 measured +0.3 % on the
  // two-field tangent, r06_sweep_hold10_ab.txt)
  alignas(16) double hold[TX * TY][9][TSI ? (TH ? 9 : 18) : kHs];
#endif
  // DEFER (rows not in lattice order): the blocks of node plane L+1's rows with the plane below
  // (dz = -1, finished in layer L) wait here and are written in layer L+1 beside the row's other
  // blocks, so that each row's cache lines are filled within one layer.  Slot (column, t) belongs
  // to the one lane that emits block t of that column every layer: it reads the held block
  // before it holds the next one (a wavefront's LDS operations execute in order), one buffer.
#ifdef FCG_HOLDLO9
  double hold_lo[DEFER ? TX * TY : 1][9][9];  // A/B probe: the round-5 rows
#else
  // rows 10 apart, 16-byte aligned as hold: renumbered 1M box through AUTO 1.149 -> 1.085 ms
  alignas(16) double hold_lo[DEFER ? TX * TY : 1][9][10];
#endif
};

__device__ inline int ring(int p) { return (p % 3 + 3) % 3; }

// Cross-lane moves of a double by DPP (all lanes of the row active)
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;  // lane i <-> 7-i within 8
constexpr int kDppRowRor8 = 0x128;     // lane i <- lane i+8 (mod 16) within a row of 16
template <int CTRL>
__device__ inline double dpp_f64(double v)
{
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// 4C hex8 node index of the node at (ox, oy, oz) of an element (4C_io_gridgenerator.cpp:371-379)
__device__ inline int node_at(int ox, int oy, int oz) { return 4 * oz + (oy ? (ox ? 2 : 3) : (ox ? 1 : 0)); }

// Stage A for element slot s, Gauss point g of layer L (element e, -1 = none).  Written for a
// small register footprint: node data stays in LDS and N_XYZ is recomputed where needed.
template <int KIN, bool TSI, class SH>
__device__ inline void sweep_stage_a(SH& sh, const SweepArgs& A, int s, int g,
    int sx, int sy, int L, int e)
{
  constexpr int NC = node_comps<TSI>();
  const bool valid = e >= 0;
  const double* nd[8];
#pragma unroll
  for (int n = 0; n < 8; ++n)
    nd[n] = sh.node[ring(L + node_oz(n))][(sy + node_oy(n)) * NXN + sx + node_ox(n)];
  // shape derivatives at Gauss point g from its coordinates (no table loads)
  const H8dN dn = h8_dn_products(sh.gxi[g][0], sh.gxi[g][1], sh.gxi[g][2]);
  double J[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) J[q] = 0.0;
#pragma unroll
  for (int n = 0; n < 8; ++n)
  {
    const double x0 = nd[n][0], x1 = nd[n][1], x2 = nd[n][2];
    double d0, d1, d2;
    h8_dn(dn, n, d0, d1, d2);
    J[0] += d0 * x0; J[1] += d1 * x0; J[2] += d2 * x0;
    J[3] += d0 * x1; J[4] += d1 * x1; J[5] += d2 * x1;
    J[6] += d0 * x2; J[7] += d1 * x2; J[8] += d2 * x2;
  }
  int bad = 0;
  // det J at node g (calc_lib.hpp:475-496): at a hex8 corner the shape derivatives are
  // +-1/2 on the node and its neighbour along each parametric direction, so J's columns are
  // half the three edge vectors through the node and det J = det(edges) / 8 (same sign).
  {
    const int ox = node_ox(g), oy = node_oy(g), oz = node_oz(g);
    const double* zl = sh.node[ring(L)][0];
    const double* zh = sh.node[ring(L + 1)][0];
    const double* pz = oz ? zh : zl;
    const int cxy = (sy + oy) * NXN + sx + ox;
    const double* o = pz + NC * cxy;
    const double* ex_ = pz + NC * (cxy + (ox ? -1 : 1));
    const double* ey_ = pz + NC * (cxy + (oy ? -NXN : NXN));
    const double* ez_ = (oz ? zl : zh) + NC * cxy;
    // edge vectors oriented along +xi, +eta, +zeta
    const double sgx = ox ? 1.0 : -1.0, sgy = oy ? 1.0 : -1.0, sgz = oz ? 1.0 : -1.0;
    const double a0 = sgx * (o[0] - ex_[0]), a1 = sgx * (o[1] - ex_[1]), a2 = sgx * (o[2] - ex_[2]);
    const double b0 = sgy * (o[0] - ey_[0]), b1 = sgy * (o[1] - ey_[1]), b2 = sgy * (o[2] - ey_[2]);
    const double c0 = sgz * (o[0] - ez_[0]), c1 = sgz * (o[1] - ez_[1]), c2 = sgz * (o[2] - ez_[2]);
    const double detn = a0 * (b1 * c2 - b2 * c1) + b0 * (c1 * a2 - c2 * a1) + c0 * (a1 * b2 - a2 * b1);
    if (detn == 0.0) bad = 2;
    else if (!(detn > 0)) bad = 1;
  }
  const double det = h8_invert3x3(J);
  if (det == 0.0) bad = 2;
  // the thermo element's check (4C_thermo_ele_impl.cpp:2663-2664)
  else if (TSI && det < 1e-16 && bad == 0) bad = 1;
  const double fac = det * sh.w8[g];
  // missing element (outside the column set): all its LDS data become exact zeros
  const double sq = valid ? sqrt(fabs(fac)) : 0.0;
  const double cf = fac < 0.0 ? -sq : sq;  // fac / sqrt|fac|
  if (KIN == 0)
  {
    // linear: scale J^-1 once; N_XYZ below is then sqrt|fac| N_XYZ, the strain sqrt|fac| E
#pragma unroll
    for (int q = 0; q < 9; ++q) J[q] *= sq;
  }
  const double ns = KIN == 0 ? 1.0 : sq;  // remaining scale of the stored N_XYZ
  // N_XYZ of node n (J now holds J^-1, column-major)
  auto nxyz = [&](int n, double& n0, double& n1, double& n2) {
    double d0, d1, d2;
    h8_dn(dn, n, d0, d1, d2);
    n0 = J[0] * d0 + J[3] * d1 + J[6] * d2;
    n1 = J[1] * d0 + J[4] * d1 + J[7] * d2;
    n2 = J[2] * d0 + J[5] * d1 + J[8] * d2;
  };
  double E[6] = {0, 0, 0, 0, 0, 0};
  double F[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  double Tg = 0.0, trv = 0.0;  // TSI: T_g = N.T, sqrt|fac| tr(B_L v)
#pragma unroll
  for (int n = 0; n < 8; ++n)
  {
    double n0, n1, n2;
    nxyz(n, n0, n1, n2);
    if (TSI)
    {
      trv += n0 * nd[n][6] + n1 * nd[n][7] + n2 * nd[n][8];
      Tg += sh.Ng[TSI ? g : 0][n] * nd[n][9];
    }
    sh.nx[nx2i(0, g >> 1, s, n) + (g & 1)] = KIN == 0 ? n0 : ns * n0;
    sh.nx[nx2i(1, g >> 1, s, n) + (g & 1)] = KIN == 0 ? n1 : ns * n1;
    sh.nx[nx2i(2, g >> 1, s, n) + (g & 1)] = KIN == 0 ? n2 : ns * n2;
    if (KIN == 1)
    {
      // hex8: F = x N_XYZ^T from current coordinates (calc_lib.hpp:585-595)
      const double u0 = nd[n][3], u1 = nd[n][4], u2 = nd[n][5];
      const double q0 = nd[n][0] + u0, q1 = nd[n][1] + u1, q2 = nd[n][2] + u2;
      F[0] += q0 * n0; F[1] += q1 * n0; F[2] += q2 * n0;
      F[3] += q0 * n1; F[4] += q1 * n1; F[5] += q2 * n1;
      F[6] += q0 * n2; F[7] += q1 * n2; F[8] += q2 * n2;
    }
  }
  if (KIN == 1)
  {
    double Fi[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) Fi[q] = F[q];
    if (h8_invert3x3(Fi) == 0.0) bad = 2;
    double C[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        C[r + 3 * q] = F[3 * r] * F[3 * q] + F[3 * r + 1] * F[3 * q + 1] + F[3 * r + 2] * F[3 * q + 2];
    E[0] = 0.5 * (C[0] - 1.0);
    E[1] = 0.5 * (C[4] - 1.0);
    E[2] = 0.5 * (C[8] - 1.0);
    E[3] = C[3];
    E[4] = C[7];
    E[5] = C[2];
  }
  if (KIN == 1)
  {
    const StVK& m = A.mat;
    double S[6];
    S[0] = m.cdiag * E[0] + m.lambda * E[1] + m.lambda * E[2];
    S[1] = m.lambda * E[0] + m.cdiag * E[1] + m.lambda * E[2];
    S[2] = m.lambda * E[0] + m.lambda * E[1] + m.cdiag * E[2];
    S[3] = m.mu * E[3];
    S[4] = m.mu * E[4];
    S[5] = m.mu * E[5];
    double* P = sh.gp[KIN ? g : 0][KIN ? s : 0];
#pragma unroll
    for (int q = 0; q < 9; ++q) P[q] = F[q];
#pragma unroll
    for (int q = 0; q < 6; ++q) P[9 + q] = S[q];
    P[15] = cf;
  }
  if (TSI)
  {
    double* t = sh.tg[TSI ? g : 0][TSI ? s : 0];
    t[0] = cf;
    t[1] = Tg;
    t[2] = A.tsi_m * cf * trv;
  }
  if (valid && bad)
  {
    atomicMax(&A.err[0], bad);
    atomicMin(&A.err[1], e);
  }
  const unsigned long long neg = __ballot(valid && fac < 0.0);
  if (g == 0) sh.neg[s] = uint32_t((neg >> (threadIdx.x & 56)) & 0xFFull);

}

// One element visit: accumulate the blocks (a, b1) into acc1 and (a, b2) into acc2 over the
// Gauss points of element slot `slot`.  Acc layout: G[9] (row-major, G[3r+q] = sum a'_r b'_q)
// then, for TotLag, H[6] and geo; for TSI (linear) sum c N_b a[3], sum c N_a T_g b[3] and
// sum m fac tr(e') N_a N_b (the factors m, -timefac timefac_d and k enter in tsi_block).
// TH (the thermal-only pass beside the linear structural sweep): no G, the thermal sums at
// acc[0..5], fac a.b at acc[6] (k_TT's conduction part) and sum m fac tr(e') N_a N_b at acc[7].
template <int KIN, bool NEG, bool TSI, bool TH = false, class SH>
__device__ inline void sweep_visit(const SH& sh, int slot, int a, int b1, int b2,
    uint32_t nm, double* acc1, double* acc2)
{
#ifndef FCG_TH_PAIRS
#define FCG_TH_PAIRS 1
#endif
  // thermal pass: the shape values of nodes a, b1, b2 at all 8 Gauss points as 12 explicit
  // 16-byte reads (the compiler paired the per-point 8-byte reads across points into
  // ds_read2_b64, 8 LDS cycles per 16 bytes against 4)
  double2 nA[TH && FCG_TH_PAIRS ? 4 : 1], n1[TH && FCG_TH_PAIRS ? 4 : 1], n2[TH && FCG_TH_PAIRS ? 4 : 1];
  if constexpr (TH && FCG_TH_PAIRS)
  {
#pragma unroll
    for (int p = 0; p < 4; ++p)
    {
      nA[p] = *reinterpret_cast<const double2*>(&sh.NgT[a][2 * p]);
      n1[p] = *reinterpret_cast<const double2*>(&sh.NgT[b1][2 * p]);
      n2[p] = *reinterpret_cast<const double2*>(&sh.NgT[b2][2 * p]);
    }
  }
  auto gp_body = [&](int g, double a0, double a1, double a2, double p0, double p1, double p2,
                     double q0, double q1, double q2) {
    if (TH)
    {
      const double* t = sh.tg[g][slot];
#if FCG_TH_PAIRS
      const double2 t01 = *reinterpret_cast<const double2*>(t), t23 = *reinterpret_cast<const double2*>(t + 2);
      const double cf = t01.x, Tg = t01.y, qq = t23.x;
      const double Na = (g & 1) ? nA[g >> 1].y : nA[g >> 1].x, N1 = (g & 1) ? n1[g >> 1].y : n1[g >> 1].x,
                   N2 = (g & 1) ? n2[g >> 1].y : n2[g >> 1].x;
#else
      const double cf = t[0], Tg = t[1], qq = t[2];
      const double Na = sh.Ng[g][a], N1 = sh.Ng[g][b1], N2 = sh.Ng[g][b2];
#endif
      const double c1 = cf * N1, c2 = cf * N2, ct = cf * Na * Tg, qa = qq * Na;
      acc1[0] += c1 * a0; acc1[1] += c1 * a1; acc1[2] += c1 * a2;
      acc2[0] += c2 * a0; acc2[1] += c2 * a1; acc2[2] += c2 * a2;
      acc1[3] += ct * p0; acc1[4] += ct * p1; acc1[5] += ct * p2;
      acc2[3] += ct * q0; acc2[4] += ct * q1; acc2[5] += ct * q2;
      acc1[7] += qa * N1;
      acc2[7] += qa * N2;
      // fac a.b: sqrt|fac| a . sqrt|fac| b with the sign of fac
      const double sg = (NEG && ((nm >> g) & 1u)) ? -1.0 : 1.0;
      acc1[6] += sg * (a0 * p0 + a1 * p1 + a2 * p2);
      acc2[6] += sg * (a0 * q0 + a1 * q1 + a2 * q2);
      return;
    }
    if (TSI)
    {
      // unflipped sqrt|fac| N_XYZ times c = fac / sqrt|fac| gives fac N_XYZ
      const double* t = sh.tg[TSI ? g : 0][TSI ? slot : 0];
      const double cf = t[0], Tg = t[1], qq = t[2];
      const double Na = sh.Ng[TSI ? g : 0][a], N1 = sh.Ng[TSI ? g : 0][b1],
                   N2 = sh.Ng[TSI ? g : 0][b2];
      const double c1 = cf * N1, c2 = cf * N2, ct = cf * Na * Tg, qa = qq * Na;
      acc1[9] += c1 * a0; acc1[10] += c1 * a1; acc1[11] += c1 * a2;
      acc2[9] += c2 * a0; acc2[10] += c2 * a1; acc2[11] += c2 * a2;
      acc1[12] += ct * p0; acc1[13] += ct * p1; acc1[14] += ct * p2;
      acc2[12] += ct * q0; acc2[13] += ct * q1; acc2[14] += ct * q2;
      acc1[15] += qa * N1;
      acc2[15] += qa * N2;
    }
    if (NEG && ((nm >> g) & 1u))
    {
      a0 = -a0;
      a1 = -a1;
      a2 = -a2;
    }
    if (KIN == 0)
    {
#ifdef FCG_PROBE_NOG
      // timing probe only (wrong results): the loads kept, 4 of the 18 FMAs
      const double sa = a0 + a1 + a2;
      acc1[0] += sa * (p0 + p1 + p2);
      acc2[0] += sa * (q0 + q1 + q2);
      return;
#endif
      acc1[0] += a0 * p0; acc1[1] += a0 * p1; acc1[2] += a0 * p2;
      acc1[3] += a1 * p0; acc1[4] += a1 * p1; acc1[5] += a1 * p2;
      acc1[6] += a2 * p0; acc1[7] += a2 * p1; acc1[8] += a2 * p2;
      acc2[0] += a0 * q0; acc2[1] += a0 * q1; acc2[2] += a0 * q2;
      acc2[3] += a1 * q0; acc2[4] += a1 * q1; acc2[5] += a1 * q2;
      acc2[6] += a2 * q0; acc2[7] += a2 * q1; acc2[8] += a2 * q2;
    }
    else
    {
      const double* P = sh.gp[g][slot];
      const double F0 = P[0], F1 = P[1], F2 = P[2], F3 = P[3], F4 = P[4], F5 = P[5], F6 = P[6],
                   F7 = P[7], F8 = P[8];
      const double S0 = P[9], S1 = P[10], S2 = P[11], S3 = P[12], S4 = P[13], S5 = P[14];
      const double fa0 = F0 * a0 + F3 * a1 + F6 * a2;
      const double fa1 = F1 * a0 + F4 * a1 + F7 * a2;
      const double fa2 = F2 * a0 + F5 * a1 + F8 * a2;
      const double M0 = F0 * F0 + F3 * F3 + F6 * F6, M1 = F1 * F1 + F4 * F4 + F7 * F7,
                   M2 = F2 * F2 + F5 * F5 + F8 * F8, M3 = F0 * F1 + F3 * F4 + F6 * F7,
                   M4 = F1 * F2 + F4 * F5 + F7 * F8, M5 = F2 * F0 + F5 * F3 + F8 * F6;
      // a.S (S symmetric): geo = (S a).b
      const double sa0 = S0 * a0 + S3 * a1 + S5 * a2;
      const double sa1 = S3 * a0 + S1 * a1 + S4 * a2;
      const double sa2 = S5 * a0 + S4 * a1 + S2 * a2;
      auto one = [&](double* acc, double b0, double bb1, double bb2) {
        const double fb0 = F0 * b0 + F3 * bb1 + F6 * bb2;
        const double fb1 = F1 * b0 + F4 * bb1 + F7 * bb2;
        const double fb2 = F2 * b0 + F5 * bb1 + F8 * bb2;
        acc[0] += fa0 * fb0; acc[1] += fa0 * fb1; acc[2] += fa0 * fb2;
        acc[3] += fa1 * fb0; acc[4] += fa1 * fb1; acc[5] += fa1 * fb2;
        acc[6] += fa2 * fb0; acc[7] += fa2 * fb1; acc[8] += fa2 * fb2;
        const double ab = a0 * b0 + a1 * bb1 + a2 * bb2;
        acc[9] += ab * M0;
        acc[10] += ab * M1;
        acc[11] += ab * M2;
        acc[12] += ab * M3;
        acc[13] += ab * M4;
        acc[14] += ab * M5;
        acc[15] += sa0 * b0 + sa1 * bb1 + sa2 * bb2;
      };
      one(acc1, p0, p1, p2);
      one(acc2, q0, q1, q2);
    }
  };
  auto load_p = [&](int p, double2* v) {
    const int nd[3] = {a, b1, b2};
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int d = 0; d < 3; ++d) v[3 * k + d] = *reinterpret_cast<const double2*>(&sh.nx[nx2i(d, p, slot, nd[k])]);
  };
#ifndef FCG_VISIT_NOPIPE
  // structural passes: software-pipelined, the nine N_XYZ pairs of Gauss-point pair p + 1 are in
  // flight while pair p computes (the scheduling barrier keeps the loads ahead of the FMAs; the
  // compiler otherwise issues each pair's loads after the previous pair's FMAs and waits for them,
  // an exposed LDS round trip per pair at two waves per SIMD).  +47 VGPRs (189 -> 236, still two
  // workgroups per CU); the TSI instantiations would spill, they keep the plain loop.
#ifdef FCG_VISIT_PIPE_TSI
  if constexpr (true)
#else
  if constexpr (!TSI)
#endif
  {
  double2 buf[2][9];
  load_p(0, buf[0]);
#pragma unroll
  for (int p = 0; p < 4; ++p)
  {
    if (p < 3) load_p(p + 1, buf[(p + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
    const double2* v = buf[p & 1];
    gp_body(2 * p, v[0].x, v[1].x, v[2].x, v[3].x, v[4].x, v[5].x, v[6].x, v[7].x, v[8].x);
    gp_body(2 * p + 1, v[0].y, v[1].y, v[2].y, v[3].y, v[4].y, v[5].y, v[6].y, v[7].y, v[8].y);
  }
  return;
  }
#endif
#pragma unroll
  for (int p = 0; p < 4; ++p)
  {
    double2 v[9];
    load_p(p, v);
    gp_body(2 * p, v[0].x, v[1].x, v[2].x, v[3].x, v[4].x, v[5].x, v[6].x, v[7].x, v[8].x);
    gp_body(2 * p + 1, v[0].y, v[1].y, v[2].y, v[3].y, v[4].y, v[5].y, v[6].y, v[7].y, v[8].y);
  }
}

// TSI blocks of an accumulated (linear) part: k_ST(A,B) [3] | k_TS(A,B) [3] | k_TT(A,B)
template <bool TH = false>
__device__ inline void tsi_block(const SweepArgs& A, const double* acc, double* Tv)
{
  const double m = A.tsi_m, mk = A.tsi_m * A.tsi_kts;
  constexpr int o = TH ? 0 : 9;
  Tv[0] = m * acc[o + 0];
  Tv[1] = m * acc[o + 1];
  Tv[2] = m * acc[o + 2];
  Tv[3] = mk * acc[o + 3];
  Tv[4] = mk * acc[o + 4];
  Tv[5] = mk * acc[o + 5];
  Tv[6] = TH ? A.tsi_k * acc[6] - acc[7] : A.tsi_k * (acc[0] + acc[4] + acc[8]) - acc[15];
}

// K_AB of an accumulated part (isotropic StVK)
template <int KIN>
__device__ inline void block_k(const StVK& m, const double* acc, double* Kb)
{
  const double lam = m.lambda, mu = m.mu;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int q = 0; q < 3; ++q) Kb[3 * r + q] = lam * acc[3 * r + q] + mu * acc[3 * q + r];
  if (KIN == 0)
  {
    const double tr = mu * (acc[0] + acc[4] + acc[8]);
    Kb[0] += tr;
    Kb[4] += tr;
    Kb[8] += tr;
  }
  else
  {
    Kb[0] += mu * acc[9] + acc[15];
    Kb[4] += mu * acc[10] + acc[15];
    Kb[8] += mu * acc[11] + acc[15];
    Kb[1] += mu * acc[12]; Kb[3] += mu * acc[12];
    Kb[5] += mu * acc[13]; Kb[7] += mu * acc[13];
    Kb[2] += mu * acc[14]; Kb[6] += mu * acc[14];
  }
}

// Diagnostic phase stamps: thread 0 of each workgroup adds the cycles of every phase (including
// the barrier wait that ends it) into A.stamps[phase]; off (uniform branch, no s_memtime) when
// A.stamps is NULL.  Phases: 0 element stage (A), 1 visit stage (B); [5] counts workgroups.
#define FCG_STAMP(i)                                                                               \
  if (A.stamps && tid == 0)                                                                        \
  {                                                                                                \
    const unsigned long long now = __builtin_amdgcn_s_memtime();                                  \
    st_acc[i] += now - st_last;                                                                    \
    st_last = now;                                                                                 \
  }

// MODE 0: structure (K, f_int); 1: fused TSI (K_SS, k_ST, k_TS, k_TT, f_S, f_T in one pass);
// 2: the thermal-only pass that follows a MODE-0 linear sweep (k_ST, k_TS, k_TT, f_T, and
// k_ST (T - T_0) added into f_S) -- 8 accumulators per block instead of 16, no K stores;
// 3: structure with the lower-plane blocks deferred one layer (hold_lo), for meshes whose CSR
// rows do not list the lattice neighbours plane by plane (input-file numbering): a row's 27
// triples then land all over its 648 bytes, and writing them in two layers' halves left its
// lines half-written in L2 between the two (1.4x the K bytes written on the renumbered 1M box).
template <int KIN, bool WANT_K, bool OVERWRITE, int MODE>
#ifndef FCG_SWEEP_WGS
#define FCG_SWEEP_WGS 2
#endif
__global__ __launch_bounds__(256, KIN ? 1 : FCG_SWEEP_WGS) void sweep_h8_kernel(SweepArgs A)
{
  constexpr bool TSI = MODE == 1 || MODE == 2, TH = MODE == 2, DEFER = MODE == 3;
  static_assert(!TSI || (KIN == 0 && WANT_K), "TSI is geometrically linear, full tangent");
  static_assert(!DEFER || WANT_K, "deferred blocks are K blocks");
  __shared__ SweepShared<KIN, TSI, TH, DEFER> sh;
  constexpr int NACC = TH ? 8 : ((KIN || TSI) ? 16 : 9);
  constexpr int NC = node_comps<TSI>();
  constexpr int NLD = (NNODE * NC + 255) / 256;  // node-load items per lane
  constexpr int NF = TSI ? 4 : 3;                // residual rows per node: f_S (3) | f_T
  const int tid = threadIdx.x;
  unsigned long long st_acc[3] = {0, 0, 0};
  unsigned long long st_last = A.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
  const int tile = blockIdx.x;
  const int tx = tile % A.tiles_x;
  const int ty = (tile / A.tiles_x) % A.tiles_y;
  const int tz = tile / (A.tiles_x * A.tiles_y);
  const int i0 = A.I0 + TX * tx, j0 = A.J0 + TY * ty;
  const int kz0 = A.K0 + A.seg_planes * tz;
  const int kz1 = min(kz0 + A.seg_planes, A.K0 + A.NK);
  const uint32_t* prec_tile = A.plane_rec + (int64_t(ty) * A.tiles_x + tx) * A.NK * PLANE_REC_WORDS;
  const int64_t LX = A.EX + 1, LY = A.EY + 1;

  if (tid < 24) sh.gxi[tid / 3][tid % 3] = A.tables[392 + tid];
  if (tid < 8) sh.w8[tid] = A.tables[384 + tid];
  if (TSI && tid < 64)
  {
    (&sh.Ng[0][0])[tid] = A.Ngp[tid];
    sh.NgT[TSI ? (tid & 7) : 0][tid >> 3] = A.Ngp[tid];
  }

  // stage-A lane: element slot s, Gauss point g
  const int s = tid >> 3, g = tid & 7;
  const bool a_lane = s < NSLOT;
  const int sx = s % EXN, sy = s / EXN;
  const int ex = i0 - 1 + sx, ey = j0 - 1 + sy;
  const bool exy_in = a_lane && ex >= A.EX0 && ex < A.EX0 + A.EX && ey >= A.EY0 && ey < A.EY0 + A.EY;
  auto load_elem = [&](int lz) -> int {
    if (!exy_in || lz < A.EZ0 || lz >= A.EZ0 + A.EZ) return -1;
    return A.elem_at[(int64_t(lz - A.EZ0) * A.EY + (ey - A.EY0)) * A.EX + (ex - A.EX0)];
  };
  // node-load items tid + 256 j: column ncol of the 6 x 6 node grid, component ncomp
  // (X 0-2, u 3-5; TSI: v 6-8, T 9)
  bool n_lane[NLD], nxy_in[NLD];
  int ncol[NLD], ncomp[NLD];
  int64_t nlat_xy[NLD];
#pragma unroll
  for (int j = 0; j < NLD; ++j)
  {
    const int v = tid + 256 * j;
    n_lane[j] = v < NNODE * NC;
    ncol[j] = v / NC;
    ncomp[j] = v - NC * (v / NC);
    const int ni = i0 - 1 + ncol[j] % NXN, nj = j0 - 1 + ncol[j] / NXN;
    nxy_in[j] = n_lane[j] && ni >= A.EX0 && ni <= A.EX0 + A.EX && nj >= A.EY0 && nj <= A.EY0 + A.EY;
    nlat_xy[j] = nxy_in[j] ? int64_t(nj - A.EY0) * LX + (ni - A.EX0) : 0;
  }
  // node loads in two steps, so that no load waits on another inside a layer: the DOF of a plane
  // is fetched one layer before its values (load_dof), the values (load_val) are issued before
  // stage A and consumed after it -- the wait for them then also covers the previous layer's K
  // stores (gfx9 counts stores in vmcnt), which stage A has had time to retire.
  auto node_li = [&](int j, int P) -> int64_t { return int64_t(P - A.EZ0) * LX * LY + nlat_xy[j]; };
  auto node_in = [&](int j, int P) -> bool { return nxy_in[j] && P >= A.EZ0 && P <= A.EZ0 + A.EZ; };
  auto load_dof = [&](int j, int P) -> int32_t {
    if (!node_in(j, P) || ncomp[j] < 3) return -1;
    return A.lat_dof[node_li(j, P)];
  };
  auto load_val = [&](int j, int P, int32_t dof) -> double {
    if (!node_in(j, P)) return 0.0;
    const int cp = ncomp[j];
    if (cp < 3) return A.lat_x[3 * node_li(j, P) + cp];
    if (dof < 0) return 0.0;
    if (!TSI || cp < 6) return A.u_col[dof + cp - 3];
    if (cp < 9) return A.v_col[dof + cp - 6];
    return A.T_col[dof / 3];
  };
  auto load_node = [&](int j, int P) -> double { return load_val(j, P, load_dof(j, P)); };
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

  // visit lane: node column c, task k
  const int c = tid >> 4, k = tid & 15;
  const int cx = c % TX, cy = c / TX;
  const uint32_t vis0 = kVisit[k][0], vis1 = kVisit[k][1];

  // --- prologue: node planes kz0-1, kz0 and their records; prefetch plane kz0+1
#pragma unroll
  for (int j = 0; j < NLD; ++j)
    if (n_lane[j])
    {
      sh.node[ring(kz0 - 1)][ncol[j]][ncomp[j]] = load_node(j, kz0 - 1);
      sh.node[ring(kz0)][ncol[j]][ncomp[j]] = load_node(j, kz0);
    }
  {
    uint32_t w[2];
    load_rec(kz0 - 1, w);
    store_rec(kz0 - 1, w);
    load_rec(kz0, w);
    store_rec(kz0, w);
  }
  int32_t dof_nxt[NLD];  // DOF of plane L+2's node-load items at the top of layer L
#pragma unroll
  for (int j = 0; j < NLD; ++j) dof_nxt[j] = n_lane[j] ? load_dof(j, kz0 + 1) : -1;
  int e_cur = load_elem(kz0 - 1);
  for (int v = tid; v < int(sizeof(sh.hold) / sizeof(double)); v += 256) (&sh.hold[0][0][0])[v] = 0.0;
  double fkeep[NF];  // lane k = 8: D-side residual part of plane L+1's rows
#pragma unroll
  for (int d = 0; d < NF; ++d) fkeep[d] = 0.0;
  // the prologue's loads land here, so that the compiler's wait bookkeeping does not carry them
  // into the loop (where the first use of e_cur would otherwise wait for every load in flight)
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  for (int L = kz0 - 1; L < kz1; ++L)
  {
    // issue the loads of plane L+2 (values, record), plane L+3's DOFs and layer L+1's element
    const int e_nxt = load_elem(L + 1);
    double node_nxt[NLD];
    int32_t dof_nn[NLD];
#pragma unroll
    for (int j = 0; j < NLD; ++j)
    {
#ifdef FCG_PROBE_TH_NOPREFETCH
      if (TH)
      {
        // timing probe only (wrong results): the thermal pass without its plane prefetch
        node_nxt[j] = 0.0;
        dof_nn[j] = -1;
        continue;
      }
#endif
      node_nxt[j] = n_lane[j] ? load_val(j, L + 2, dof_nxt[j]) : 0.0;
      dof_nn[j] = n_lane[j] ? load_dof(j, L + 3) : -1;
    }
    uint32_t rec_nxt[2];
    load_rec(L + 2, rec_nxt);
    // A. element stage
#ifdef FCG_PROBE_NOSTAGEA
    // timing probe only (wrong results): no element stage
    if (a_lane && e_cur == -12345) sweep_stage_a<KIN, TSI>(sh, A, s, g, sx, sy, L, e_cur);
#else
    if (a_lane) sweep_stage_a<KIN, TSI>(sh, A, s, g, sx, sy, L, e_cur);
#endif
    __syncthreads();
    FCG_STAMP(0);
    // commit plane L+2 (nodes and record into plane L-1's ring slot)
#pragma unroll
    for (int j = 0; j < NLD; ++j)
    {
      if (n_lane[j]) sh.node[ring(L + 2)][ncol[j]][ncomp[j]] = node_nxt[j];
      dof_nxt[j] = dof_nn[j];
    }
    store_rec(L + 2, rec_nxt);
#ifdef FCG_SWEEP_COMMIT_STAMP
    // diagnostic builds only (it costs the fused TSI pass a spill)
    if (A.stamps)
    {
      // phase 2: the commit's wait for plane L+2's loads (and, behind them in vmcnt, the previous
      // layer's K stores)
      __asm__ volatile("" ::"v"(rec_nxt[0]), "v"(node_nxt[0]));
      FCG_STAMP(2);
    }
#endif

    // B. visit stage
    const bool wl = L >= kz0, wl1 = L + 1 < kz1;
    const uint32_t* recL = sh.prec[ring(L)];
    const uint32_t* recL1 = sh.prec[ring(L + 1)];
    // linear kinematics: this lane's share of f_A = sum_B K_AB u_B for the row node A of its side
    // (plane L + (k >> 3))
    double fpart[NF];
#pragma unroll
    for (int d = 0; d < NF; ++d) fpart[d] = 0.0;
    if (WANT_K || KIN == 0)
    {
      // finished block t of this lane's column (this layer's elements): hold it, or write it plus
      // the part held by lane k + 8 (same role, D side) since the previous layer.  TSI: Tv holds
      // the block's k_ST / k_TS / k_TT entries (tsi_block), treated the same way.
      auto emit = [&](int act, int t, double* Kb, double* Tv) {
        // the block's record fields first, all four reads before any branch: one LDS round trip,
        // which the residual and hold work below overlaps (read one by one behind the early
        // returns, each waited for in turn)
        const bool to_l1 = act == kActWriteL1;
        const uint32_t* rec = to_l1 ? recL1 : recL;
        const int32_t row0 = WANT_K ? int32_t(rec[PR_ROW0 + c]) : -1;
        const uint16_t pos = WANT_K ? reinterpret_cast<const uint16_t*>(rec + PR_NPOS)[27 * c + t] : 0;
        const uint32_t base_lo = WANT_K ? rec[PR_BASE + 2 * c] : 0u;
        const uint32_t base_hi = WANT_K ? rec[PR_BASE + 2 * c + 1] : 0u;
        const int32_t len32 = WANT_K ? int32_t(rec[PR_LEN + c]) : 0;
        if (KIN == 0)
        {
          const int dx = t % 3 - 1, dy = (t / 3) % 3 - 1, dz = t / 9 - 1;
          const double* ub = &sh.node[ring(L + (k >> 3) + dz)][(cy + 1 + dy) * NXN + cx + 1 + dx][3];
          const double u0 = ub[0], u1 = ub[1], u2 = ub[2];
          if (!TH)
#pragma unroll
            for (int r = 0; r < 3; ++r) fpart[r] += Kb[3 * r] * u0 + Kb[3 * r + 1] * u1 + Kb[3 * r + 2] * u2;
          if (TSI)
          {
            // f_S += k_ST (T - T_0) (partition of unity), f_T = k_TT T (exact for linear TSI)
            const double TB = ub[6];
            const double dT = TB - A.tsi_T0;
#pragma unroll
            for (int r = 0; r < 3; ++r) fpart[r] += Tv[r] * dT;
            fpart[NF - 1] += Tv[6] * TB;
          }
        }
        // in-plane blocks: every lane of the pair reads the held entry first, then the holder
        // (D side) stores this layer's part and the U side adds the part held since last layer
        if (act == kActHold || act == kActWriteLHold)
        {
          constexpr int NK = TH ? 0 : 9;  // structural entries held (none in the thermal pass)
          constexpr int NH = NK + (TSI ? 7 : 0);
#ifdef FCG_PROBE_WG3
          double* h = sh.hold[0][t - 9];
#else
          double* h = sh.hold[c][t - 9];
#endif
          double held[NH];
#pragma unroll
          for (int i = 0; i < NH; ++i) held[i] = h[i];
          // all reads issue before any write (the compiler must not sink the U side's reads into
          // its branch behind the D side's writes; the LDS executes a wavefront's ops in order)
          __asm__ volatile("" ::: "memory");
          if (act == kActHold)
          {
#pragma unroll
            for (int i = 0; i < NK; ++i) h[i] = Kb[i];
            if (TSI)
#pragma unroll
              for (int i = 0; i < 7; ++i) h[NK + i] = Tv[i];
          }
          else
          {
#pragma unroll
            for (int i = 0; i < NK; ++i) Kb[i] = held[i] + Kb[i];
            if (TSI)
#pragma unroll
              for (int i = 0; i < 7; ++i) Tv[i] = held[NK + i] + Tv[i];
          }
        }
        if (act == kActHold || !WANT_K) return;
        if constexpr (DEFER)
        {
          if (act == kActWriteL1)
          {
            // the block held since the previous layer belongs to plane L's row: write it now,
            // beside that row's other blocks; hold this layer's block for plane L+1
            const int32_t row0L = int32_t(recL[PR_ROW0 + c]);
            const uint16_t posL = reinterpret_cast<const uint16_t*>(recL + PR_NPOS)[27 * c + t];
            const uint32_t bloL = recL[PR_BASE + 2 * c], bhiL = recL[PR_BASE + 2 * c + 1];
            const int64_t lenL = int32_t(recL[PR_LEN + c]);
            double* h = sh.hold_lo[c][t];
            double old[9];
#pragma unroll
            for (int i = 0; i < 9; ++i) old[i] = h[i];
            __asm__ volatile("" ::: "memory");
#pragma unroll
            for (int i = 0; i < 9; ++i) h[i] = Kb[i];
            if (!wl || row0L < 0 || posL == 0xFFFF) return;
            double* dlo = A.K + (int64_t(bloL) | (int64_t(bhiL) << 32)) + posL;
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
              for (int qq = 0; qq < 3; ++qq)
              {
                if (OVERWRITE)
                  dlo[r * lenL + qq] = old[3 * r + qq];
                else
                  dlo[r * lenL + qq] += old[3 * r + qq];
              }
            return;
          }
        }
        if (!(to_l1 ? wl1 : wl) || row0 < 0 || pos == 0xFFFF) return;
        const int64_t base = int64_t(base_lo) | (int64_t(base_hi) << 32);
        const int64_t len = len32;
#ifdef FCG_PROBE_KL2
        // timing probe only (wrong results): the same stores, folded into 256 KB (L2-resident)
        double* dst = A.K + ((base + pos) & 0x7FFF);
#else
        double* dst = A.K + base + pos;
#endif
#ifdef FCG_PROBE_NOKSTORE
        // timing probe only (wrong results): no K stores
        if (Kb[0] == 12345.678) dst[0] = Kb[1];
        if (false)
#else
        if (!TH)
#endif
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int qq = 0; qq < 3; ++qq)
            {
              if (OVERWRITE)
#ifdef FCG_PROBE_KNT  // timing probe: non-temporal K stores (4.2 ms instead of 0.98: partial lines)
                __builtin_nontemporal_store(Kb[3 * r + qq], dst + r * len + qq);
#else
                dst[r * len + qq] = Kb[3 * r + qq];
#endif
              else
                dst[r * len + qq] += Kb[3 * r + qq];
            }
#if defined(FCG_PROBE_TH_NOSTORE) || defined(FCG_PROBE_TH_1STORE)
        if (TH)
        {
          // timing probes only (wrong results): no thermal stores / one 8-byte store per block
#ifdef FCG_PROBE_TH_1STORE
          A.Ktt[base / 9 + pos / 3] = Tv[0] + Tv[1] + Tv[2] + Tv[3] + Tv[4] + Tv[5] + Tv[6];
#else
          if (Tv[0] == 12345.678) A.Ktt[0] = Tv[1];
#endif
          return;
        }
#endif
        if (TSI)
        {
          // node-consistent block graphs (checked by fcg_tsi_evaluate_fused): the k_ST rows of the
          // node start at base / 3 (length len / 3), its k_TS row at base / 3, its k_TT row at
          // base / 9; the neighbour's thermo column sits at pos / 3, its displacements at pos
          const int64_t bst = base / 3, lst = len / 3, pst = pos / 3;
#ifdef FCG_PROBE_TSI_STORE_INTERLEAVED
          if constexpr (true)  // timing probe: the order before round 6
#else
          if constexpr (false)
#endif
          {
#pragma unroll
          for (int r = 0; r < 3; ++r)
          {
            double* d1 = A.Kst + bst + r * lst + pst;
            double* d2 = A.Kts + bst + pos + r;
            if (OVERWRITE)
            {
              *d1 = Tv[r];
              *d2 = Tv[3 + r];
            }
            else
            {
              *d1 += Tv[r];
              *d2 += Tv[3 + r];
            }
          }
          }
          else
          {
          // k_TS's three adjacent values first, with no k_ST store between them (the two arrays
          // may alias as far as the compiler knows), so that they leave as one 16-byte and one
          // 8-byte store instead of three 8-byte stores
          double* d2 = A.Kts + bst + pos;
#pragma unroll
          for (int r = 0; r < 3; ++r)
          {
            if (OVERWRITE)
              d2[r] = Tv[3 + r];
            else
              d2[r] += Tv[3 + r];
          }
#pragma unroll
          for (int r = 0; r < 3; ++r)
          {
            double* d1 = A.Kst + bst + r * lst + pst;
            if (OVERWRITE)
              *d1 = Tv[r];
            else
              *d1 += Tv[r];
          }
          }
          double* d3 = A.Ktt + base / 9 + pst;
          if (OVERWRITE)
            *d3 = Tv[6];
          else
            *d3 += Tv[6];
        }
      };
      double acc1[NACC], acc2[NACC];
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc1[i] = acc2[i] = 0.0;
      // the two element visits of this lane; acc2 is finished after a visit when flush2 is set.
      // Without TSI both visits' negative-fac masks are read up front (one LDS round trip instead
      // of one ahead of each visit's branch; the TSI instantiation has no registers to spare).
      auto slot_of = [&](uint32_t w) { return (cx + int(w & 1)) + EXN * (cy + int((w >> 1) & 1)); };
      uint32_t nm_pre[2] = {0u, 0u};
      if constexpr (!TSI)
      {
        nm_pre[0] = sh.neg[slot_of(vis0)];
        nm_pre[1] = sh.neg[slot_of(vis1)];
      }
      // the two visits unrolled where the registers allow it (the structural linear passes: 254
      // VGPRs, no spills; the next visit's loads then overlap the first one's emit, -3 % on the
      // headline kernel, profiles/r06/r06_sweep_visit_unroll_ab.txt); the TSI passes spill
      // unrolled, and the TotLag ones keep the rolled loop (FCG_SWEEP_VISIT_UNROLL=0/1 overrides)
#ifndef FCG_SWEEP_VISIT_UNROLL
#define FCG_SWEEP_VISIT_UNROLL (!TSI && KIN == 0)
#endif
      constexpr int kVisitUnroll = (FCG_SWEEP_VISIT_UNROLL) ? 2 : 1;
#pragma unroll kVisitUnroll
      for (int v = 0; v < 2; ++v)
      {
        const uint32_t w = v == 0 ? vis0 : vis1;
        const int a = (w >> 2) & 7, b1 = (w >> 5) & 7, b2 = (w >> 8) & 7;
        const int slot = slot_of(w);
        const uint32_t nm = TSI ? sh.neg[slot] : (v == 0 ? nm_pre[0] : nm_pre[1]);
        if (nm == 0u)
          sweep_visit<KIN, false, TSI, TH>(sh, slot, a, b1, b2, nm, acc1, acc2);
        else
          sweep_visit<KIN, true, TSI, TH>(sh, slot, a, b1, b2, nm, acc1, acc2);
        if ((w >> 24) & 1u)
        {
          double Kb[9], Tv[7];
          if (!TH) block_k<KIN>(A.mat, acc2, Kb);
          if (TSI) tsi_block<TH>(A, acc2, Tv);
#pragma unroll
          for (int i = 0; i < NACC; ++i) acc2[i] = 0.0;
          emit(int((w >> 21) & 7), int((w >> 16) & 31), Kb, Tv);
        }
      }
      // acc1: the self block's two halves meet in lane r = 2 (order: qy = 1 half + qy = 0 half)
      {
        const int pair = int((vis1 >> 26) & 3);
        double Kb[9], Tv[7];
        if (!TH)
        {
          block_k<KIN>(A.mat, acc1, Kb);
#pragma unroll
          for (int i = 0; i < 9; ++i)
          {
            const double o = dpp_f64<kDppXor1>(Kb[i]);
            Kb[i] = pair == kPairRecv ? Kb[i] + o : Kb[i];  // a select, not a branch per entry
          }
        }
        if (TSI)
        {
          tsi_block<TH>(A, acc1, Tv);
#pragma unroll
          for (int i = 0; i < 7; ++i)
          {
            const double o = dpp_f64<kDppXor1>(Tv[i]);
            Tv[i] = pair == kPairRecv ? Tv[i] + o : Tv[i];
          }
        }
        if (pair != kPairGive) emit(int((vis1 >> 21) & 7), int((vis1 >> 11) & 31), Kb, Tv);
      }
    }
    // residual rows of the column: the 8 lanes of a side sum their parts by a butterfly (every
    // lane ends with the same bits); lane 8 keeps plane L+1's D-side part for the next layer, lane
    // 0 adds the part lane 8 kept in the previous layer and writes plane L's rows.
    {
      double f[NF];
      if (KIN == 0)
      {
#pragma unroll
        for (int d = 0; d < NF; ++d) f[d] = fpart[d];
      }
      else
      {
        // f_A = sum_e sum_g fac F S N_XYZ_A: lane k takes Gauss points 4h..4h+3 (h = k & 1) of
        // quadrant q = (k >> 1) & 3 for the row node on side k >> 3 (0: plane L, the elements'
        // bottom node; 1: plane L+1, their top node)
        const int fside = k >> 3, fq = (k >> 1) & 3, fh = k & 1;
        const int fqx = fq & 1, fqy = fq >> 1;
        const int fslot = (cx + fqx) + EXN * (cy + fqy);
        const int fn = node_at(1 - fqx, 1 - fqy, fside);
#pragma unroll
        for (int d = 0; d < 3; ++d) f[d] = 0.0;
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
        {
          const int gq = 4 * fh + gg;
          const double a0 = sh.nx[nx2i(0, gq >> 1, fslot, fn) + (gq & 1)],
                       a1 = sh.nx[nx2i(1, gq >> 1, fslot, fn) + (gq & 1)],
                       a2 = sh.nx[nx2i(2, gq >> 1, fslot, fn) + (gq & 1)];
          const double* P = sh.gp[KIN ? gq : 0][KIN ? fslot : 0];
          const double t0 = P[9] * a0 + P[12] * a1 + P[14] * a2;
          const double t1 = P[12] * a0 + P[10] * a1 + P[13] * a2;
          const double t2 = P[14] * a0 + P[13] * a1 + P[11] * a2;
          const double cc = P[15];
          f[0] += cc * (P[0] * t0 + P[3] * t1 + P[6] * t2);
          f[1] += cc * (P[1] * t0 + P[4] * t1 + P[7] * t2);
          f[2] += cc * (P[2] * t0 + P[5] * t1 + P[8] * t2);
        }
      }
      const int32_t frow0 = int32_t(recL[PR_ROW0 + c]);  // read ahead of the butterfly
      double fp[NF];
#pragma unroll
      for (int d = 0; d < NF; ++d)
      {
        f[d] += dpp_f64<kDppXor1>(f[d]);
        f[d] += dpp_f64<kDppXor2>(f[d]);
        f[d] += dpp_f64<kDppHalfMirror>(f[d]);
        fp[d] = dpp_f64<kDppRowRor8>(fkeep[d]);
      }
      if (k == 8)
      {
#pragma unroll
        for (int d = 0; d < NF; ++d) fkeep[d] = f[d];
      }
      else if (k == 0 && wl)
      {
        const int32_t row0 = frow0;
        if (row0 >= 0)
        {
#pragma unroll
          for (int d = 0; d < 3; ++d)
          {
#ifdef FCG_PROBE_TH_NORMW
            if (OVERWRITE)  // timing probe only (wrong f_S): no read-modify-write in the thermal pass
#else
            if (OVERWRITE && !TH)  // the thermal pass adds k_ST (T - T_0) to the structural f_S
#endif
              A.fint[row0 + d] = fp[d] + f[d];
            else
              A.fint[row0 + d] += fp[d] + f[d];
          }
          if (TSI)
          {
            // thermo row of the node = first structural row / 3 (checked at the fused call)
            if (OVERWRITE)
              A.fT[row0 / 3] = fp[NF - 1] + f[NF - 1];
            else
              A.fT[row0 / 3] += fp[NF - 1] + f[NF - 1];
          }
        }
      }
    }
    e_cur = e_nxt;
    __syncthreads();
    FCG_STAMP(1);
  }
  if (A.stamps && tid == 0)
  {
    for (int i = 0; i < 3; ++i) atomicAdd(&A.stamps[i], st_acc[i]);
    atomicAdd(&A.stamps[5], 1ull);
  }
}

}  // namespace

namespace {
SweepArgs sweep_args(const DeviceMesh& m, const double* d_u_col, double* d_K, double* d_fint)
{
  SweepArgs a{};
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
  return a;
}
}  // namespace

#define FCG_SWEEP(KIN)                                                                             \
  if (want_k && m.sweep_defer && overwrite)                                                        \
    hipLaunchKernelGGL((sweep_h8_kernel<KIN, true, true, 3>), grid, block, 0, stream, a);      \
  else if (want_k && m.sweep_defer)                                                                \
    hipLaunchKernelGGL((sweep_h8_kernel<KIN, true, false, 3>), grid, block, 0, stream, a);     \
  else if (want_k && overwrite)                                                                    \
    hipLaunchKernelGGL((sweep_h8_kernel<KIN, true, true, 0>), grid, block, 0, stream, a);      \
  else if (want_k)                                                                                 \
    hipLaunchKernelGGL((sweep_h8_kernel<KIN, true, false, 0>), grid, block, 0, stream, a);     \
  else if (overwrite)                                                                              \
    hipLaunchKernelGGL((sweep_h8_kernel<KIN, false, true, 0>), grid, block, 0, stream, a);     \
  else                                                                                             \
    hipLaunchKernelGGL((sweep_h8_kernel<KIN, false, false, 0>), grid, block, 0, stream, a);

// The TotLag instantiations live in their own translation unit, fcg_sweep_totlag.hip (this file
// with FCG_SWEEP_TOTLAG_TU), compiled without the SLP vectorizer: its pairing of the F / S
// arithmetic into 2-wide vectors costs the TotLag sweep 7-10 % (same-box A/B, 1M hex8: 3.09 ->
// 2.79 ms; profiles/r05/r05_noslp_sweep_ab.txt), while the linear and TSI sweeps gain nothing.
hipError_t launch_sweep_h8_totlag(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream);

#ifdef FCG_SWEEP_TOTLAG_TU
hipError_t launch_sweep_h8_totlag(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream)
{
  const int64_t ntiles = int64_t(m.tiles_x) * m.tiles_y * m.tiles_z;
  if (ntiles == 0) return hipSuccess;
  const SweepArgs a = sweep_args(m, d_u_col, d_K, d_fint);
  const dim3 grid{static_cast<unsigned>(ntiles), 1, 1};
  const dim3 block{256, 1, 1};
  FCG_SWEEP(1)
  return hipGetLastError();
}
#else
hipError_t launch_sweep_h8(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream)
{
  if (m.kinem != 0) return launch_sweep_h8_totlag(m, d_u_col, want_k, overwrite, d_K, d_fint, stream);
  const int64_t ntiles = int64_t(m.tiles_x) * m.tiles_y * m.tiles_z;
  if (ntiles == 0) return hipSuccess;
  const SweepArgs a = sweep_args(m, d_u_col, d_K, d_fint);
  const dim3 grid{static_cast<unsigned>(ntiles), 1, 1};
  const dim3 block{256, 1, 1};
  FCG_SWEEP(0)
  return hipGetLastError();
}

hipError_t launch_sweep_h8_tsi(const DeviceMesh& m, const double* d_u_col, bool overwrite,
    double* d_K, double* d_fint, const SweepTsi& t, hipStream_t stream)
{
  const int64_t ntiles = int64_t(m.tiles_x) * m.tiles_y * m.tiles_z;
  if (ntiles == 0) return hipSuccess;
  SweepArgs a = sweep_args(m, d_u_col, d_K, d_fint);
  a.v_col = t.v_col;
  a.T_col = t.T_col;
  a.Ngp = t.Ngp;
  a.Kst = t.Kst;
  a.Kts = t.Kts;
  a.Ktt = t.Ktt;
  a.fT = t.fT;
  a.tsi_m = t.m;
  a.tsi_T0 = t.T0;
  a.tsi_k = t.conduct;
  a.tsi_kts = t.kts;
  const dim3 grid{static_cast<unsigned>(ntiles), 1, 1};
  const dim3 block{256, 1, 1};
  if (!t.split)
  {
    if (overwrite)
      hipLaunchKernelGGL((sweep_h8_kernel<0, true, true, 1>), grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL((sweep_h8_kernel<0, true, false, 1>), grid, block, 0, stream, a);
    return hipGetLastError();
  }
  // split: the linear structural sweep (K_SS, f_S = K_SS u), then the thermal-only pass
  if (overwrite)
  {
    hipLaunchKernelGGL((sweep_h8_kernel<0, true, true, 0>), grid, block, 0, stream, a);
    hipLaunchKernelGGL((sweep_h8_kernel<0, true, true, 2>), grid, block, 0, stream, a);
  }
  else
  {
    hipLaunchKernelGGL((sweep_h8_kernel<0, true, false, 0>), grid, block, 0, stream, a);
    hipLaunchKernelGGL((sweep_h8_kernel<0, true, false, 2>), grid, block, 0, stream, a);
  }
  return hipGetLastError();
}
#endif  // FCG_SWEEP_TOTLAG_TU
#undef FCG_SWEEP

}  // namespace fcg
