// fcg_hex27.hip -- hex27 StVenantKirchhoff element evaluation + assembly for any mesh (the general
// path of BASELINE config 3's element), redesigned around the FP64 matrix cores and a symmetric
// per-element record.
//
//  h27_element_kernel<KIN, ASM>  256 lanes per workgroup (two per CU) with two elements in
//      flight: wave 3 produces element s while waves 0-2 consume element s - 1 (LDS double
//      buffers, one barrier between the phases, one after).  SolidEleCalc's Gauss-point loop
//      (4C_solid_3D_ele_calc.cpp:110-240, calc_lib.hpp:380-993) in reference coordinates:
//        producer (wave 3):
//        1. J and du/dxi at the 27 Gauss points (dN . X, dN . u), the nodal det J > 0 check
//           (calc_lib.hpp:475-496);
//        2. lanes g: J^-1, fac = det J w (calc_lib.hpp:435-448, 974-993), F = I + du/dX
//           (calc_lib.hpp:579-605), E, StVK S (4C_mat_stvenantkirchhoff.cpp:169-177), and the
//           per-point 3 x 3 factors that let every later stage work on the constant dN_a(xi_g):
//             q_a = T d_a  with T = F J^-1 (linear: J^-1)            (B-operator columns F N_XYZ)
//             fac N_XYZ_a . N_XYZ_b = d_a^T W d_b,  W = fac J^-T J^-1
//             fac N_XYZ_a . S N_XYZ_b = d_a^T V d_b, V = fac J^-T S J^-1
//        and f_a = sum_g R_g d_a, R = fac F S J^-1 (linear: fac S J^-1) (calc_lib.hpp:851-860),
//           written at once;
//        consumers (waves 0-2, one 16 x 16 tile of node pairs each):
//        3. the isotropic StVK blocks of every node pair a <= b (B_a^T C B_b + K_geo,
//           calc_lib.hpp:872-927), all on v_mfma_f64_16x16x4_f64:
//             K_ab = lambda G + mu G^T + mu H + geo I          (linear: mu tr(G) I, no H / geo)
//             G_ij = sum_g fac q_a,i q_b,j                     (K = 27 Gauss points)
//             H = sum_g c_ab(g) F F^T, c_ab = d_a^T W d_b     (one MFMA per point for c,
//                                                                then 24 lane FMAs)
//             geo = sum_g d_a^T V d_b                          (one accumulating MFMA per point,
//                                                                same B operand as c)
//           every operand formed on the fly from the constant dN_a(xi_g) and the per-point
//           factors (no per-(g, a) work arrays);
//        4. K_ab into an LDS image of the element's 378 blocks a <= b, which all four waves write
//           out after the phase barrier.
//      Output (ASM 0): the owned incidences' block rows (3 x 81 + f, the general path's record,
//      read contiguously by assemble27_kernel) -- or, FCG_H27_SYMREC=1, one record per element with
//      the 378 blocks a <= b and f_e for h27_assemble_kernel.  ASM 1/2 (FCG_PATH_COLORED on a
//      verified lattice): pencil order, the blocks added straight into the owned CSR rows.
//  h27_assemble_kernel  SparseMatrix::assemble + LinAlg::assemble (4C_linalg_sparsematrix.cpp:
//      444-576, 4C_linalg_utils_sparse_algebra_assemble.cpp:72-92) for owned rows: one wavefront
//      per owned row node sums the block rows of its incident elements (K_ab or K_ba^T from the
//      records) in element order in an LDS row image and writes its 3 CSR rows once.  Row nodes
//      are visited in the Morton order of their coordinates, so the records that concurrently
//      running wavefronts read stay within a compact piece of the mesh (L2 / Infinity Cache).
// Fixed summation orders everywhere: bitwise reproducible, no atomics on K or f.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "fcg_internal.hpp"
#include "fcg_shape.hpp"

namespace fcg {

namespace {

constexpr int kNpe = 27;
constexpr int kNpair = 378;
constexpr int kBlk = 256;
constexpr int64_t kRec = kH27RecDoubles;  // 378 blocks x 9 | f 27 x 3 | pad
constexpr int64_t kIncRec = record_doubles(kNpe);  // increc: one owned incidence's 3 x 81 block row | f | pad
#ifndef FCG_H27_REC_STORE
#define FCG_H27_REC_STORE 0
#endif

__constant__ double c_dN[27 * 27 * 3];  // dN_c,d at Gauss point g: [g][c][d]
__constant__ double c_w[27];
__constant__ double c_dLn[9];  // 1D Lagrange derivatives at the nodes (fcg_kernels.hip)
__constant__ uint8_t c_loc[27], c_latnode[27];

__device__ inline int pidx(int a, int b)  // a <= b
{
  return 27 * a - (a * (a - 1)) / 2 + b - a;
}

// invert3x3 of the reference (4C_linalg_fixedsizematrix.hpp:1382-1409), column-major m[r + 3c]
__device__ inline double inv3(double* m)
{
  const double t00 = m[4] * m[8] - m[5] * m[7];
  const double t10 = m[2] * m[7] - m[1] * m[8];
  const double t20 = m[1] * m[5] - m[2] * m[4];
  const double det = m[0] * t00 + m[3] * t10 + m[6] * t20;
  if (det == 0.0) return 0.0;
  const double id = 1.0 / det;
  const double t01 = m[3], t11 = m[4], t12 = m[7];
  const double r3 = id * (m[5] * m[6] - t01 * m[8]);
  const double r4 = id * (m[0] * m[8] - m[2] * m[6]);
  const double r7 = id * (m[1] * m[6] - m[0] * t12);
  const double r5 = id * (m[2] * t01 - m[0] * m[5]);
  const double r6 = id * (t01 * t12 - t11 * m[6]);
  const double r8 = id * (m[0] * t11 - m[1] * t01);
  m[3] = r3;
  m[4] = r4;
  m[7] = r7;
  m[5] = r5;
  m[6] = r6;
  m[8] = r8;
  m[0] = id * t00;
  m[1] = id * t10;
  m[2] = id * t20;
  return det;
}

// LDS of one workgroup.  The element pipeline (h27_element_kernel) keeps two elements in flight:
// wave 3 produces element s (its Jacobians in J | Gu, its per-point factors into gpf[s & 1]) while
// waves 0-2 consume element s - 1 from gpf[(s - 1) & 1] into the K image.  Per-point factors:
// T | W | V | M | R (offsets below) and fac.
// Layouts of the factor buffers and of the dN table (TotLag; linear kinematics keep the round-5
// layouts, which measured 7-10 % faster for them: profiles/r06/r06_h27_lds_align_ab.txt).
// T and R take kTs doubles per Gauss point: 10 (9 + a pad) keeps every point's 3 x 3 factor and
// every buffer 16-byte aligned, so that the consumers read them as ds_read_b128 pieces instead of
// ds_read2_b64 pairs (8 LDS cycles per 16 bytes against 4).  dN_c(xi_g): node c's 3 derivatives at
// 4 c + 2 (c >> 3) of its Gauss point's 114-double row (16-byte aligned; nodes c and c + 8 on
// different banks, so that 16 lanes reading 16 nodes' first two derivatives as one ds_read_b128
// each do not conflict).  FCG_H27_GPF9 / FCG_H27_DN3: the round-5 layouts for TotLag too (A/B).
template <int KIN>
struct H27Layout {
#ifdef FCG_H27_GPF9
  static constexpr int kTs = 9;
#else
  static constexpr int kTs = KIN ? 10 : 9;
#endif
  static constexpr int OFF_T = 0, OFF_W = 27 * kTs, OFF_V = OFF_W + 162, OFF_M = OFF_V + 162,
                       OFF_R = OFF_M + 162, GPF = OFF_R + 27 * kTs;
#ifdef FCG_H27_DN3
  static constexpr bool kDnPad = false;
#else
  static constexpr bool kDnPad = KIN == 1;
#endif
  static constexpr int kDnG = kDnPad ? 114 : 81;
  // K image blocks (a <= b), kKs doubles each: 10 for TotLag (16-byte aligned, the record phase
  // reads a block as 4 ds_read_b128 + 1 ds_read_b64); FCG_H27_KIMG9 = rows of 9 (A/B)
#ifdef FCG_H27_KIMG9
  static constexpr int kKs = 9;
#else
  static constexpr int kKs = KIN ? 10 : 9;
#endif
  __device__ __host__ static constexpr int dn_off(int g, int c)
  {
    return kDnPad ? 114 * g + 4 * c + 2 * (c >> 3) : 81 * g + 3 * c;
  }
};
constexpr int kRowImg = 3 * 375;  // one row node's 3 CSR rows (hex27 rows hold <= 375 columns)
template <int KIN>
struct H27Shared {
  using L = H27Layout<KIN>;
  alignas(16) double dN[27 * L::kDnG];  // dN_c,d(xi_g) at dn_off(g, c) + d, loaded once per workgroup
  union {
    struct {
      double X[81], U[81];          // the produced element's coordinates and displacements
      double J[243], Gu[243];       // producer scratch: J, du/dxi per Gauss point
      alignas(16) double gpf[2][L::GPF];           // per-point factors of the produced / consumed element
      double fac[2][27];
      alignas(16) double kimg[kNpair * L::kKs];  // consumed element's blocks a <= b (col-major 3 x 3)
    };
    // overlapped schedule (ASM 3): the row images of the four waves' row nodes, used only while
    // the element pipeline is drained
    double rowimg[4][kRowImg];
  };
  double dLn[9];                // 1D Lagrange derivatives at the nodes (nodal det J check)
  int32_t inc[3][27];           // incidence of (e, a), -1 = not owned, by sequence index mod 3
  // pencil output of the consumed element (by sequence parity): CSR offset of row (a, 0), row
  // length, column position of node b in a's rows, first-holder bits of the pair classes
  int64_t rbase[2][27];
  int32_t rlen[2][27];
  uint16_t ipos[2][27 * 27];
  uint32_t fmask[2];
  uint8_t pcls[27 * 27];        // pair class of (a, b)
  int bad[2];
  int32_t nodal[27];            // nodal det J check of the produced element: 0 | 1 (<= 0) | 2 (= 0)
  uint8_t loc[27], latnode[27];
  int32_t qitem[2];             // ASM 3: work items claimed from the queue (look-ahead slots)
  // views of gpf[b]: T(i, k) at 3i + k, W, V, M symmetric (xx yy zz xy yz zx), R(i, k) at 3i + k
  __device__ double* T(int b) { return gpf[b] + L::OFF_T; }
  __device__ double* W(int b) { return gpf[b] + L::OFF_W; }
  __device__ double* V(int b) { return gpf[b] + L::OFF_V; }
  __device__ double* M(int b) { return gpf[b] + L::OFF_M; }
  __device__ double* R(int b) { return gpf[b] + L::OFF_R; }
};

struct H27Args {
  int64_t n_ele;
  const int32_t* ele_nodes;
  const double* node_x;
  const int32_t* node_dof_col;
  const double* u_col;
  double* rec;
  const int32_t* inc_of;  // increc: [n_ele][27] record slot of (e, a) (the incidence, or its ring
                          // slot under the slab schedule), -1 = a not owned
  int increc;             // 1: per-incidence block rows [slots][246] (assembled by assemble27_kernel)
  int64_t e_end;          // ASM 0: elements [blockIdx.x-th of e_begin.., e_end) (a slab)
  int64_t e_begin;
  int32_t* err;
  double lambda, mu, cdiag;
  int want_k;
  unsigned long long* stamps;  // FCG_STAMPS=1: per-phase s_memtime sums of thread 0, else NULL
  // pencil output (ASM != 0): pencils [pen_begin, pen_end) of one colour, elements col_ele in x
  // order per pencil; the blocks go straight into the owned CSR rows
  const int32_t* col_ele;
  const int64_t* pen_ptr;
  int64_t pen_begin, pen_end;
  const uint32_t* ele_nb;
  const uint16_t* inc_pos;
  const int32_t* inc_row0;
  const int64_t* rowptr;
  double* K;
  double* fint;
  // overlapped schedule (ASM 3): one work queue of element chunks and row items
  const int32_t* queue;      // [n_items]: c >= 0 element chunk c, ~q < 0 row item q
  int64_t n_items;
  int64_t chunk;             // elements per chunk (the last one may be shorter)
  int64_t n_chunks;
  int band_chunks;           // chunks per band (the unit of completion counting)
  unsigned* sync;            // [0] the claim counter, [1 + b] chunks of band b completed (zeroed)
  const int32_t* ritem;      // [n_ritems][4]: rows[j0, j1) and the bands [lo, hi] they need
  const int32_t* rows;       // row nodes by completing band, Morton order inside a band
  const int64_t* rmeta;      // [rows][4]: CSR offset, first row, first incidence, length | n << 16
  const int64_t* inc_ptr;    // row node -> its incidences (record slots)
  const int32_t* rownode_row0;
  int overwrite;
};

typedef double f64x4_t __attribute__((ext_vector_type(4)));

// Pair class of element nodes (a, b): per axis 0 = both on the lower face, 2 = both on the upper
// face, 1 = otherwise; class = t_x + 3 t_y + 9 t_z.  The elements holding both nodes are e
// shifted by the offsets {-1, 0}, {0}, {0, +1} of the three axes.
__device__ inline int pair_class(uint32_t la, uint32_t lb)
{
  int c = 0, m = 1;
#pragma unroll
  for (int d = 0; d < 3; ++d, m *= 3)
  {
    const uint32_t x = (la >> (2 * d)) & 3u, y = (lb >> (2 * d)) & 3u;
    c += m * ((x == y && x != 1u) ? int(x) : 1);
  }
  return c;
}

// Pencil order: colour (ey & 1) + 2 (ez & 1), then x along the pencil.  The first of the present
// holders of a pair class in that order writes (OVERWRITE), the others add.  nb: ele_nb[e].
__device__ inline bool first_holder(int cls, uint32_t nb)
{
  const int t[3] = {cls % 3, (cls / 3) % 3, cls / 9};
  const int py = int((nb >> 27) & 1u), pz = int((nb >> 28) & 1u);
  const int ekey = 4 * (py + 2 * pz) + 1;
  bool first = true;
  for (int dz = (t[2] == 0 ? -1 : 0); dz <= (t[2] == 2 ? 1 : 0); ++dz)
    for (int dy = (t[1] == 0 ? -1 : 0); dy <= (t[1] == 2 ? 1 : 0); ++dy)
      for (int dx = (t[0] == 0 ? -1 : 0); dx <= (t[0] == 2 ? 1 : 0); ++dx)
      {
        if (!((nb >> ((dx + 1) + 3 * (dy + 1) + 9 * (dz + 1))) & 1u)) continue;
        const int key = 4 * (((py + dy) & 1) + 2 * ((pz + dz) & 1)) + dx + 1;
        if (key < ekey) first = false;
      }
  return first;
}

#ifndef FCG_H27_HUNROLL
#define FCG_H27_HUNROLL 3  // unroll of the consumers' H + geo loop over the Gauss points
#endif
#ifndef FCG_H27P_NV
#define FCG_H27P_NV 9  // pencil output: entries in flight per lane
#endif
#ifndef FCG_H27_OVL_STORE
// ASM 3 record stores: 0 write-through (sc1), 1 plain + release fence per chunk, 2 nt + release
#define FCG_H27_OVL_STORE 2
#endif
#ifndef FCG_H27_OVL_NB
#define FCG_H27_OVL_NB 2  // ASM 3 row work: records of a row loaded ahead (the rest when summed)
#endif
constexpr int32_t kQEnd = INT32_MIN;  // ASM 3: the queue is exhausted

// ASM 3 record store: the bytes must reach memory before the chunk's completion count does, so
// that a row node on another XCD (whose L2 is not coherent with this one) reads them
__device__ inline void ovl_store(double* p, double v)
{
#if FCG_H27_OVL_STORE == 0
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store sc1
#elif FCG_H27_OVL_STORE == 1
  *p = v;
#else
  __builtin_nontemporal_store(v, p);
#endif
}

// ASM 3 row work of one wavefront: rows j, j + 4, ... < j1 of ovl_rows (j, j1 and the wave
// uniform).  A row node's three CSR rows from its incidence records (assemble27_kernel's summation:
// incidence order, bitwise the same K and f), the row image in this wave's part of the drained
// pipeline's LDS (a wavefront's LDS operations complete in order: no barrier between the records'
// sums and the read-out).  Pipelined two rows deep: the first NB records of the row after next
// are loaded before this row is summed and written.  Vector-memory instructions complete in issue order, so
// every load and store here is unconditional (clamped addresses, repeated stores of the same value)
// and the compiler's wait for this row's records can leave the next row's loads and this row's
// stores in flight; a row's metadata is one uniform (scalar) load, not a chain of three.
// Lane l takes the record entries d = 2 v2 + h, v2 = l + 64 s2 (double2 pieces): entry d is row
// i = d / 81 of the block row, node b = (d % 81) / 3, component j = d % 3 -- fixed per lane.
__device__ inline void h27_rows(const H27Args& A, int64_t j, int64_t j1, double* acc, int lane_in)
{
  // opaque to the optimiser, so that nothing derived from the lane index is hoisted out of the
  // kernel's loops and held live across the element pipeline
  int lane = lane_in;
  __asm__ volatile("" : "+v"(lane));
  constexpr int NB = FCG_H27_OVL_NB, NV2 = 2;  // NV2 double2 pieces per lane: 122 of the 243 entries
  constexpr int NOUT = (3 * 375 + 63) / 64;   // stores per lane of the longest row node's rows
  struct Meta {
    int64_t base, k0;
    int32_t row0, rowlen, nk;
  };
  struct Recs {
    double2 val[NB][NV2];
    uint32_t pos[NB][NV2];  // the column positions of the lane's two entries, 16 bits each
    double f[NB];
  };
  int32_t ent[NV2][2];  // i | b << 2 | j << 7 of the lane's entry (s2, h), -1 = none
  int v2c[NV2];         // the lane's double2 pieces, clamped into the record
#pragma unroll
  for (int s2 = 0; s2 < NV2; ++s2)
  {
    v2c[s2] = min(lane + 64 * s2, 121);
#pragma unroll
    for (int h = 0; h < 2; ++h)
    {
      const int d = 2 * (lane + 64 * s2) + h;
      ent[s2][h] = d < 243 ? (d / 81) | (((d % 81) / 3) << 2) | ((d % 3) << 7) : -1;
    }
  }
  auto meta = [&](int64_t jj, Meta& M) {
    M.nk = 0;
    M.k0 = 0;
    M.base = 0;
    M.row0 = 0;
    M.rowlen = 1;
    if (jj >= j1) return;
    const int64_t* p = A.rmeta + 4 * jj;
    M.base = p[0];
    M.row0 = int32_t(p[1]);
    M.k0 = p[2];
    M.rowlen = int32_t(p[3] & 0xFFFF);
    M.nk = int32_t(p[3] >> 16);
  };
  // records k0 + q0 + q, q < NB, each address clamped to a valid record (the surplus is not summed)
  auto load = [&](const Meta& M, int q0, Recs& R) {
    const int last = max(M.nk - 1, 0);
#pragma unroll
    for (int q = 0; q < NB; ++q)
    {
      const int64_t k = M.k0 + min(q0 + q, last);
      const double* src = A.rec + k * kIncRec;
      const uint16_t* posb = A.inc_pos + k * kNpe;
      R.f[q] = src[243 + min(lane, 2)];
#pragma unroll
      for (int s2 = 0; s2 < NV2; ++s2)
      {
        R.val[q][s2] = *reinterpret_cast<const double2*>(src + 2 * v2c[s2]);
        const uint32_t p0 = posb[ent[s2][0] < 0 ? 0 : (ent[s2][0] >> 2) & 31];
        const uint32_t p1 = posb[ent[s2][1] < 0 ? 0 : (ent[s2][1] >> 2) & 31];
        R.pos[q][s2] = p0 | (p1 << 16);
      }
    }
  };
  auto add = [&](const Meta& M, int q0, const Recs& R, double& f) {
#pragma unroll
    for (int q = 0; q < NB; ++q)
    {
      if (q0 + q >= M.nk) break;
      f += R.f[q];
      if (!A.want_k) continue;
#pragma unroll
      for (int s2 = 0; s2 < NV2; ++s2)
#pragma unroll
        for (int h = 0; h < 2; ++h)
        {
          const int32_t e = ent[s2][h];
          if (e < 0) continue;
          const int dst = (e & 3) * M.rowlen + int((R.pos[q][s2] >> (16 * h)) & 0xFFFFu) + (e >> 7);
          // one LDS add instruction (ds_add_f64) instead of a read, an add and a write; the
          // lane's entries are distinct addresses, so the sum is the plain one, bitwise
          __hip_atomic_fetch_add(acc + dst, h ? R.val[q][s2].y : R.val[q][s2].x, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
  };
  Meta Mc, Mn, Mnn;
  Recs Rc, Rn, Rnn;
  meta(j, Mc);
  load(Mc, 0, Rc);
  meta(j + 4, Mn);
  load(Mn, 0, Rn);
  for (; Mc.nk > 0; j += 4)
  {
    meta(j + 8, Mnn);
    load(Mnn, 0, Rnn);  // two rows ahead: in flight while this row and the next are done
    const int n3 = 3 * Mc.rowlen;
    if (A.want_k)
#pragma unroll
      for (int t = 0; t < NOUT; ++t) acc[min(lane + 64 * t, n3 - 1)] = 0.0;
    double f = 0.0;
    add(Mc, 0, Rc, f);
    for (int q0 = NB; q0 < Mc.nk; q0 += NB)  // rows with more than NB incidences
    {
      load(Mc, q0, Rc);
      add(Mc, q0, Rc, f);
    }
    if (A.overwrite)
    {
      if (A.want_k)
      {
        double* out = A.K + Mc.base;  // the node's 3 rows are contiguous (checked at setup)
#pragma unroll
        for (int t = 0; t < NOUT; ++t)
        {
          const int v = min(lane + 64 * t, n3 - 1);  // lanes past the end repeat the last entry
          out[v] = acc[v];
        }
      }
      A.fint[Mc.row0 + min(lane, 2)] = f;  // lanes past 2 repeat component 2
    }
    else
    {
      if (A.want_k)
      {
        double* out = A.K + Mc.base;
        for (int v = lane; v < n3; v += 64) out[v] += acc[v];
      }
      if (lane < 3) A.fint[Mc.row0 + lane] += f;
    }
    Mc = Mn;
    Rc = Rn;
    Mn = Mnn;
    Rn = Rnn;
  }
}

// ASM: 0 = records for the row assembly; 1 = pencil order, add into K; 2 = pencil order, the first
// holder writes (OVERWRITE); 3 = the overlapped schedule: records as ASM 0, and the row assembly in
// the same launch.  ASM 3 workgroups take work items in queue order from one claim counter:
// element chunks (runs of consecutive elements through the two-element pipeline, each chunk
// counted complete in its band once its records have reached memory) and row items (a run of row
// nodes whose incident elements all lie in completed bands, one row node per wave as
// assemble27_kernel).  A workgroup that meets a row item drains its pipeline first, so it only
// ever waits for chunks that running workgroups claimed before it: no cycle, no deadlock whatever
// the number of resident workgroups.  The point: one workgroup's element work (latency-bound,
// 1.28x slower alone on a CU than beside a second one) overlaps the other's row work (HBM-bound).
template <int KIN, int ASM>
__global__ __launch_bounds__(kBlk, 2) void h27_element_kernel(H27Args A)
{
  constexpr bool PEN = ASM == 1 || ASM == 2, OVL = ASM == 3;
  __shared__ H27Shared<KIN> sh;
  using L = H27Layout<KIN>;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  for (int v = tid; v < 27 * 27 * 3; v += kBlk) sh.dN[L::dn_off(v / 81, (v % 81) / 3) + v % 3] = c_dN[v];
  if (PEN)
    for (int v = tid; v < 27 * 27; v += kBlk)
    {
      const int a = v / 27;
      sh.pcls[v] = uint8_t(pair_class(c_loc[a], c_loc[v - 27 * a]));
    }
  if (tid < 9)
  {
    sh.dLn[tid] = c_dLn[tid];
  }
  if (tid < 27)
  {
    sh.loc[tid] = c_loc[tid];
    sh.latnode[tid] = c_latnode[tid];
  }
  const double lam = A.lambda, mu = A.mu;

  // the elements of this workgroup, in sequence: e = blockIdx.x + k gridDim.x, or (pencil order)
  // the pencils pen_begin + blockIdx.x + k gridDim.x, each walked in x order.  Every thread walks
  // the same sequence.
  int64_t pen = A.pen_begin + blockIdx.x, pos = -1, pend = -1;
  // ASM 3: the current chunk ends at element ch_end; the next item waits in sh.qitem[qs] (claimed
  // by thread 0 at least one barrier before it is read); stop = the item that ended the pipeline
  int64_t ch_end = -1;
  int qs = 0;
  int32_t item = kQEnd, stop = kQEnd;
  auto claim = [&](int slot) {  // thread 0 only
    const unsigned q = __hip_atomic_fetch_add(&A.sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh.qitem[slot] = int64_t(q) < A.n_items ? A.queue[q] : kQEnd;
  };
  auto first_element = [&]() -> int64_t {
    if (OVL)
    {
      // item: an element chunk; claim the look-ahead item (read when this chunk runs out)
      ch_end = min(A.n_ele, (int64_t(item) + 1) * A.chunk);
      if (tid == 0) claim(qs);
      __syncthreads();
      return int64_t(item) * A.chunk;
    }
    if (!PEN) return A.e_begin + blockIdx.x < A.e_end ? A.e_begin + blockIdx.x : -1;
    if (pen >= A.pen_end) return -1;
    pos = A.pen_ptr[pen];
    pend = A.pen_ptr[pen + 1];
    return A.col_ele[pos];
  };
  bool nx_last = false;  // ASM 3: next_element's argument was the last element of its chunk
  auto next_element = [&](int64_t e) -> int64_t {
    nx_last = false;
    if (e < 0) return -1;
    if (OVL)
    {
      if (e + 1 < ch_end) return e + 1;
      nx_last = true;
      const int32_t x = __builtin_amdgcn_readfirstlane(sh.qitem[qs]);
      qs ^= 1;  // that slot is read: the next claim goes to the other one
      if (x < 0)
      {
        stop = x;  // a row item or the end: the pipeline drains
        return -1;
      }
      ch_end = min(A.n_ele, (int64_t(x) + 1) * A.chunk);
      if (tid == 0) claim(qs);
      return int64_t(x) * A.chunk;
    }
    if (!PEN) return e + gridDim.x < A.e_end ? e + gridDim.x : -1;
    if (++pos < pend) return A.col_ele[pos];
    pen += gridDim.x;
    if (pen >= A.pen_end) return -1;
    pos = A.pen_ptr[pen];
    pend = A.pen_ptr[pen + 1];
    return A.col_ele[pos];
  };

  // X, u and the incidences of an element (evaluate_element_nodes, calc_lib.hpp:180-203), by the
  // producer wave: item t = lane + 64 q of 81 X | 81 u | 27 incidences
  double xu_r[3];
  int32_t inc_r[3];
  auto load_xu = [&](int64_t e) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
    {
      const int t = lane + 64 * q;
      xu_r[q] = 0.0;
      inc_r[q] = -1;
      if (e < 0) continue;
      if (t < 162)
      {
        const int tt = t < 81 ? t : t - 81, a = tt / 3, d = tt - 3 * (tt / 3);
        const int node = A.ele_nodes[e * kNpe + a];
        xu_r[q] = t < 81 ? A.node_x[3 * int64_t(node) + d] : A.u_col[A.node_dof_col[node] + d];
      }
      else if (t < 162 + kNpe && (ASM || A.increc))
        inc_r[q] = A.inc_of[e * kNpe + t - 162];
    }
  };
  auto store_xu = [&](int ib) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
    {
      const int t = lane + 64 * q;
      if (t < 81)
        sh.X[t] = xu_r[q];
      else if (t < 162)
        sh.U[t - 81] = xu_r[q];
      else if (t < 162 + kNpe)
        sh.inc[ib][t - 162] = inc_r[q];
    }
  };
  // LDS written by some lanes of the producer wave and read by others: a wavefront's LDS
  // operations complete in order, so a wait for its own accesses plus a compiler barrier suffice
  auto wave_lds_sync = [&]() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };

  // 1. J and du/dxi at the Gauss points (task t < 162: g, k, X|u) and the nodal det J check
  //    (calc_lib.hpp:475-496, t = 162 + node; code into sh.nodal) via the 1D factors: at a node
  //    they are Kronecker deltas, so J sums the 3 nodes on each parametric line
  auto s1_task = [&](int t) {
    if (t < 162)
    {
      const int g = t / 6, rem = t - 6 * (t / 6);
      const int k = rem % 3, sx = rem / 3;
      const double* src = sx ? sh.U : sh.X;
      const int gdn = g;
      double j0 = 0.0, j1 = 0.0, j2 = 0.0;
#pragma unroll 9
      for (int c = 0; c < kNpe; ++c)
      {
        const double x = src[3 * c + k];
        const double* d = sh.dN + L::dn_off(gdn, c);
        j0 += d[0] * x;
        j1 += d[1] * x;
        j2 += d[2] * x;
      }
      double* dst = (sx ? sh.Gu : sh.J) + 9 * g + 3 * k;
      dst[0] = j0;
      dst[1] = j1;
      dst[2] = j2;
    }
    else if (t < 162 + kNpe)
    {
      const int g = t - 162;
      const uint32_t l = sh.loc[g];
      const int p = l & 3, qq = (l >> 2) & 3, r = l >> 4;
      double J[9];
#pragma unroll
      for (int kk = 0; kk < 9; ++kk) J[kk] = 0.0;
#pragma unroll
      for (int m = 0; m < 3; ++m)
      {
        const double* x0 = sh.X + 3 * sh.latnode[m + 3 * qq + 9 * r];
        const double* x1 = sh.X + 3 * sh.latnode[p + 3 * m + 9 * r];
        const double* x2 = sh.X + 3 * sh.latnode[p + 3 * qq + 9 * m];
        const double d0 = sh.dLn[3 * p + m], d1 = sh.dLn[3 * qq + m], d2 = sh.dLn[3 * r + m];
#pragma unroll
        for (int c = 0; c < 3; ++c)
        {
          J[3 * c + 0] += d0 * x0[c];
          J[3 * c + 1] += d1 * x1[c];
          J[3 * c + 2] += d2 * x2[c];
        }
      }
      const double det = inv3(J);
      sh.nodal[g] = det == 0.0 ? 2 : (!(det > 0) ? 1 : 0);
    }
  };

  // f_a = sum_g R_g d_a (add_internal_force_vector, calc_lib.hpp:851-860) of element e from the
  // factor buffer fb, written at once (a skipped element leaves its rows to the error report)
  auto emit_f = [&](int64_t e, int fb, int ib, uint32_t nbv) {
    if (lane < kNpe && sh.bad[fb] == 0)
    {
      const int a = lane;
      double f0 = 0.0, f1 = 0.0, f2 = 0.0;
#pragma unroll 3
      for (int g = 0; g < kNpe; ++g)
      {
        const double* R = sh.R(fb) + L::kTs * g;
        const double* d = sh.dN + L::dn_off(g, a);
        const double d0 = d[0], d1 = d[1], d2 = d[2];
        f0 += R[0] * d0 + R[1] * d1 + R[2] * d2;
        f1 += R[3] * d0 + R[4] * d1 + R[5] * d2;
        f2 += R[6] * d0 + R[7] * d1 + R[8] * d2;
      }
      const int32_t k = sh.inc[ib][a];
      if (OVL)
      {
        if (k >= 0)
        {
          double* o = A.rec + int64_t(k) * kIncRec + 243;
          ovl_store(o, f0);
          ovl_store(o + 1, f1);
          ovl_store(o + 2, f2);
        }
      }
      else if (PEN)
      {
        if (k >= 0)
        {
          double* o = A.fint + A.inc_row0[k];
          if (ASM == 2 && first_holder(pair_class(sh.loc[a], sh.loc[a]), nbv))
          {
            o[0] = f0;
            o[1] = f1;
            o[2] = f2;
          }
          else
          {
            o[0] += f0;
            o[1] += f1;
            o[2] += f2;
          }
        }
      }
      else if (!A.increc)
      {
        double* o = A.rec + e * kRec + kNpair * 9 + 3 * a;
        o[0] = f0;
        o[1] = f1;
        o[2] = f2;
      }
      else if (k >= 0)
      {
        double* o = A.rec + int64_t(k) * kIncRec + 243;
        o[0] = f0;
        o[1] = f1;
        o[2] = f2;
      }
    }
  };

  // diagnostic phase timers (FCG_STAMPS=1, tools/h27_stamps.py): s_memtime deltas per element,
  // thread 0 (consumer): 0 wait at the top barrier, 1 H + geo, 2 G, 3 K image, 4 barrier + stores;
  // thread 192 (producer): 5 gather + J + Gauss-point algebra + f
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long st_last = A.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
  int64_t st_n = 0;
#define H27_STAMP(i)                                                                               \
  if (A.stamps && (tid == 0 || tid == 192))                                                        \
  {                                                                                                \
    const unsigned long long now = __builtin_amdgcn_s_memtime();                                  \
    st_acc[i] += now - st_last;                                                                    \
    st_last = now;                                                                                 \
  }

  // ASM 3 row item ~it: wait until every chunk of the bands its rows need has been counted (thread
  // 0 polls, bounded: a stuck count is reported as FCG_ERR_DEVICE instead of hanging), one agent
  // acquire for this CU, then the rows, wave w taking rows j0 + w, j0 + w + 4, ...
  auto ovl_rows = [&](int32_t it) {
    const int64_t q = ~int64_t(it);
    const int32_t j0 = A.ritem[4 * q], j1 = A.ritem[4 * q + 1];
    const int32_t blo = A.ritem[4 * q + 2], bhi = A.ritem[4 * q + 3];
    // FCG_STAMPS=1: thread 0's cycles polling (stamps[8]) and in its rows (stamps[9]), row items
    // (stamps[10])
    const unsigned long long t_in = A.stamps && tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
    if (tid == 0)
    {
      for (int32_t b = blo; b <= bhi; ++b)
      {
        const unsigned target = unsigned(min(int64_t(A.band_chunks), A.n_chunks - int64_t(b) * A.band_chunks));
        for (int spin = 0; __hip_atomic_load(&A.sync[1 + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin)
        {
          if (spin == (1 << 22))
          {
            atomicMax(&A.err[0], int32_t(FCG_ERR_DEVICE));
            break;
          }
          __builtin_amdgcn_s_sleep(8);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const unsigned long long t_go = A.stamps && tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
    const int w = __builtin_amdgcn_readfirstlane(wave);  // uniform: the rows' metadata loads are scalar
    h27_rows(A, j0 + w, j1, sh.rowimg[w], lane);
    if (A.stamps && tid == 0)
    {
      atomicAdd(&A.stamps[8], t_go - t_in);
      atomicAdd(&A.stamps[9], __builtin_amdgcn_s_memtime() - t_go);
      atomicAdd(&A.stamps[10], 1ull);
    }
  };

  // ASM 3: the first item
  if (OVL)
  {
    if (tid == 0) claim(0);
    __syncthreads();
    item = __builtin_amdgcn_readfirstlane(sh.qitem[0]);
    qs = 1;
  }
  for (;;)  // ASM 3: one pass per run of element chunks between row items; the others: one pass
  {
    if (OVL)
    {
      // row items until the next element chunk (each claim read after a barrier)
      while (item != kQEnd && item < 0)
      {
        ovl_rows(item);
        if (tid == 0) claim(qs);
        __syncthreads();
        item = __builtin_amdgcn_readfirstlane(sh.qitem[qs]);
        qs ^= 1;
      }
      if (A.stamps) st_last = __builtin_amdgcn_s_memtime();  // row work is not an element phase
      if (item == kQEnd) break;
    }
    // prologue: the first element's X, u, incidences
    int64_t ep = first_element();  // element produced in this iteration (sequence index s)
    if (wave == 3)
    {
      load_xu(ep);
      store_xu(0);
    }
    int64_t ec = -1;                    // element consumed in this iteration (sequence index s - 1)
    int64_t epp = next_element(ep);     // element produced in the next iteration
    bool ep_last = nx_last, ec_last = false;  // ASM 3: ep / ec end their chunk
    for (int s = 0; ec >= 0 || ep >= 0; ++s)
    {
      const int pb = s & 1, cb = pb ^ 1;              // factor buffers of ep, ec
      const int pi = s % 3, ci = (s + 2) % 3, ni = (s + 1) % 3;  // incidence buffers of ep, ec, epp
      __syncthreads();
      H27_STAMP(0);
      const bool cons = ec >= 0 && sh.bad[cb] == 0;
      if (KIN == 0 && ep >= 0)
      {
        // linear kinematics: the producer would be the longer side, so stage 1 of ep runs on all
        // four waves first (wave 3 issues the next element's loads meanwhile)
        if (wave == 3) load_xu(epp);
        s1_task(tid);
        __syncthreads();
      }

      if (wave == 3)
      {
        // ---------------- producer: element ep
        if (ep >= 0)
        {
          ++st_n;
          if (KIN == 1) load_xu(epp);  // lands while ep's stages run; stored after stage 1 has read X, u
          if (lane == 0) sh.bad[pb] = 0;
          // pencil output bookkeeping of ep (read by all waves when ep is consumed)
          const uint32_t nb = PEN ? A.ele_nb[ep] : 0u;
          if (PEN)
          {
            uint32_t ipos_r[12];
#pragma unroll
            for (int q = 0; q < 12; ++q)
            {
              const int v = lane + 64 * q;
              ipos_r[q] = 0u;
              if (v < kNpe * kNpe)
              {
                const int a = v / kNpe;
                const int32_t k = sh.inc[pi][a];
                if (k >= 0) ipos_r[q] = A.inc_pos[int64_t(k) * kNpe + (v - kNpe * a)];
              }
            }
            if (lane < kNpe)
            {
              const int32_t k = sh.inc[pi][lane];
              int64_t rb = 0;
              int32_t rl = 0;
              if (k >= 0)
              {
                const int32_t r0 = A.inc_row0[k];
                rb = A.rowptr[r0];
                rl = int32_t(A.rowptr[r0 + 1] - rb);
              }
              sh.rbase[pb][lane] = rb;
              sh.rlen[pb][lane] = rl;
            }
            if (ASM == 2)
            {
              const uint64_t m = __ballot(lane < 27 && first_holder(lane, nb));
              if (lane == 0) sh.fmask[pb] = uint32_t(m);
            }
#pragma unroll
            for (int q = 0; q < 12; ++q)
            {
              const int v = lane + 64 * q;
              if (v < kNpe * kNpe) sh.ipos[pb][v] = uint16_t(ipos_r[q]);
            }
          }

          // 1. (TotLag: here, by this wave; linear: by all four waves before the phase barrier)
          if (KIN == 1)
          {
#pragma unroll 1
            for (int q = 0; q < 3; ++q) s1_task(lane + 64 * q);
            wave_lds_sync();
          }
          if (lane < kNpe && sh.nodal[lane] != 0) atomicMax(&sh.bad[pb], sh.nodal[lane]);
          wave_lds_sync();

          // 2. per Gauss point: J^-1, fac, strains, StVK stress and the folded 3 x 3 factors
          if (lane < kNpe)
          {
            const int g = lane;
            double iJ[9];
#pragma unroll
            for (int kk = 0; kk < 9; ++kk) iJ[kk] = sh.J[9 * g + kk];
            const double det = inv3(iJ);
            if (det == 0.0) atomicMax(&sh.bad[pb], 2);
            const double fac = det * c_w[g];
            sh.fac[pb][g] = fac;
            // grad u: Hu(i, j) = du_i / dX_j = sum_k J^-1(j, k) du_i / dxi_k
            double Hu[3][3];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int j = 0; j < 3; ++j)
                Hu[i][j] = iJ[j] * sh.Gu[9 * g + 3 * i] + iJ[j + 3] * sh.Gu[9 * g + 3 * i + 1] +
                           iJ[j + 6] * sh.Gu[9 * g + 3 * i + 2];
            double E[6], F[3][3];
            if (KIN == 0)
            {
              // evaluate_linear_gl_strain (calc_lib.hpp:682-695): engineering shear
              E[0] = Hu[0][0];
              E[1] = Hu[1][1];
              E[2] = Hu[2][2];
              E[3] = Hu[0][1] + Hu[1][0];
              E[4] = Hu[1][2] + Hu[2][1];
              E[5] = Hu[0][2] + Hu[2][0];
#pragma unroll
              for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) F[i][j] = i == j ? 1.0 : 0.0;
            }
            else
            {
              // F = I + u N_XYZ^T (hex27, calc_lib.hpp:579-605); F^-1 must exist (calc_lib.hpp:562)
#pragma unroll
              for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) F[i][j] = Hu[i][j] + (i == j ? 1.0 : 0.0);
              double Fi[9];
#pragma unroll
              for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) Fi[i + 3 * j] = F[i][j];
              if (inv3(Fi) == 0.0) atomicMax(&sh.bad[pb], 2);
              // C = F^T F, E = (C - I) / 2 in strain-like Voigt form (calc_lib.hpp:639-676)
              double C[3][3];
#pragma unroll
              for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) C[i][j] = F[0][i] * F[0][j] + F[1][i] * F[1][j] + F[2][i] * F[2][j];
              E[0] = 0.5 * (C[0][0] - 1.0);
              E[1] = 0.5 * (C[1][1] - 1.0);
              E[2] = 0.5 * (C[2][2] - 1.0);
              E[3] = C[0][1];
              E[4] = C[1][2];
              E[5] = C[0][2];
            }
            // S = C E (fill_cmat, 4C_mat_stvenantkirchhoff.cpp:115-145)
            double S[3][3];
            S[0][0] = A.cdiag * E[0] + A.lambda * (E[1] + E[2]);
            S[1][1] = A.cdiag * E[1] + A.lambda * (E[0] + E[2]);
            S[2][2] = A.cdiag * E[2] + A.lambda * (E[0] + E[1]);
            S[0][1] = S[1][0] = A.mu * E[3];
            S[1][2] = S[2][1] = A.mu * E[4];
            S[0][2] = S[2][0] = A.mu * E[5];
            // T = F J^-1, R = fac F S J^-1
            double FS[3][3];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int j = 0; j < 3; ++j) FS[i][j] = F[i][0] * S[0][j] + F[i][1] * S[1][j] + F[i][2] * S[2][j];
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int k = 0; k < 3; ++k)
              {
                sh.T(pb)[L::kTs * g + 3 * i + k] = F[i][0] * iJ[3 * k] + F[i][1] * iJ[3 * k + 1] + F[i][2] * iJ[3 * k + 2];
                sh.R(pb)[L::kTs * g + 3 * i + k] =
                    fac * (FS[i][0] * iJ[3 * k] + FS[i][1] * iJ[3 * k + 1] + FS[i][2] * iJ[3 * k + 2]);
              }
            if (KIN == 1)
            {
              // W = fac J^-T J^-1, V = fac J^-T S J^-1, M = F F^T  (xx yy zz xy yz zx)
              double SJ[3][3];  // S J^-1
#pragma unroll
              for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int l = 0; l < 3; ++l) SJ[i][l] = S[i][0] * iJ[3 * l] + S[i][1] * iJ[3 * l + 1] + S[i][2] * iJ[3 * l + 2];
              const int kk[6] = {0, 1, 2, 0, 1, 0}, ll[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
              for (int x = 0; x < 6; ++x)
              {
                const int k = kk[x], l = ll[x];
                // J^-1(j, k) = iJ[j + 3 k]
                sh.W(pb)[6 * g + x] = fac * (iJ[3 * k] * iJ[3 * l] + iJ[3 * k + 1] * iJ[3 * l + 1] + iJ[3 * k + 2] * iJ[3 * l + 2]);
                sh.V(pb)[6 * g + x] = fac * (iJ[3 * k] * SJ[0][l] + iJ[3 * k + 1] * SJ[1][l] + iJ[3 * k + 2] * SJ[2][l]);
                sh.M(pb)[6 * g + x] = F[k][0] * F[l][0] + F[k][1] * F[l][1] + F[k][2] * F[l][2];
              }
            }
          }
          wave_lds_sync();
          store_xu(ni);  // stage 1 has read X, u: the next element's take their place

          emit_f(ep, pb, pi, nb);
        }
        H27_STAMP(5);
      }
      else if (cons && A.want_k)
      {
        // ---------------- consumers (waves 0-2): element ec's node-pair blocks on the matrix cores.
        // Wave w takes the node ranges (0,0), (0,1), (1,1) of 16; lane (r16, kq) feeds A[r16][kq]
        // and B[kq][r16] and holds D[kq + 4 r][r16], r = 0..3.  Operands come from the constant
        // dN_a(xi_g) and the per-point 3 x 3 factors at clamped indices, always loaded and masked by
        // multiplication (a load under a lane condition turns into a branch with its own wait).
        const int at = wave == 2 ? 1 : 0, bt = wave == 0 ? 0 : 1;
        const int r16 = lane & 15, kq = lane >> 4;
        const int a_l = 16 * at + r16, b_l = 16 * bt + r16;
        const bool va = a_l < 27, vb = b_l < 27;
        const int a_c = va ? a_l : 0, b_c = vb ? b_l : 0;
        const f64x4_t zero4 = {0.0, 0.0, 0.0, 0.0};
        const int b = 16 * bt + r16;

        // 3. TotLag: mu H + geo I.  Per Gauss point one MFMA over k (K = 3, padded to 4) gives
        //    c_ab = d_a^T W d_b, and H += c_ab M_g on the lanes; a second MFMA with the same B operand
        //    accumulates geo_ab += d_a^T V d_b in its C input.  Both go into the K image at once, so
        //    that stage 4 holds only G.
        if (KIN == 1)
        {
          f64x4_t Hm[6];  // H per component (xx yy zz xy yz zx)
#pragma unroll
          for (int k = 0; k < 6; ++k) Hm[k] = zero4;
          f64x4_t Geo = zero4;
          const bool vk = kq < 3;
          const int kc = vk ? kq : 0;
          const double ma = (va && vk) ? 1.0 : 0.0, mb = (vb && vk) ? 1.0 : 0.0;
          const int wr0 = kc == 0 ? 0 : (kc == 1 ? 3 : 5), wr1 = kc == 0 ? 3 : (kc == 1 ? 1 : 4),
                    wr2 = kc == 0 ? 5 : (kc == 1 ? 4 : 2);  // row kc of the symmetric W, V
#pragma unroll FCG_H27_HUNROLL
          for (int g = 0; g < kNpe; ++g)
          {
            const double* da = sh.dN + L::dn_off(g, a_c);
            const double* Wg = sh.W(cb) + 6 * g;
            const double* Vg = sh.V(cb) + 6 * g;
            const double d0 = da[0], d1 = da[1], d2 = da[2];
            const double av = (Wg[wr0] * d0 + Wg[wr1] * d1 + Wg[wr2] * d2) * ma;
            const double avv = (Vg[wr0] * d0 + Vg[wr1] * d1 + Vg[wr2] * d2) * ma;
            const double bv = sh.dN[L::dn_off(g, b_c) + kc] * mb;
            const f64x4_t c = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, zero4, 0, 0, 0);
            Geo = __builtin_amdgcn_mfma_f64_16x16x4f64(avv, bv, Geo, 0, 0, 0);
            const double* Mg = sh.M(cb) + 6 * g;
#pragma unroll
            for (int x = 0; x < 6; ++x)
            {
              const double m = Mg[x];
#pragma unroll
              for (int r = 0; r < 4; ++r) Hm[x][r] += c[r] * m;
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r)
          {
            const int a = 16 * at + kq + 4 * r;
            if (a < 27 && b < 27 && a <= b)
            {
              double* K = sh.kimg + L::kKs * pidx(a, b);
              const double geo = Geo[r];
              K[0] = mu * Hm[0][r] + geo;
              K[4] = mu * Hm[1][r] + geo;
              K[8] = mu * Hm[2][r] + geo;
              K[1] = K[3] = mu * Hm[3][r];
              K[5] = K[7] = mu * Hm[4][r];
              K[2] = K[6] = mu * Hm[5][r];
            }
          }
        }
        H27_STAMP(1);

        // 4. G_ij = sum_g fac q_a,i q_b,j (7 steps of 4 Gauss points; q_a = T_g d_a on the fly)
        f64x4_t X[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) X[k] = zero4;
#pragma unroll
        for (int st = 0; st < 7; ++st)
        {
          const int g = 4 * st + kq;
          const bool vg = g < 27;
          const int gc = vg ? g : 0;
          const double fg = sh.fac[cb][gc] * ((vg && va) ? 1.0 : 0.0);
          const double mb = (vg && vb) ? 1.0 : 0.0;
          const double* T = sh.T(cb) + L::kTs * gc;
          const double* da = sh.dN + L::dn_off(gc, a_c);
          const double* db = sh.dN + L::dn_off(gc, b_c);
          const double a0 = da[0], a1 = da[1], a2 = da[2], b0 = db[0], b1 = db[1], b2 = db[2];
          double av[3], bv[3];
#pragma unroll
          for (int i = 0; i < 3; ++i)
          {
            const double t0 = T[3 * i], t1 = T[3 * i + 1], t2 = T[3 * i + 2];
            av[i] = fg * (t0 * a0 + t1 * a1 + t2 * a2);
            bv[i] = mb * (t0 * b0 + t1 * b1 + t2 * b2);
          }
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
              X[3 * i + j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], X[3 * i + j], 0, 0, 0);
        }
        H27_STAMP(2);

        // 5. K_ab = lambda G + mu G^T + (mu tr G I | mu H + geo I) into the LDS image, which leaves
        //    as contiguous pieces: one store instruction covers 1 KB instead of 64 scattered entries
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
          const int a = 16 * at + kq + 4 * r;
          if (a < 27 && b < 27 && a <= b)
          {
            double* K = sh.kimg + L::kKs * pidx(a, b);
            double add[9];
            if (KIN == 0)
            {
              const double tr = mu * (X[0][r] + X[4][r] + X[8][r]);
#pragma unroll
              for (int k = 0; k < 9; ++k) add[k] = (k == 0 || k == 4 || k == 8) ? tr : 0.0;
            }
            else
            {
#pragma unroll
              for (int k = 0; k < 9; ++k) add[k] = K[k];  // mu H + geo I from stage 3
            }
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int j = 0; j < 3; ++j)
                K[i + 3 * j] = lam * X[3 * i + j][r] + mu * X[3 * j + i][r] + add[i + 3 * j];
          }
        }
        H27_STAMP(3);
      }
      __syncthreads();

      // 6. element ec's record(s) or rows, by all waves
      if (ec >= 0 && sh.bad[cb] != 0)
      {
        if (tid == 0)
        {
          atomicMax(&A.err[0], sh.bad[cb]);
          atomicMin(&A.err[1], int32_t(ec));
        }
      }
      else if (cons && A.want_k)
      {
        if (PEN)
        {
          // straight into the owned rows: entry v = (a, i, c) of a's 3 rows over the 81 columns in
          // lattice order (c / 3 = lattice node, so lanes v, v + 1 hit contiguous CSR columns in runs
          // of 3 nodes); every load of a batch is issued before its stores.  The pencil's previous
          // element wrote its shared rows in the previous iteration, from this workgroup.
          constexpr int NV = FCG_H27P_NV;
          const uint32_t fmask = sh.fmask[cb];
          for (int v0 = 0; v0 < kNpe * 243; v0 += NV * kBlk)
          {
            int64_t addr[NV];
            double val[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k)
            {
              const int v = v0 + tid + kBlk * k;
              addr[k] = -1;
              val[k] = 0.0;
              if (v >= kNpe * 243) continue;
              const int a = v / 243;
              if (sh.inc[ci][a] < 0) continue;
              const int r = v - 243 * a;
              const int i = r / 81, c = r - 81 * (r / 81);
              const int b = sh.latnode[c / 3], j = c - 3 * (c / 3);
              addr[k] = sh.rbase[cb][a] + int64_t(i * sh.rlen[cb][a] + sh.ipos[cb][kNpe * a + b] + j);
              const bool up = a <= b;
              val[k] = sh.kimg[L::kKs * (up ? pidx(a, b) : pidx(b, a)) + (up ? i + 3 * j : j + 3 * i)];
              if (ASM == 1 || !((fmask >> sh.pcls[kNpe * a + b]) & 1u)) val[k] += A.K[addr[k]];
            }
#pragma unroll
            for (int k = 0; k < NV; ++k)
              if (addr[k] >= 0) A.K[addr[k]] = val[k];
          }
        }
        else if (A.increc)
        {
          // the owned incidences' block rows K_ab, b = 0..26 (K_ba^T for b < a), row-major 3 x 81:
          // the record of the general path's assemble27_kernel.  One (a, b) block per lane: its 9
          // entries from the image, then 3 pieces of 3 into the rows (lanes b, b + 1 contiguous)
          for (int p = tid; p < kNpe * kNpe; p += kBlk)
          {
            const int a = p / kNpe, b = p - kNpe * a;
            const int32_t k = sh.inc[ci][a];
            if (k < 0) continue;
            const bool up = a <= b;
            const double* src = sh.kimg + L::kKs * (up ? pidx(a, b) : pidx(b, a));
            double v[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) v[q] = src[q];  // col-major K_(min,max)
            double* dst = A.rec + int64_t(k) * kIncRec + 3 * b;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int j = 0; j < 3; ++j)
              {
                if (OVL)
                  ovl_store(dst + 81 * i + j, up ? v[i + 3 * j] : v[j + 3 * i]);
                else
#if FCG_H27_REC_STORE == 0  // streamed (nt): read once, by the row assembly
                  __builtin_nontemporal_store(up ? v[i + 3 * j] : v[j + 3 * i], dst + 81 * i + j);
#else  // plain: the pieces of a line meet in L2 before it is written back
                  dst[81 * i + j] = up ? v[i + 3 * j] : v[j + 3 * i];
#endif
              }
          }
        }
        else
        {
          if constexpr (L::kKs == 9)
          {
            const double2* src = reinterpret_cast<const double2*>(sh.kimg);
            double2* dst = reinterpret_cast<double2*>(A.rec + ec * kRec);  // 16-byte aligned (kRec even)
            for (int v = tid; v < kNpair * 9 / 2; v += kBlk) dst[v] = src[v];
          }
          else
          {
            double* dst = A.rec + ec * kRec;  // the record keeps 9 doubles per block
            for (int v = tid; v < kNpair * 9; v += kBlk) dst[v] = sh.kimg[L::kKs * (v / 9) + v % 9];
          }
        }
      }
      // ASM 3: ec ended its chunk -- once every wave's record stores (and the producer's f stores,
      // issued an iteration earlier) have reached memory, the chunk counts in its band
      if (OVL && ec >= 0 && ec_last)
      {
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
        {
#if FCG_H27_OVL_STORE != 0
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
          const int64_t band = ec / A.chunk / A.band_chunks;
          __hip_atomic_fetch_add(&A.sync[1 + band], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      H27_STAMP(4);
      ec = ep;
      ec_last = ep_last;
      ep = epp;
      epp = next_element(epp);
      ep_last = nx_last;
    }
    if (!OVL) break;
    item = stop;  // a row item or the end
  }
  if (A.stamps && (tid == 0 || tid == 192))
  {
    if (tid == 0)
      for (int i = 0; i < 5; ++i) atomicAdd(&A.stamps[i], st_acc[i]);
    else
    {
      atomicAdd(&A.stamps[5], st_acc[5]);
      atomicAdd(&A.stamps[7], (unsigned long long)st_n);
    }
    if (tid == 0) atomicAdd(&A.stamps[6], 1ull);
  }
#undef H27_STAMP
}

struct H27AsmArgs {
  int64_t n_rownodes;
  const int32_t* order;  // row nodes in Morton order
  const int64_t* inc_ptr;
  const int32_t* inc_ele;
  const uint8_t* inc_a;
  const uint16_t* inc_pos;
  const int32_t* rownode_row0;
  const int64_t* rowptr;
  const double* rec;
  double* K;
  double* fint;
};

template <bool WANT_K, bool OVERWRITE>
__global__ __launch_bounds__(64) void h27_assemble_kernel(H27AsmArgs A)
{
  constexpr int NS = 4;  // 243 entries of a node's block row (3 rows x 27 nodes x 3) over 64 lanes
  constexpr int NB = 3;  // incidences in flight
  __shared__ double acc[WANT_K ? 3 * 375 : 1];
  const int lane = threadIdx.x;
  // Entry t of incidence (e, a), lanes reading consecutive record addresses:
  //   t <  9 (27 - a): the contiguous blocks (a, b >= a) from pidx(a, a) on, K_ab col-major;
  //   t >= 9 (27 - a): block (b, a) of b = (t - 9 (27 - a)) / 9 < a, read transposed (K_ab = K_ba^T).
  struct Inc {
    double val[NS];
    int off[NS];
    double f;
  };
  auto load = [&](int64_t k, int rowlen, Inc& c) {
    const int64_t e = A.inc_ele[k];
    const int a = A.inc_a[k];
    const double* src = A.rec + e * kRec;
    const uint16_t* pos = A.inc_pos + k * kNpe;
    const int n1 = 9 * (27 - a), p0 = 9 * pidx(a, a);
    c.f = lane < 3 ? src[kNpair * 9 + 3 * a + lane] : 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s)
    {
      const int t = lane + 64 * s;
      c.val[s] = 0.0;
      c.off[s] = -1;
      if (!WANT_K || t >= 243) continue;
      int addr, b, i, j;
      if (t < n1)
      {
        const int q = t / 9, kk = t - 9 * q;
        b = a + q;
        i = kk % 3;
        j = kk / 3;
        addr = p0 + t;
      }
      else
      {
        const int tt = t - n1, q = tt / 9, kk = tt - 9 * q;
        b = q;
        i = kk / 3;
        j = kk % 3;
        addr = 9 * pidx(b, a) + kk;
      }
      c.val[s] = src[addr];
      c.off[s] = i * rowlen + pos[b] + j;
    }
  };
  // XCD-contiguous work: workgroup b runs on XCD b % 8 (round-robin dispatch); XCD x walks its
  // own eighth of the Morton order, its workgroups interleaved, so that the row nodes in flight on
  // one XCD are a compact piece of the mesh and the records they share stay in that XCD's L2
  const int xcd = int(blockIdx.x & 7u);
  const int64_t per_xcd = (int64_t(gridDim.x) + 7 - xcd) / 8;
  const int64_t chunk = (A.n_rownodes + 7) / 8;
  const int64_t x0 = min(A.n_rownodes, int64_t(xcd) * chunk), x1 = min(A.n_rownodes, x0 + chunk);
  for (int64_t it = x0 + (blockIdx.x >> 3); it < x1; it += per_xcd)
  {
    const int64_t r = A.order ? A.order[it] : it;
    const int32_t row0 = A.rownode_row0[r];
    const int64_t base = A.rowptr[row0];
    const int rowlen = int(A.rowptr[row0 + 1] - base);
    if (WANT_K)
      for (int v = lane; v < 3 * rowlen; v += 64) acc[v] = 0.0;
    double f = 0.0;
    const int64_t k0 = A.inc_ptr[r], k1 = A.inc_ptr[r + 1];
    Inc ring[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q)
      if (k0 + q < k1) load(k0 + q, rowlen, ring[q]);
    for (int64_t k = k0; k < k1; k += NB)
    {
#pragma unroll
      for (int q = 0; q < NB; ++q)
      {
        if (k + q >= k1) break;
        Inc& c = ring[q];
        if (WANT_K)
#pragma unroll
          for (int s = 0; s < NS; ++s)
            if (c.off[s] >= 0) acc[c.off[s]] += c.val[s];
        f += c.f;
        if (k + q + NB < k1) load(k + q + NB, rowlen, c);
      }
    }
    __syncthreads();
    if (WANT_K)
    {
      double* out = A.K + base;  // the node's 3 rows are contiguous (checked at setup)
      for (int v = lane; v < 3 * rowlen; v += 64)
      {
        if (OVERWRITE)
          out[v] = acc[v];
        else
          out[v] += acc[v];
      }
    }
    if (lane < 3)
    {
      if (OVERWRITE)
        A.fint[row0 + lane] = f;
      else
        A.fint[row0 + lane] += f;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Matrix-free tangent action y = K(u) x (fcg_tangent_apply): the operator the assembled tangent
// of this element would apply, B^T C B + K_geo over the Gauss points (calc_lib.hpp:872-927),
// without forming the element or global matrix.  At Gauss point g with H = grad_X x:
//   linear  P = fac C sym(H)                                  (F = I, no geometric part)
//   TotLag  P = fac (F C sym(F^T H) + H S),  S = C E(u)       (material + geometric part)
// and y_a = sum_g P N_XYZ_a = sum_g (P J^-1) dN_a(xi_g) -- the same folding as f_a = sum_g R_g d_a
// in emit_f.  One workgroup pass takes kApE elements: lanes (element, Gauss point) form J,
// du/dxi and dx/dxi from the element's nodal X | u | x in LDS and the shape derivatives built
// from the 1-D Lagrange factors of their point (registers, no table reads), then Q = P J^-1 into
// LDS; lanes (element, node) sum Q_g dN_a(xi_g) over the points and write y_a at the node's
// incidence; h27_inc_sum_kernel adds a row node's incidences in incidence order.  Per element
// 81 + 81 doubles of X, u (TotLag) and x are read instead of the 6,561 stored entries an SpMV
// with the assembled element matrices reads.
constexpr int kApE = 9;  // elements per workgroup pass (243 of 256 lanes)
__constant__ double c_L1[9], c_dL1[9];  // 1-D Lagrange L_p(x_m), L'_p(x_m) at the rule's points: [3 m + p]

struct H27ApplyArgs {
  int64_t n_ele;
  const int32_t* ele_nodes;
  const double* node_x;
  const int32_t* node_dof_col;
  const double* u_col;
  const double* x_col;
  const int32_t* inc_of;
  const int32_t* ele_dof;  // [n_ele][27] column LID of each element node's first DOF
  double* ye;  // [n_inc + 1][3] (the last triple: target of the unowned nodes' stores)
  int64_t n_inc;
  double lambda, mu, cdiag;
};

template <int KIN>
__global__ __launch_bounds__(256, 2) void h27_apply_kernel(H27ApplyArgs A)
{
  __shared__ double nd[kApE][3][81];  // X | u | x of the pass's elements (node-major xyz)
  __shared__ double Qs[kApE][27][9];  // Q = P J^-1 per Gauss point, row-major 3 x 3
  __shared__ double tL[9], tdL[9];    // c_L1, c_dL1
  __shared__ uint8_t lat[27];         // node (= Gauss point) at lattice position i0 + 3 i1 + 9 i2
  const int tid = threadIdx.x;
  if (tid < 9)
  {
    tL[tid] = c_L1[tid];
    tdL[tid] = c_dL1[tid];
  }
  if (tid < 27) lat[tid] = c_latnode[tid];
  const bool act = tid < 27 * kApE;
  const int s = tid / 27, g = tid - 27 * s;  // (element slot, Gauss point | node)
  // lattice position of this lane's Gauss point g (gauss phase) = of its node a = g (node phase)
  const uint32_t pg = c_loc[act ? g : 0];
  const int p0 = pg & 3, p1 = (pg >> 2) & 3, p2 = pg >> 4;
  const double w = c_w[act ? g : 0];
  const double lam = A.lambda, mu = A.mu, cd = A.cdiag;
  constexpr int NSRC = KIN == 0 ? 2 : 3;  // X | x (linear) or X | u | x
  constexpr int NLD = (kApE * 81 * NSRC + 255) / 256;
  double pre[NLD];
  auto load = [&](int64_t e0) {
#pragma unroll
    for (int q = 0; q < NLD; ++q)
    {
      const int t = tid + 256 * q;
      pre[q] = 0.0;
      if (t >= kApE * 81 * NSRC) continue;
      const int sl = t / (81 * NSRC), r = t - 81 * NSRC * sl;
      const int src = r / 81, rr = r - 81 * src, a = rr / 3, d = rr - 3 * a;
      const int64_t e = e0 + sl;
      if (e0 < 0 || e >= A.n_ele) continue;
      const int32_t node = A.ele_nodes[e * 27 + a];
      const double* base = src == 0 ? A.node_x : (src == NSRC - 1 ? A.x_col : A.u_col);
      pre[q] = src == 0 ? base[3 * int64_t(node) + d] : base[A.node_dof_col[node] + d];
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int q = 0; q < NLD; ++q)
    {
      const int t = tid + 256 * q;
      if (t >= kApE * 81 * NSRC) continue;
      const int sl = t / (81 * NSRC), r = t - 81 * NSRC * sl;
      const int src = r / 81, rr = r - 81 * src;
      nd[sl][src == NSRC - 1 ? 2 : src][rr] = pre[q];
    }
  };
  const int64_t stride = int64_t(gridDim.x) * kApE;
  int64_t e0 = int64_t(blockIdx.x) * kApE;
  load(e0 < A.n_ele ? e0 : -1);
  for (; e0 < A.n_ele; e0 += stride)
  {
    store();
    __syncthreads();
    load(e0 + stride < A.n_ele ? e0 + stride : -1);  // next pass's gathers in flight
    const int64_t e = e0 + s;
    if (act && e < A.n_ele)
    {
      // J (col-major, J[d + 3k] = dX_k/dxi_d), du_i/dxi_d and dx_i/dxi_d at point g.  Nodes by
      // lattice position (i0, i1, i2): the 1-D factors of the point along x in registers, along y
      // and z read per (i1, i2); the products in shape_deriv's order (fcg_shape.hpp), so dN is
      // the element kernel's table value bit for bit.
      double J[9], Gu[9], Gx[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) J[q] = Gu[q] = Gx[q] = 0.0;
      double Lx[3], dLx[3];
#pragma unroll
      for (int i = 0; i < 3; ++i)
      {
        Lx[i] = tL[3 * p0 + i];
        dLx[i] = tdL[3 * p0 + i];
      }
#pragma unroll 1
      for (int i12 = 0; i12 < 9; ++i12)
      {
        const int i1 = i12 % 3, i2 = i12 / 3;
        const double Ly = tL[3 * p1 + i1], dLy = tdL[3 * p1 + i1];
        const double Lz = tL[3 * p2 + i2], dLz = tdL[3 * p2 + i2];
        const double yz = Ly * Lz;
#pragma unroll
        for (int i0 = 0; i0 < 3; ++i0)
        {
          const int c = lat[i0 + 3 * i12];
          const double d0 = yz * dLx[i0];
          const double d1 = Lx[i0] * Lz * dLy;
          const double d2 = Lx[i0] * Ly * dLz;
#pragma unroll
          for (int k = 0; k < 3; ++k)
          {
            const double xk = nd[s][0][3 * c + k], vk = nd[s][2][3 * c + k];
            J[3 * k + 0] += d0 * xk;
            J[3 * k + 1] += d1 * xk;
            J[3 * k + 2] += d2 * xk;
            Gx[3 * k + 0] += d0 * vk;
            Gx[3 * k + 1] += d1 * vk;
            Gx[3 * k + 2] += d2 * vk;
            if (KIN == 1)
            {
              const double uk = nd[s][1][3 * c + k];
              Gu[3 * k + 0] += d0 * uk;
              Gu[3 * k + 1] += d1 * uk;
              Gu[3 * k + 2] += d2 * uk;
            }
          }
        }
      }
      double iJ[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) iJ[q] = J[q];
      const double fac = inv3(iJ) * w;  // det == 0 was reported by the evaluate of this state
      // grad_X of x and u: H(i, j) = sum_k J^-1(j, k) d(.)_i / dxi_k
      double Hx[3][3], F[3][3];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
        {
          Hx[i][j] = iJ[j] * Gx[3 * i] + iJ[j + 3] * Gx[3 * i + 1] + iJ[j + 6] * Gx[3 * i + 2];
          F[i][j] = KIN == 0 ? 0.0
                             : iJ[j] * Gu[3 * i] + iJ[j + 3] * Gu[3 * i + 1] + iJ[j + 6] * Gu[3 * i + 2];
        }
      double P[3][3];
      auto cmat = [&](const double* ev, double Sm[3][3]) {  // S = C e (fill_cmat), e engineering Voigt
        Sm[0][0] = cd * ev[0] + lam * (ev[1] + ev[2]);
        Sm[1][1] = cd * ev[1] + lam * (ev[0] + ev[2]);
        Sm[2][2] = cd * ev[2] + lam * (ev[0] + ev[1]);
        Sm[0][1] = Sm[1][0] = mu * ev[3];
        Sm[1][2] = Sm[2][1] = mu * ev[4];
        Sm[0][2] = Sm[2][0] = mu * ev[5];
      };
      if (KIN == 0)
      {
        const double ev[6] = {Hx[0][0], Hx[1][1], Hx[2][2], Hx[0][1] + Hx[1][0], Hx[1][2] + Hx[2][1],
                              Hx[0][2] + Hx[2][0]};
        double dS[3][3];
        cmat(ev, dS);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) P[i][j] = fac * dS[i][j];
      }
      else
      {
#pragma unroll
        for (int i = 0; i < 3; ++i) F[i][i] += 1.0;
        double C[3][3], Ah[3][3];  // C = F^T F, Ah = F^T H
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
          {
            C[i][j] = F[0][i] * F[0][j] + F[1][i] * F[1][j] + F[2][i] * F[2][j];
            Ah[i][j] = F[0][i] * Hx[0][j] + F[1][i] * Hx[1][j] + F[2][i] * Hx[2][j];
          }
        const double E[6] = {0.5 * (C[0][0] - 1.0), 0.5 * (C[1][1] - 1.0), 0.5 * (C[2][2] - 1.0),
                             C[0][1], C[1][2], C[0][2]};
        const double dE[6] = {Ah[0][0], Ah[1][1], Ah[2][2], Ah[0][1] + Ah[1][0], Ah[1][2] + Ah[2][1],
                              Ah[0][2] + Ah[2][0]};
        double S[3][3], dS[3][3];
        cmat(E, S);
        cmat(dE, dS);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            P[i][j] = fac * (F[i][0] * dS[0][j] + F[i][1] * dS[1][j] + F[i][2] * dS[2][j] +
                             Hx[i][0] * S[0][j] + Hx[i][1] * S[1][j] + Hx[i][2] * S[2][j]);
      }
      double* Q = Qs[s][g];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k)
          Q[3 * i + k] = P[i][0] * iJ[3 * k] + P[i][1] * iJ[3 * k + 1] + P[i][2] * iJ[3 * k + 2];
    }
    __syncthreads();
    if (act && e < A.n_ele)
    {
      // node a = g at lattice position (p0, p1, p2): y_a = sum_g Q_g dN_a(xi_g), the points by
      // lattice position (m0, m1, m2), dN_a(xi_g) from L_{p_d}(x_{m_d}) = tL[3 m_d + p_d]
      const int32_t k = A.inc_of[e * 27 + g];
      double La0[3], dLa0[3];
#pragma unroll
      for (int m = 0; m < 3; ++m)
      {
        La0[m] = tL[3 * m + p0];
        dLa0[m] = tdL[3 * m + p0];
      }
      double y0 = 0.0, y1 = 0.0, y2 = 0.0;
#pragma unroll 1
      for (int m12 = 0; m12 < 9; ++m12)
      {
        const int m1 = m12 % 3, m2 = m12 / 3;
        const double Ly = tL[3 * m1 + p1], dLy = tdL[3 * m1 + p1];
        const double Lz = tL[3 * m2 + p2], dLz = tdL[3 * m2 + p2];
        const double yz = Ly * Lz;
#pragma unroll
        for (int m0 = 0; m0 < 3; ++m0)
        {
          const double d0 = yz * dLa0[m0];
          const double d1 = La0[m0] * Lz * dLy;
          const double d2 = La0[m0] * Ly * dLz;
          const double* Q = Qs[s][lat[m0 + 3 * m12]];
          y0 += Q[0] * d0 + Q[1] * d1 + Q[2] * d2;
          y1 += Q[3] * d0 + Q[4] * d1 + Q[5] * d2;
          y2 += Q[6] * d0 + Q[7] * d1 + Q[8] * d2;
        }
      }
      if (k >= 0)
      {
        double* o = A.ye + 3 * int64_t(k);
        o[0] = y0;
        o[1] = y1;
        o[2] = y2;
      }
    }
  }
}

// The same action sum-factorised over the tensor-product structure of hex27 (the default; the
// kernel above stays as FCG_H27_APPLY=direct).  With L_p(x_m), L'_p(x_m) the 1-D factors and
// nodes / points by lattice position:
//   gradients  lanes (element, point line (m1, m2), source X | u | x): per component the node
//              values contracted over (i1, i2) with L L, L' L, L L' of the line, then over i0 with
//              L' | L | L for the three points of the line -- 108 FMA per component and line
//              instead of 243;
//   points     lanes (element, point): J, F, S, P and Q = P J^-1 from the gradients in LDS;
//   nodes      lanes (element, node line (a1, a2), component i): Q contracted over (m1, m2) with
//              the line's factors, then over m0 for the line's three nodes -- 99 FMA instead of 729.
// Four barriers per pass (Q reuses the nodal values' LDS).
template <int KIN, int BT, int NE>
__global__ __launch_bounds__(BT, BT == 64 ? 2 : 2) void h27_apply_sf_kernel(H27ApplyArgs A)
{
  // BT = 64: one wavefront holds whole elements (NE = 2, 54 of 64 lanes) and its phases are
  // ordered by the wavefront's in-order LDS accesses, no workgroup barrier; BT = 256: NE = 9
  // elements, the phases separated by __syncthreads
  auto phase_sync = [&]() {
    if constexpr (BT == 64)
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else
      __syncthreads();
  };
  constexpr int NSRC = KIN == 0 ? 2 : 3;  // X | x (linear) or X | u | x
#ifdef FCG_H27_APPLY_OLD
  // A/B probe: the round-5 layouts (node-major values, Q[g][3 x 3], 9 NSRC doubles per point),
  // read as ds_read2_b64 pairs
  constexpr int NND = 81 * NSRC > 243 ? 81 * NSRC : 243;
  constexpr int kGs = 9 * NSRC, kSs = 9;
  auto nv = [](int src, int k, int l) { return 81 * src + 3 * l + k; };  // nodal value
  auto qv = [](int g, int i, int k) { return 9 * g + 3 * i + k; };        // Q_ik at point g
#else
  // component-major: the 27 nodal values of one (source, component) and the 27 points' Q_ik are
  // contiguous and 16-byte aligned rows of 28, and a point's gradients take 30 doubles (TotLag), so
  // that the phases read ds_read_b128 pieces (4 LDS cycles per 16 bytes) instead of ds_read2_b64
  // pairs (8) -- conflict-free for the lane groups of each phase
  constexpr int NND = 252;
  // (sources 10 apart, every 3 x 3 block 16-byte aligned with 22 / 30 per point: 2 % slower for
  // TotLag, linear the same; profiles/r06/r06_h27_lds_align_ab.txt)
  constexpr int kGs = NSRC == 3 ? 30 : 18, kSs = 9;
  auto nv = [](int src, int k, int l) { return 84 * src + 28 * k + l; };
  auto qv = [](int g, int i, int k) { return 28 * (3 * i + k) + g; };
#endif
  __shared__ alignas(16) double nq[NE][NND];      // nodal X | (u) | x, then Q
  __shared__ alignas(16) double gr[NE][27 * kGs];  // d(src)_k / dxi_d at point l: l kGs + kSs src + 3 k + d
  __shared__ double tL[9], tdL[9], wl[27];
  __shared__ uint8_t lat[27], posl[27];  // lattice position -> node (= point) number, and back
  __shared__ int32_t incs[NE][27];        // the pass's incidences of (element, node), -1 = unowned
  // every LDS array is indexed by lattice position l = p0 + 3 p1 + 9 p2 (nodes and points alike)
  const int tid = threadIdx.x;
  if (tid < 9)
  {
    tL[tid] = c_L1[tid];
    tdL[tid] = c_dL1[tid];
  }
  if (tid < 27)
  {
    lat[tid] = c_latnode[tid];
    const uint32_t pc = c_loc[tid];
    posl[tid] = uint8_t((pc & 3) + 3 * ((pc >> 2) & 3) + 9 * (pc >> 4));
    wl[tid] = c_w[c_latnode[tid]];
  }
  const double lam = A.lambda, mu = A.mu, cd = A.cdiag;
  constexpr int NLD = (NE * 81 * NSRC + BT - 1) / BT;
  // the gathers in two stages, one pass apart, so that no wait on a dependent load falls inside a
  // pass: stage 1 reads the element's node / DOF index of each item for the pass after next
  // (ele_nodes, apply_dof: independent loads), stage 2 the values for the next pass at the
  // indices stage 1 read one pass earlier
  double pre[NLD];
  int32_t ix1[NLD];
  // Every gather is unconditional (a clamped address; validity is re-derived from the pass's
  // first element where the value is consumed), so each pass issues a fixed number of memory
  // operations and the compiler's wait before a use can skip what was issued after it.  Per
  // pass: value_of for the next pass (at the indices index_of loaded one pass earlier), then
  // index_of for the pass after next, then the compute phases and the node stores.
  auto item_ok = [&](int t, int64_t e0) {
    return t < NE * 81 * NSRC && e0 >= 0 && e0 + t / (81 * NSRC) < A.n_ele;
  };
  auto index_of = [&](int64_t e0, int32_t* ix) {
#pragma unroll
    for (int q = 0; q < NLD; ++q)
    {
      int t = tid + BT * q;
      __asm__ volatile("" : "+v"(t));  // index math per pass, not hoisted into live registers
      const int sl = t / (81 * NSRC), r = t - 81 * NSRC * sl;
      const int src = r / 81, a = (r - 81 * src) / 3;
      const int64_t e = item_ok(t, e0) ? e0 + sl : 0;
      const int32_t* tab = src == 0 ? A.ele_nodes : A.ele_dof;
      ix[q] = tab[e * 27 + (t < NE * 81 * NSRC ? a : 0)];
    }
  };
  int32_t incp = 0;  // lane < 27 NE: incidence of (element, node) of the next pass
  auto value_of = [&](const int32_t* ix, int64_t e0n) {
    {
      const int sl = tid / 27;
      const bool ok = tid < 27 * NE && e0n >= 0 && e0n + sl < A.n_ele;
      incp = A.inc_of[ok ? (e0n + sl) * 27 + tid - 27 * sl : 0];
    }
#pragma unroll
    for (int q = 0; q < NLD; ++q)
    {
      int t = tid + BT * q;
      __asm__ volatile("" : "+v"(t));
      const int r = t - 81 * NSRC * (t / (81 * NSRC));
      const int src = r / 81, d = r - 81 * src - 3 * ((r - 81 * src) / 3);
      const double* base = src == 0 ? A.node_x : (src == NSRC - 1 ? A.x_col : A.u_col);
      const int32_t at = (src == 0 ? 3 * ix[q] : ix[q]) + d;
      pre[q] = base[item_ok(t, e0n) ? at : 0];
    }
  };
  // lane roles: gradients (s, line, src), points (s, g), nodes (s, line, i)
  const int s27 = tid / 27, r27 = tid - 27 * s27;
  const int sg = tid / (9 * NSRC), rg = tid - 9 * NSRC * sg;
  // XCD-contiguous passes: workgroup b runs on XCD b % 8 (round-robin dispatch); XCD x takes its
  // own eighth of the element chunks, its workgroups interleaved, so that elements sharing nodes
  // are gathered through one L2
  const int64_t nch = (A.n_ele + NE - 1) / NE;
  const int xcd = int(blockIdx.x & 7u);
  const int64_t per_xcd = (int64_t(gridDim.x) + 7 - xcd) / 8;
  const int64_t span = (nch + 7) / 8;
  const int64_t c0 = min(nch, int64_t(xcd) * span), c1 = min(nch, c0 + span);
  auto first_of = [&](int64_t c) { return c < c1 ? c * NE : int64_t(-1); };
  int64_t ch = c0 + (blockIdx.x >> 3);
  index_of(first_of(ch), ix1);
  value_of(ix1, first_of(ch));
  index_of(first_of(ch + per_xcd), ix1);
  int64_t e0pre = first_of(ch);  // the pass whose values sit in pre / incp
  for (; ch < c1; ch += per_xcd)
  {
    const int64_t e0 = ch * NE;
    phase_sync();  // the previous pass's node phase has read Q
#pragma unroll
    for (int q = 0; q < NLD; ++q)
    {
      const int t = tid + BT * q;
      if (t < NE * 81 * NSRC)
      {
        const int sl = t / (81 * NSRC), r = t - 81 * NSRC * sl;
        const int src = r / 81, rr = r - 81 * src, a = rr / 3;
        nq[sl][nv(src, rr - 3 * a, posl[a])] = pre[q];
      }
    }
    if (tid < 27 * NE) incs[tid / 27][tid - 27 * (tid / 27)] = incp;
    phase_sync();
    e0pre = first_of(ch + per_xcd);
    value_of(ix1, e0pre);                        // next pass: values at last pass's indices
    index_of(first_of(ch + 2 * per_xcd), ix1);  // pass after next: indices
    // ---- gradients at the points of line (m1, m2), one source
    if (sg < NE && e0 + sg < A.n_ele)
    {
      const int line = rg / NSRC, src = rg - NSRC * (rg / NSRC);
      const int m1 = line % 3, m2 = line / 3;
      double f0[9], f1[9], f2[9];  // L L, L' L, L L' of (i1, i2)
#pragma unroll
      for (int i2 = 0; i2 < 3; ++i2)
#pragma unroll
        for (int i1 = 0; i1 < 3; ++i1)
        {
          const double ly = tL[3 * m1 + i1], dly = tdL[3 * m1 + i1];
          const double lz = tL[3 * m2 + i2], dlz = tdL[3 * m2 + i2];
          f0[i1 + 3 * i2] = ly * lz;
          f1[i1 + 3 * i2] = dly * lz;
          f2[i1 + 3 * i2] = ly * dlz;
        }
      double lx[3][3], dlx[3][3];  // [m0][i0]
#pragma unroll
      for (int m0 = 0; m0 < 3; ++m0)
#pragma unroll
        for (int i0 = 0; i0 < 3; ++i0)
        {
          lx[m0][i0] = tL[3 * m0 + i0];
          dlx[m0][i0] = tdL[3 * m0 + i0];
        }
#pragma unroll
      for (int j = 0; j < 9; ++j)
        __asm__ volatile("" : "+v"(f0[j]), "+v"(f1[j]), "+v"(f2[j]));  // rebuilt per pass, not kept live
#pragma unroll 1
      for (int k = 0; k < 3; ++k)
      {
        const double* v = nq[sg] + nv(src, k, 0);
        double w0[3] = {0.0, 0.0, 0.0}, w1[3] = {0.0, 0.0, 0.0}, w2[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < 9; ++j)
#pragma unroll
          for (int i0 = 0; i0 < 3; ++i0)
          {
            const double x = v[nv(0, 0, i0 + 3 * j)];
            w0[i0] += f0[j] * x;
            w1[i0] += f1[j] * x;
            w2[i0] += f2[j] * x;
          }
#pragma unroll
        for (int m0 = 0; m0 < 3; ++m0)
        {
          double* o = gr[sg] + kGs * (m0 + 3 * line) + kSs * src + 3 * k;
          o[0] = dlx[m0][0] * w0[0] + dlx[m0][1] * w0[1] + dlx[m0][2] * w0[2];
          o[1] = lx[m0][0] * w1[0] + lx[m0][1] * w1[1] + lx[m0][2] * w1[2];
          o[2] = lx[m0][0] * w2[0] + lx[m0][1] * w2[1] + lx[m0][2] * w2[2];
        }
      }
    }
    phase_sync();
    // ---- point algebra: lanes (s27, g)
    if (s27 < NE && e0 + s27 < A.n_ele)
    {
      const int g = r27;  // lattice position of the point
      const double* G = gr[s27] + kGs * g;
      double iJ[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) iJ[q] = G[q];  // [k][d] row-major = J[d + 3k] col-major
      const double fac = inv3(iJ) * wl[g];
      const double* Gx = G + kSs * (NSRC - 1);
      double Hx[3][3], F[3][3];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
        {
          Hx[i][j] = iJ[j] * Gx[3 * i] + iJ[j + 3] * Gx[3 * i + 1] + iJ[j + 6] * Gx[3 * i + 2];
          F[i][j] = KIN == 0 ? 0.0
                             : iJ[j] * G[kSs + 3 * i] + iJ[j + 3] * G[kSs + 3 * i + 1] + iJ[j + 6] * G[kSs + 3 * i + 2];
        }
      double P[3][3];
      auto cmat = [&](const double* ev, double Sm[3][3]) {
        Sm[0][0] = cd * ev[0] + lam * (ev[1] + ev[2]);
        Sm[1][1] = cd * ev[1] + lam * (ev[0] + ev[2]);
        Sm[2][2] = cd * ev[2] + lam * (ev[0] + ev[1]);
        Sm[0][1] = Sm[1][0] = mu * ev[3];
        Sm[1][2] = Sm[2][1] = mu * ev[4];
        Sm[0][2] = Sm[2][0] = mu * ev[5];
      };
      if (KIN == 0)
      {
        const double ev[6] = {Hx[0][0], Hx[1][1], Hx[2][2], Hx[0][1] + Hx[1][0], Hx[1][2] + Hx[2][1],
                              Hx[0][2] + Hx[2][0]};
        double dS[3][3];
        cmat(ev, dS);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) P[i][j] = fac * dS[i][j];
      }
      else
      {
#pragma unroll
        for (int i = 0; i < 3; ++i) F[i][i] += 1.0;
        double C[3][3], Ah[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
          {
            C[i][j] = F[0][i] * F[0][j] + F[1][i] * F[1][j] + F[2][i] * F[2][j];
            Ah[i][j] = F[0][i] * Hx[0][j] + F[1][i] * Hx[1][j] + F[2][i] * Hx[2][j];
          }
        const double E[6] = {0.5 * (C[0][0] - 1.0), 0.5 * (C[1][1] - 1.0), 0.5 * (C[2][2] - 1.0),
                             C[0][1], C[1][2], C[0][2]};
        const double dE[6] = {Ah[0][0], Ah[1][1], Ah[2][2], Ah[0][1] + Ah[1][0], Ah[1][2] + Ah[2][1],
                              Ah[0][2] + Ah[2][0]};
        double S[3][3], dS[3][3];
        cmat(E, S);
        cmat(dE, dS);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            P[i][j] = fac * (F[i][0] * dS[0][j] + F[i][1] * dS[1][j] + F[i][2] * dS[2][j] +
                             Hx[i][0] * S[0][j] + Hx[i][1] * S[1][j] + Hx[i][2] * S[2][j]);
      }
      double* Q = nq[s27];  // the nodal values are dead: the gradients are in gr
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k)
          Q[qv(g, i, k)] = P[i][0] * iJ[3 * k] + P[i][1] * iJ[3 * k + 1] + P[i][2] * iJ[3 * k + 2];
    }
    phase_sync();
    // ---- node lines: lanes (s27, line (a1, a2), component i)
    if (s27 < NE && e0 + s27 < A.n_ele)
    {
      const int line = r27 / 3, i = r27 - 3 * (r27 / 3);
      const int a1 = line % 3, a2 = line / 3;
      const double* Q = nq[s27];
      double z0[3] = {0.0, 0.0, 0.0}, z12[3] = {0.0, 0.0, 0.0};
      // fully unrolled (was unroll 1): -1.2 % per action, no spills (profiles/r06/r06_apply_z_unroll_ab.txt)
#pragma unroll
      for (int m2 = 0; m2 < 3; ++m2)
#pragma unroll
        for (int m1 = 0; m1 < 3; ++m1)
        {
          const double ly = tL[3 * m1 + a1], dly = tdL[3 * m1 + a1];
          const double lz = tL[3 * m2 + a2], dlz = tdL[3 * m2 + a2];
          const double c0 = ly * lz, c1 = dly * lz, c2 = ly * dlz;
#pragma unroll
          for (int m0 = 0; m0 < 3; ++m0)
          {
            const int m = m0 + 3 * m1 + 9 * m2;
            z0[m0] += c0 * Q[qv(m, i, 0)];
            z12[m0] += c1 * Q[qv(m, i, 1)] + c2 * Q[qv(m, i, 2)];
          }
        }
#pragma unroll
      for (int a0 = 0; a0 < 3; ++a0)
      {
        const int a = lat[a0 + 3 * line];
        const int32_t k = incs[s27][a];
        const double y = tdL[a0] * z0[0] + tdL[3 + a0] * z0[1] + tdL[6 + a0] * z0[2] +
                         tL[a0] * z12[0] + tL[3 + a0] * z12[1] + tL[6 + a0] * z12[2];
        // unconditional (an unowned node's value goes to the spare triple): a static store count
        // per pass lets the next pass's wait skip these stores
        A.ye[3 * (k >= 0 ? int64_t(k) : A.n_inc) + i] = y;
      }
    }
  }
}

// apply_dof[e][a] = node_dof_col[ele_nodes[e][a]] (the matrix-free action's gather plan)
__global__ __launch_bounds__(256) void h27_apply_plan_kernel(int64_t n, const int32_t* __restrict__ ele_nodes,
    const int32_t* __restrict__ node_dof_col, int32_t* __restrict__ out)
{
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = node_dof_col[ele_nodes[i]];
}

// y_row of each owned row node = the sum of its incidences' parts in incidence order
__global__ __launch_bounds__(256) void h27_inc_sum_kernel(int64_t n_rownodes,
    const int64_t* __restrict__ inc_ptr, const int32_t* __restrict__ rownode_row0,
    const double* __restrict__ ye, double* __restrict__ y)
{
  const int64_t r = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= n_rownodes) return;
  double y0 = 0.0, y1 = 0.0, y2 = 0.0;
  const int64_t p0 = inc_ptr[r], p1 = inc_ptr[r + 1];
  const int64_t cnt = p1 - p0;
#ifndef FCG_PROBE_INCSUM_LOOP
  // the first 8 incidences (a lattice node's most) loaded unconditionally -- addresses clamped to
  // the node's last one, all 24 loads in flight at once -- and summed in order by selects
  // (bit-identical to the loop); a node with more incidences continues in the loop
  double v[8][3];
#pragma unroll
  for (int j = 0; j < 8; ++j)
  {
    const int64_t k = p0 + (j < cnt ? j : (cnt > 0 ? cnt - 1 : 0));  // ye has a spare last triple
    v[j][0] = ye[3 * k];
    v[j][1] = ye[3 * k + 1];
    v[j][2] = ye[3 * k + 2];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
  {
    y0 = j < cnt ? y0 + v[j][0] : y0;
    y1 = j < cnt ? y1 + v[j][1] : y1;
    y2 = j < cnt ? y2 + v[j][2] : y2;
  }
  for (int64_t k = p0 + 8; k < p1; ++k)
#else
  for (int64_t k = p0; k < p1; ++k)
#endif
  {
    y0 += ye[3 * k];
    y1 += ye[3 * k + 1];
    y2 += ye[3 * k + 2];
  }
  const int32_t row0 = rownode_row0[r];
  y[row0] = y0;
  y[row0 + 1] = y1;
  y[row0 + 2] = y2;
}

}  // namespace

void upload_h27_tables()
{
  static bool done = false;
  if (done) return;
  double xi[81], w[27];
  gauss_rule(kHex27, xi, w);
  double dN[27 * 27 * 3];
  for (int g = 0; g < 27; ++g) shape_deriv(kHex27, &xi[3 * g], &dN[81 * g]);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dN), dN, sizeof(dN));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_w), w, sizeof(w));
  // 1D quadratic Lagrange derivatives L_i'(x_p) at the nodes x = -1, 0, 1 (as fcg_kernels.hip)
  double dLn[9];
  for (int p = 0; p < 3; ++p)
  {
    const double t = double(p - 1);
    dLn[3 * p + 0] = t - 0.5;
    dLn[3 * p + 1] = -2.0 * t;
    dLn[3 * p + 2] = t + 0.5;
  }
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dLn), dLn, sizeof(dLn));
  // 1-D factors at the rule's points (the same r as gauss_rule, the same L / dL as shape_deriv)
  double L1[9], dL1[9];
  for (int m = 0; m < 3; ++m)
  {
    const double r = xi[3 * (m == 0 ? 0 : (m == 1 ? 8 : 1))];  // points 0, 8, 1: x = -a, 0, +a
    L1[3 * m + 0] = 0.5 * r * (r - 1.0);
    L1[3 * m + 1] = 1.0 - r * r;
    L1[3 * m + 2] = 0.5 * r * (r + 1.0);
    dL1[3 * m + 0] = r - 0.5;
    dL1[3 * m + 1] = -2.0 * r;
    dL1[3 * m + 2] = r + 0.5;
  }
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_L1), L1, sizeof(L1));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dL1), dL1, sizeof(dL1));
  uint8_t loc[27], latnode[27];
  for (int a = 0; a < 27; ++a)
  {
    loc[a] = uint8_t(kHex27NodePos[a][0] | (kHex27NodePos[a][1] << 2) | (kHex27NodePos[a][2] << 4));
    latnode[kHex27NodePos[a][0] + 3 * kHex27NodePos[a][1] + 9 * kHex27NodePos[a][2]] = uint8_t(a);
  }
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_loc), loc, sizeof(loc));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_latnode), latnode, sizeof(latnode));
  done = true;
}

hipError_t launch_h27_element(const DeviceMesh& m, const double* d_u_col, bool want_k,
    hipStream_t stream, int64_t e_begin, int64_t e_end)
{
  if (e_end < 0) e_end = m.n_ele;
  const int64_t n = e_end - e_begin;
  if (n <= 0) return hipSuccess;
  H27Args a{};
  a.n_ele = m.n_ele;
  a.e_begin = e_begin;
  a.e_end = e_end;
  a.ele_nodes = m.ele_nodes;
  a.node_x = m.node_x;
  a.node_dof_col = m.node_dof_col;
  a.u_col = d_u_col;
  a.rec = m.scratch;
  a.inc_of = m.h27_slot ? m.h27_slot : m.inc_of;  // slab schedule: the ring slot of each incidence
  a.increc = m.h27_increc ? 1 : 0;
  a.err = m.err;
  a.lambda = m.lambda;
  a.mu = m.mu;
  a.cdiag = m.cdiag;
  a.want_k = want_k ? 1 : 0;
  a.stamps = m.stamps;
  // the whole mesh: 4 workgroups per CU queued (2 resident); a slab: at most the resident ones,
  // so that every workgroup keeps several elements in its two-element pipeline
  const int64_t cap = m.h27_nslab > 1 ? m.h27_el_grid : 256 * 8;
  const dim3 grid(unsigned(n < cap ? n : cap)), block(kBlk);
  // FCG_H27_DYNLDS=<bytes>: unused dynamic LDS per workgroup (occupancy probes: 20000 leaves one
  // resident workgroup per CU)
  static const unsigned dyn = [] {
    const char* e = std::getenv("FCG_H27_DYNLDS");
    return e ? unsigned(std::atoi(e)) : 0u;
  }();
  if (m.kinem == 0)
    hipLaunchKernelGGL((h27_element_kernel<0, 0>), grid, block, dyn, stream, a);
  else
    hipLaunchKernelGGL((h27_element_kernel<1, 0>), grid, block, dyn, stream, a);
  return hipGetLastError();
}

// hex27 overlapped schedule (DeviceMesh::ovl_*): element chunks and row items of one queue in one
// launch of the resident workgroups; the claim counter and the band counts are zeroed first
hipError_t launch_h27_overlap(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream)
{
  if (m.n_ele == 0 && m.n_rownodes == 0) return hipSuccess;
  hipError_t he = hipMemsetAsync(m.ovl_sync, 0, sizeof(unsigned) * size_t(1 + m.ovl_nbands), stream);
  if (he != hipSuccess) return he;
  H27Args a{};
  a.n_ele = m.n_ele;
  a.e_begin = 0;
  a.e_end = m.n_ele;
  a.ele_nodes = m.ele_nodes;
  a.node_x = m.node_x;
  a.node_dof_col = m.node_dof_col;
  a.u_col = d_u_col;
  a.rec = m.scratch;
  a.inc_of = m.inc_of;
  a.increc = 1;
  a.err = m.err;
  a.lambda = m.lambda;
  a.mu = m.mu;
  a.cdiag = m.cdiag;
  a.want_k = want_k ? 1 : 0;
  a.stamps = m.stamps;
  a.inc_pos = m.inc_pos;
  a.rowptr = m.rowptr;
  a.K = d_K;
  a.fint = d_fint;
  a.queue = m.ovl_queue;
  a.n_items = m.ovl_items;
  a.chunk = m.ovl_chunk;
  a.n_chunks = m.ovl_nchunks;
  a.band_chunks = m.ovl_band_chunks;
  a.sync = m.ovl_sync;
  a.ritem = m.ovl_ritem;
  a.rows = m.ovl_rows;
  a.rmeta = m.ovl_rmeta;
  a.inc_ptr = m.inc_ptr;
  a.rownode_row0 = m.rownode_row0;
  a.overwrite = overwrite ? 1 : 0;
  const dim3 grid(unsigned(std::max(1, m.h27_el_grid))), block(kBlk);
  if (m.kinem == 0)
    hipLaunchKernelGGL((h27_element_kernel<0, 3>), grid, block, 0, stream, a);
  else
    hipLaunchKernelGGL((h27_element_kernel<1, 3>), grid, block, 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_h27_pencil(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream)
{
  if (m.n_ele == 0) return hipSuccess;
  H27Args a{};
  a.n_ele = m.n_ele;
  a.ele_nodes = m.ele_nodes;
  a.node_x = m.node_x;
  a.node_dof_col = m.node_dof_col;
  a.u_col = d_u_col;
  a.rec = nullptr;
  a.inc_of = m.inc_of;
  a.increc = 0;
  a.err = m.err;
  a.lambda = m.lambda;
  a.mu = m.mu;
  a.cdiag = m.cdiag;
  a.want_k = want_k ? 1 : 0;
  a.stamps = m.stamps;
  a.col_ele = m.col_ele;
  a.pen_ptr = m.pen_ptr;
  a.ele_nb = m.ele_nb;
  a.inc_pos = m.inc_pos;
  a.inc_row0 = m.inc_row0;
  a.rowptr = m.rowptr;
  a.K = d_K;
  a.fint = d_fint;
  // one workgroup per pencil (two resident per CU); the pencils of a colour have equal lengths
  // on a box, so the hardware's dispatch balances them
  const int64_t cap = int64_t(1) << 30;
  for (int c = 0; c < 4; ++c)
  {
    a.pen_begin = m.pen_color[c];
    a.pen_end = m.pen_color[c + 1];
    const int64_t n = a.pen_end - a.pen_begin;
    if (n == 0) continue;
    const dim3 grid(unsigned(n < cap ? n : cap)), block(kBlk);
#define FCG_H27P(KIN)                                                                              \
  if (overwrite)                                                                                   \
    hipLaunchKernelGGL((h27_element_kernel<KIN, 2>), grid, block, 0, stream, a);                   \
  else                                                                                             \
    hipLaunchKernelGGL((h27_element_kernel<KIN, 1>), grid, block, 0, stream, a);
    if (m.kinem == 0)
    {
      FCG_H27P(0)
    }
    else
    {
      FCG_H27P(1)
    }
#undef FCG_H27P
    const hipError_t he = hipGetLastError();
    if (he != hipSuccess) return he;
  }
  return hipSuccess;
}

hipError_t launch_h27_assemble(const DeviceMesh& m, bool want_k, bool overwrite, double* d_K,
    double* d_fint, hipStream_t stream)
{
  if (m.n_rownodes == 0) return hipSuccess;
  H27AsmArgs a{};
  a.n_rownodes = m.n_rownodes;
  a.order = m.asm_order;
  a.inc_ptr = m.inc_ptr;
  a.inc_ele = m.inc_ele;
  a.inc_a = m.inc_a;
  a.inc_pos = m.inc_pos;
  a.rownode_row0 = m.rownode_row0;
  a.rowptr = m.rowptr;
  a.rec = m.scratch;
  a.K = d_K;
  a.fint = d_fint;
  // a multiple of the 8 XCDs; 512 wavefronts in flight per XCD keep its records' working set
  // near its 4 MB L2 (FCG_H27_ASM_GRID overrides, for A/B runs)
  static const int64_t cap = [] {
    const char* e = std::getenv("FCG_H27_ASM_GRID");
    return e ? std::max<int64_t>(8, std::atoll(e) / 8 * 8) : int64_t(4096);
  }();
  const int64_t want = std::min<int64_t>(cap, (m.n_rownodes + 7) / 8 * 8);
  const dim3 grid(unsigned(std::max<int64_t>(8, want))), block(64);
  if (want_k && overwrite)
    hipLaunchKernelGGL((h27_assemble_kernel<true, true>), grid, block, 0, stream, a);
  else if (want_k)
    hipLaunchKernelGGL((h27_assemble_kernel<true, false>), grid, block, 0, stream, a);
  else if (overwrite)
    hipLaunchKernelGGL((h27_assemble_kernel<false, true>), grid, block, 0, stream, a);
  else
    hipLaunchKernelGGL((h27_assemble_kernel<false, false>), grid, block, 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_h27_apply_plan(const DeviceMesh& m, hipStream_t stream)
{
  const int64_t n = m.n_ele * 27;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(h27_apply_plan_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, stream,
      n, m.ele_nodes, m.node_dof_col, m.apply_dof);
  return hipGetLastError();
}

hipError_t launch_h27_apply(const DeviceMesh& m, const double* d_u_col, const double* d_x_col,
    double* d_y_row, hipStream_t stream)
{
  if (m.n_ele > 0)
  {
    H27ApplyArgs a{};
    a.n_ele = m.n_ele;
    a.ele_nodes = m.ele_nodes;
    a.node_x = m.node_x;
    a.node_dof_col = m.node_dof_col;
    a.u_col = d_u_col;
    a.x_col = d_x_col;
    a.inc_of = m.inc_of;
    a.ele_dof = m.apply_dof;
    a.ye = m.apply_ye;
    a.n_inc = m.n_inc;
    a.lambda = m.lambda;
    a.mu = m.mu;
    a.cdiag = m.cdiag;
    const int64_t passes = (m.n_ele + kApE - 1) / kApE;
    // persistent: two resident workgroups per CU (LDS), so that each XCD's workgroups walk its
    // element range together (FCG_H27_APPLY_GRID overrides, for A/B runs)
    static const int64_t cap = [] {
      const char* e = std::getenv("FCG_H27_APPLY_GRID");
      return e ? std::max<int64_t>(8, std::atoll(e)) : int64_t(256 * 2);
    }();
    const dim3 grid(unsigned(std::min<int64_t>(passes, cap))), block(256);
    // FCG_H27_APPLY=direct: the per-point kernel without sum factorisation (A/B runs)
    // FCG_H27_APPLY=sf: the 256-lane sum-factorised kernel (9 elements per pass, barriers)
    static const std::string variant = [] {
      const char* e = std::getenv("FCG_H27_APPLY");
      return std::string(e ? e : "wave");
    }();
    const bool direct = variant == "direct", workgroup = variant == "sf";
    static const int64_t cap_w = [] {
      const char* e = std::getenv("FCG_H27_APPLY_GRID");
      return e ? std::max<int64_t>(8, std::atoll(e)) : int64_t(256 * 8);
    }();
    if (direct)
    {
      if (m.kinem == 0)
        hipLaunchKernelGGL((h27_apply_kernel<0>), grid, block, 0, stream, a);
      else
        hipLaunchKernelGGL((h27_apply_kernel<1>), grid, block, 0, stream, a);
    }
    else if (workgroup)
    {
      if (m.kinem == 0)
        hipLaunchKernelGGL((h27_apply_sf_kernel<0, 256, kApE>), grid, block, 0, stream, a);
      else
        hipLaunchKernelGGL((h27_apply_sf_kernel<1, 256, kApE>), grid, block, 0, stream, a);
    }
    else
    {
      // one wavefront per workgroup, 8 resident per CU (LDS 15.7 KB, <= 256 VGPRs)
      const dim3 gw(unsigned(std::min<int64_t>((m.n_ele + 1) / 2, cap_w))), bw(64);
      if (m.kinem == 0)
        hipLaunchKernelGGL((h27_apply_sf_kernel<0, 64, 2>), gw, bw, 0, stream, a);
      else
        hipLaunchKernelGGL((h27_apply_sf_kernel<1, 64, 2>), gw, bw, 0, stream, a);
    }
    const hipError_t he = hipGetLastError();
    if (he != hipSuccess) return he;
  }
  if (m.n_rownodes == 0) return hipSuccess;
  const dim3 grid(unsigned((m.n_rownodes + 255) / 256)), block(256);
  hipLaunchKernelGGL(h27_inc_sum_kernel, grid, block, 0, stream, m.n_rownodes, m.inc_ptr,
      m.rownode_row0, m.apply_ye, d_y_row);
  return hipGetLastError();
}

}  // namespace fcg
