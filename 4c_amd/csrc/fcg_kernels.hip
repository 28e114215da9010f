// fcg_kernels.hip -- CDNA4 (gfx950) kernels of the solid element evaluation + assembly path.
//
//  element_kernel   Discretization::evaluate's column-element loop + SolidEleCalc's Gauss-point
//                   loop (4C_fem_discretization_evaluate.cpp:83-102,
//                   4C_solid_3D_ele_calc.cpp:110-240): gathers X and u, checks the nodal Jacobian
//                   determinants, evaluates J^-1, N_XYZ, strains, StVK stresses, f_e and K_e, and
//                   writes every owned block-row of K_e plus f_a into an incidence-ordered scratch.
//  assemble_kernel  SparseMatrix::assemble + LinAlg::assemble(Vector) for owned rows
//                   (4C_linalg_sparsematrix.cpp:444-576, 4C_linalg_utils_sparse_algebra_assemble.cpp:72-92)
//                   as a deterministic gather: one wavefront per owned row node sums the block-rows
//                   of its incident elements in LDS (fixed element order -> bitwise reproducible, no
//                   atomics) and writes the node's 3 CSR rows once, coalesced.
//
// Isotropic StVK lets the element stiffness be written without the 6 x 3n B-matrix:
//   linear:  K_ab = sum_g fac [ lambda a b^T + mu b a^T + mu (a.b) I ]           a = N_XYZ of node a
//   TotLag:  K_ab = sum_g fac [ lambda (Fa)(Fb)^T + mu (Fb)(Fa)^T + mu (a.b) F F^T + (a.S.b) I ]
// which is B_a^T C B_b (+ K_geo, calc_lib.hpp:872-927) with C from fill_cmat
// (4C_mat_stvenantkirchhoff.cpp:115-145); see DESIGN.md for the derivation.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <cstdio>

#include "fcg_hex8_element.hpp"
#include "fcg_internal.hpp"
#include "fcg_shape.hpp"

namespace fcg {

// ---------------------------------------------------------------------------------- tables
__constant__ double c_dN8_gp[8 * 8 * 3];      // [g][node][d]
__constant__ double c_dN8_node[8 * 8 * 3];    // [at node][node][d]
__constant__ double c_w8[8];
__constant__ double c_dN27_gp[27 * 27 * 3];
__constant__ double c_dN27_node[27 * 27 * 3];
__constant__ double c_w27[27];
__constant__ uint16_t c_pairs27[378];          // symmetric pairs a <= b, packed a | b << 8
__constant__ uint8_t c_loc27[27];              // hex27 node lattice offsets, x | y << 2 | z << 4
__constant__ uint8_t c_latnode27[27];          // hex27 node at lattice offset x + 3 y + 9 z
__constant__ double c_L27gp[3][3];             // L_i(xi_p) of the 1D quadratic Lagrange factors
__constant__ double c_dL27gp[3][3];            // L_i'(xi_p), xi_p = -a, 0, a (hex_27point)
__constant__ double c_dL27nd[3][3];            // L_i'(x_p), x_p = -1, 0, 1 (the nodes)
// hex27 node lattice offsets (4C order, 4C_io_gridgenerator.cpp:348-369) for compile-time use
struct Hex27Pos {
  static constexpr int p[27][3] = {{0, 0, 0}, {2, 0, 0}, {2, 2, 0}, {0, 2, 0}, {0, 0, 2}, {2, 0, 2},
      {2, 2, 2}, {0, 2, 2}, {1, 0, 0}, {2, 1, 0}, {1, 2, 0}, {0, 1, 0}, {0, 0, 1}, {2, 0, 1},
      {2, 2, 1}, {0, 2, 1}, {1, 0, 2}, {2, 1, 2}, {1, 2, 2}, {0, 1, 2}, {1, 1, 0}, {1, 0, 1},
      {2, 1, 1}, {1, 2, 1}, {0, 1, 1}, {1, 1, 2}, {1, 1, 1}};
};
#define kPos27 Hex27Pos::p
__device__ inline int lat27(int a)
{
  const int l = c_loc27[a];
  return (l & 3) + 3 * ((l >> 2) & 3) + 9 * (l >> 4);
}

template <int NPE> struct Tables;
template <> struct Tables<8> {
  __device__ static const double* dNgp() { return c_dN8_gp; }
  __device__ static const double* dNnode() { return c_dN8_node; }
  __device__ static const double* w() { return c_w8; }
};
template <> struct Tables<27> {
  __device__ static const double* dNgp() { return c_dN27_gp; }
  __device__ static const double* dNnode() { return c_dN27_node; }
  __device__ static const double* w() { return c_w27; }
};

void upload_constant_tables(int /*celltype*/)
{
  static bool done = false;
  if (done) return;
  for (int ct = 0; ct < 2; ++ct)
  {
    const int n = num_nodes(ct);
    double xi[81], w[27], xn[81];
    gauss_rule(ct, xi, w);
    node_param_coords(ct, xn);
    double gp[27 * 27 * 3], nd[27 * 27 * 3];
    for (int g = 0; g < n; ++g) shape_deriv(ct, &xi[3 * g], &gp[3 * n * g]);
    for (int g = 0; g < n; ++g) shape_deriv(ct, &xn[3 * g], &nd[3 * n * g]);
    if (ct == kHex8)
    {
      (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dN8_gp), gp, sizeof(double) * 8 * 8 * 3);
      (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dN8_node), nd, sizeof(double) * 8 * 8 * 3);
      (void)hipMemcpyToSymbol(HIP_SYMBOL(c_w8), w, sizeof(double) * 8);
    }
    else
    {
      (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dN27_gp), gp, sizeof(gp));
      (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dN27_node), nd, sizeof(nd));
      (void)hipMemcpyToSymbol(HIP_SYMBOL(c_w27), w, sizeof(double) * 27);
    }
  }
  uint16_t pairs[378];
  int p = 0;
  for (int a = 0; a < 27; ++a)
    for (int b = a; b < 27; ++b) pairs[p++] = uint16_t(a | (b << 8));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_pairs27), pairs, sizeof(pairs));
  uint8_t loc[27];
  for (int a = 0; a < 27; ++a)
    loc[a] = uint8_t(kHex27NodePos[a][0] | (kHex27NodePos[a][1] << 2) | (kHex27NodePos[a][2] << 4));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_loc27), loc, sizeof(loc));
  uint8_t latnode[27];
  for (int a = 0; a < 27; ++a)
    latnode[kHex27NodePos[a][0] + 3 * kHex27NodePos[a][1] + 9 * kHex27NodePos[a][2]] = uint8_t(a);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_latnode27), latnode, sizeof(latnode));
  {
    // 1D factors, evaluated as in shape_deriv (fcg_shape.hpp)
    double xg[27 * 3], wg[27];
    gauss_rule(kHex27, xg, wg);
    const double xs[3] = {xg[3 * 0], xg[3 * 8], xg[3 * 1]};  // -a, 0, a (nodes 0, 8, 1 along xi)
    const double xn[3] = {-1.0, 0.0, 1.0};
    double L[3][3], dL[3][3], dLn[3][3];
    for (int p = 0; p < 3; ++p)
    {
      const double r = xs[p], t = xn[p];
      L[p][0] = 0.5 * r * (r - 1.0);
      L[p][1] = 1.0 - r * r;
      L[p][2] = 0.5 * r * (r + 1.0);
      dL[p][0] = r - 0.5;
      dL[p][1] = -2.0 * r;
      dL[p][2] = r + 0.5;
      dLn[p][0] = t - 0.5;
      dLn[p][1] = -2.0 * t;
      dLn[p][2] = t + 0.5;
    }
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_L27gp), L, sizeof(L));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dL27gp), dL, sizeof(dL));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dL27nd), dLn, sizeof(dLn));
  }
  done = true;
}

// ---------------------------------------------------------------------------------- helpers
// invert3x3 of the reference (4C_linalg_fixedsizematrix.hpp:1382-1409), column-major m[r + 3c].
__device__ inline double invert3x3(double* m)
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

// J(i,j) = sum_c dN(i,c) X(j,c)  (multiply_nt(deriv, xref), calc_lib.hpp:444)
template <int NPE>
__device__ inline void jacobian(const double* __restrict__ dN, const double* __restrict__ X, double* J)
{
#pragma unroll
  for (int k = 0; k < 9; ++k) J[k] = 0.0;
  for (int c = 0; c < NPE; ++c)
  {
    const double d0 = dN[3 * c + 0], d1 = dN[3 * c + 1], d2 = dN[3 * c + 2];
    const double x0 = X[3 * c + 0], x1 = X[3 * c + 1], x2 = X[3 * c + 2];
    J[0] += d0 * x0; J[1] += d1 * x0; J[2] += d2 * x0;
    J[3] += d0 * x1; J[4] += d1 * x1; J[5] += d2 * x1;
    J[6] += d0 * x2; J[7] += d1 * x2; J[8] += d2 * x2;
  }
}

template <int NPE, int KIN, int MAT = 0>
struct ElementShared {
  static constexpr int NGP = NPE;
  double X[3 * NPE];
  double U[3 * NPE];
  union {
    struct {
      double NX[NGP * NPE * 3];           // [g][c][d]
      double P[KIN ? NGP * NPE * 3 : 1];  // F * N_XYZ_c  (TotLag)
    };
    // TotLag hex27, colour-ordered path: the element's blocks a <= b (c_pairs27 order, 3 x 3
    // column-major), written once N_XYZ and P are no longer read
    double KSu[(NPE == 27 && KIN) ? 378 * 9 : 1];
  };
  // linear hex27: the same image in its own space (24 + 27 KB still allow 3 workgroups per CU),
  // written by the pair threads directly
  double KSs[(NPE == 27 && !KIN) ? 378 * 9 : 1];
  __device__ double* ks() { return KIN ? KSu : KSs; }
  double invJ[NGP * 9];
  double fac[NGP];
  double S[NGP * 6];                      // PK2 stress, Voigt xx yy zz xy yz zx
  double F[KIN ? NGP * 9 : 1];
  double M[KIN ? NGP * 6 : 1];            // F F^T (sym)
  double Cm[MAT ? NGP * 36 : 1];          // ElastHyper: cmat (column-major 6x6) per Gauss point
  int bad;
  // colour-ordered direct assembly: per local node its incidence (-1 = row not owned), the CSR
  // offset and length of its rows, and the column position of every element node in them
  int32_t inc[NPE];
  int32_t rlen[NPE];
  int64_t rbase[NPE];
  uint16_t ipos[NPE * NPE];
  uint8_t loc[NPE];      // hex27 lattice offsets of the nodes (c_loc27)
  uint8_t latnode[NPE];  // node at lattice offset (c_latnode27)
  // hex27 1D quadratic Lagrange factors: L_i and L_i' at the 3 Gauss abscissae, L_i' at -1, 0, 1
  double L1[3][3], dL1[3][3], dLn[3][3];
};

// Mat::ElastHyper with one ELAST_CoupNeoHooke summand: S and cmat from the principal invariants
// of C = 2E + I (4C_mat_elasthyper_service.cpp:19-215, 4C_mat_elast_coupneohooke.cpp,
// calculate_gamma_delta :413-432, add_holzapfel_product
// 4C_linalg_fixedsizematrix_tensor_products.cpp:264-312).  E in strain-like Voigt notation.
__device__ inline void neohooke_stress_cmat(double c, double beta, const double* E, double* S,
    double* cm)
{
  double C[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) C[i] = 2.0 * E[i];
  C[0] += 1.0;
  C[1] += 1.0;
  C[2] += 1.0;
  // determinant and inverse in strain-like Voigt notation (shear entries carry 2x)
  const double c3 = 0.5 * C[3], c4 = 0.5 * C[4], c5 = 0.5 * C[5];
  const double det = C[0] * C[1] * C[2] + 2 * c3 * c4 * c5 - C[1] * c5 * c5 - C[2] * c3 * c3 -
                     C[0] * c4 * c4;
  double iC[6];
  iC[0] = (C[1] * C[2] - c4 * c4) / det;
  iC[1] = (C[0] * C[2] - c5 * c5) / det;
  iC[2] = (C[0] * C[1] - c3 * c3) / det;
  iC[3] = (c5 * c4 - c3 * C[2]) / det;  // stress-like (tensor) components
  iC[4] = (c3 * c5 - C[0] * c4) / det;
  iC[5] = (c3 * c4 - c5 * C[1]) / det;
  const double I1 = C[0] + C[1] + C[2];
  const double I3 = det;
  // CoupNeoHooke::add_derivatives_principal: dPI = (c, 0, -c I3^(-beta-1)), ddPII(2)
  double dP2 = NAN, ddP2 = NAN;
  if (I3 > 0)
  {
    const double p = exp(log(I3) * (-beta - 1.));
    dP2 = -c * p;
    ddP2 = c * (beta + 1.) * p / I3;
  }
  const double g0 = 2. * c, g2 = 2. * I3 * dP2;
  const double d5 = 4. * (I3 * dP2 + I3 * I3 * ddP2), d6 = -4. * I3 * dP2;
  (void)I1;
  // S = g0 I + g2 C^-1 (stress-like)
  S[0] = g0 + g2 * iC[0];
  S[1] = g0 + g2 * iC[1];
  S[2] = g0 + g2 * iC[2];
  S[3] = g2 * iC[3];
  S[4] = g2 * iC[4];
  S[5] = g2 * iC[5];
  // cmat = d5 C^-1 (x) C^-1 + d6 (C^-1 odot C^-1)  (the other delta vanish for CoupNeoHooke)
  const double* v = iC;
#define CM(i, j) cm[(i) + 6 * (j)]
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int i = 0; i < 6; ++i) CM(i, j) = d5 * v[i] * v[j];
  CM(0, 0) += d6 * v[0] * v[0]; CM(0, 1) += d6 * v[3] * v[3]; CM(0, 2) += d6 * v[5] * v[5];
  CM(0, 3) += d6 * v[0] * v[3]; CM(0, 4) += d6 * v[3] * v[5]; CM(0, 5) += d6 * v[0] * v[5];
  CM(1, 0) += d6 * v[3] * v[3]; CM(1, 1) += d6 * v[1] * v[1]; CM(1, 2) += d6 * v[4] * v[4];
  CM(1, 3) += d6 * v[3] * v[1]; CM(1, 4) += d6 * v[1] * v[4]; CM(1, 5) += d6 * v[3] * v[4];
  CM(2, 0) += d6 * v[5] * v[5]; CM(2, 1) += d6 * v[4] * v[4]; CM(2, 2) += d6 * v[2] * v[2];
  CM(2, 3) += d6 * v[5] * v[4]; CM(2, 4) += d6 * v[4] * v[2]; CM(2, 5) += d6 * v[5] * v[2];
  CM(3, 0) += d6 * v[0] * v[3]; CM(3, 1) += d6 * v[3] * v[1]; CM(3, 2) += d6 * v[5] * v[4];
  CM(3, 3) += d6 * 0.5 * (v[0] * v[1] + v[3] * v[3]);
  CM(3, 4) += d6 * 0.5 * (v[3] * v[4] + v[5] * v[1]);
  CM(3, 5) += d6 * 0.5 * (v[0] * v[4] + v[5] * v[3]);
  CM(4, 0) += d6 * v[3] * v[5]; CM(4, 1) += d6 * v[1] * v[4]; CM(4, 2) += d6 * v[4] * v[2];
  CM(4, 3) += d6 * 0.5 * (v[3] * v[4] + v[5] * v[1]);
  CM(4, 4) += d6 * 0.5 * (v[1] * v[2] + v[4] * v[4]);
  CM(4, 5) += d6 * 0.5 * (v[3] * v[2] + v[4] * v[5]);
  CM(5, 0) += d6 * v[0] * v[5]; CM(5, 1) += d6 * v[3] * v[4]; CM(5, 2) += d6 * v[5] * v[2];
  CM(5, 3) += d6 * 0.5 * (v[0] * v[4] + v[5] * v[3]);
  CM(5, 4) += d6 * 0.5 * (v[3] * v[2] + v[4] * v[5]);
  CM(5, 5) += d6 * 0.5 * (v[0] * v[2] + v[5] * v[5]);
#undef CM
}

// B_NL of node n (evaluate_strain_gradient, calc_lib.hpp:708-760): B[r][e], F column-major
__device__ inline void strain_gradient(const double* F, const double* nx, double (*B)[3])
{
#pragma unroll
  for (int e = 0; e < 3; ++e)
  {
    B[0][e] = F[e] * nx[0];
    B[1][e] = F[e + 3] * nx[1];
    B[2][e] = F[e + 6] * nx[2];
    B[3][e] = F[e] * nx[1] + F[e + 3] * nx[0];
    B[4][e] = F[e + 3] * nx[2] + F[e + 6] * nx[1];
    B[5][e] = F[e + 6] * nx[0] + F[e] * nx[2];
  }
}

struct ElementArgs {
  int64_t n_ele;
  const int32_t* ele_nodes;
  const double* node_x;
  const int32_t* node_dof_col;
  const double* u_col;
  const int32_t* inc_of;
  double* scratch;
  int32_t* err;
  double lambda, mu, cdiag;
  double nh_c, nh_beta;  // ElastHyper/CoupNeoHooke: c = E / (4 (1 + nu)), beta = nu / (1 - 2 nu)
  int want_k;
  unsigned long long* stamps;  // diagnostic phase timers (NULL = off)
  // colour-ordered direct assembly (ASM != 0): elements col_ele[e_begin, e_end) of one colour
  const int32_t* col_ele;
  int64_t e_begin, e_end;
  const uint8_t* ele_ft;
  const int32_t* inc_row0;
  const uint16_t* inc_pos;
  const int64_t* rowptr;
  double* K;
  double* fint;
  int mfma;  // hex27 StVK: node-pair blocks on v_mfma_f64_16x16x4_f64 (else the VALU pair loop)
};

// Colour-ordered direct assembly: is element e (first-touch bits ft, see build_colored_plan in
// fcg_context.cpp) the first, in colour order, of the elements holding both hex27 nodes a and b?
// Along an axis where both nodes lie on e's lower (upper) face the lower (upper) neighbour holds
// them too; e comes first there iff bit 2d (2d+1) of ft is set.  Along every other axis e is alone.
__device__ inline bool first_touch27(const uint8_t* loc, uint32_t ft, int a, int b)
{
  const uint32_t la = loc[a], lb = loc[b];
  bool first = true;
#pragma unroll
  for (int d = 0; d < 3; ++d)
  {
    const uint32_t x = (la >> (2 * d)) & 3u, y = (lb >> (2 * d)) & 3u;
    if (x == y && x != 1u) first = first && ((ft >> (2 * d + (x == 2u ? 1 : 0))) & 1u);
  }
  return first;
}

// hex27 StVK node-pair blocks on the FP64 matrix cores (v_mfma_f64_16x16x4_f64).  With the rows
// (a, i) of the element's 81 DOFs ordered i-major and each node range padded to 32,
//   X_ij[a][b] = sum_g fac_g Q_g[a][i] Q_g[b][j]       (Q = N_XYZ linear, F N_XYZ TotLag)
// is 9 tiles of 16 x 16 per (a-range, b-range) pair over K = 27 Gauss points (7 steps of 4), and
// because the f64 MFMA's output layout depends only on the position in the tile, one lane holds
// X_ij and X_ji of the same (a, b) for all i, j: K_ab[i][j] = lambda X_ij + mu X_ji + ... is formed
// in registers.  TotLag adds mu H_ij + delta_ij geo = sum over (g, k) of N_a,k times
// fac (mu (F F^T)_ij N_b,k + delta_ij (S N_b)_k) -- 6 more tiles over K = 81 (21 steps).  Waves
// 0..2 take the (a, b) ranges (0,0), (0,1), (1,1) (a <= b is all the image needs); the blocks go to
// the LDS image KS (which TotLag aliases with N_XYZ / P: written after a barrier).
typedef double f64x4_t __attribute__((ext_vector_type(4)));
template <int KIN, typename SH>
__device__ inline void pair_phase_mfma27(SH& sh, double* KS, double lam, double mu, int tid)
{
  const int wave = tid >> 6, lane = tid & 63;
  const int at = wave == 2 ? 1 : 0, bt = wave == 0 ? 0 : 1;
  const int r16 = lane & 15, kq = lane >> 4;
  const int a_l = 16 * at + r16, b_l = 16 * bt + r16;
  const bool va = a_l < 27, vb = b_l < 27;
  const int a_c = va ? a_l : 0, b_c = vb ? b_l : 0;  // clamped: no read past the node range
  f64x4_t X[9], H[6];
#pragma unroll
  for (int q = 0; q < 9; ++q) X[q] = f64x4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < 6; ++q) H[q] = f64x4_t{0.0, 0.0, 0.0, 0.0};
  if (wave < 3)
  {
    const double* Q = KIN ? sh.P : sh.NX;  // [g][node][d]
#pragma unroll
    for (int st = 0; st < 7; ++st)
    {
      const int g = 4 * st + kq;
      const bool vg = g < 27;
      const int gc = vg ? g : 0;
      const double fg = vg ? sh.fac[gc] : 0.0;
      double av[3], bv[3];
#pragma unroll
      for (int i = 0; i < 3; ++i)
      {
        av[i] = va ? fg * Q[3 * (27 * gc + a_c) + i] : 0.0;
        bv[i] = (vg && vb) ? Q[3 * (27 * gc + b_c) + i] : 0.0;
      }
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          X[3 * i + j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], X[3 * i + j], 0, 0, 0);
    }
    if constexpr (KIN == 1)
    {
      for (int st = 0; st < 21; ++st)
      {
        const int kk = 4 * st + kq;
        const bool vk = kk < 81;
        const int g = vk ? kk / 3 : 0, k = vk ? kk - 3 * (kk / 3) : 0;
        const double fg = vk ? sh.fac[g] : 0.0;
        const double an = va ? sh.NX[3 * (27 * g + a_c) + k] : 0.0;
        const double* nb = sh.NX + 3 * (27 * g + b_c);
        const double n0 = vb ? nb[0] : 0.0, n1 = vb ? nb[1] : 0.0, n2 = vb ? nb[2] : 0.0;
        const double* S = sh.S + 6 * g;
        const double* M = sh.M + 6 * g;
        const double nk = k == 0 ? n0 : (k == 1 ? n1 : n2);
        const double snk = k == 0 ? S[0] * n0 + S[3] * n1 + S[5] * n2
                                  : (k == 1 ? S[3] * n0 + S[1] * n1 + S[4] * n2
                                            : S[5] * n0 + S[4] * n1 + S[2] * n2);
        const double fs = fg * snk, fm = fg * mu * nk;
        H[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(an, fs + fm * M[0], H[0], 0, 0, 0);
        H[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(an, fs + fm * M[1], H[1], 0, 0, 0);
        H[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(an, fs + fm * M[2], H[2], 0, 0, 0);
        H[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(an, fm * M[3], H[3], 0, 0, 0);
        H[4] = __builtin_amdgcn_mfma_f64_16x16x4f64(an, fm * M[4], H[4], 0, 0, 0);
        H[5] = __builtin_amdgcn_mfma_f64_16x16x4f64(an, fm * M[5], H[5], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // TotLag: KS aliases N_XYZ / P
  if (wave < 3)
  {
    const int b = 16 * bt + r16;
#pragma unroll
    for (int r = 0; r < 4; ++r)
    {
      const int a = 16 * at + kq + 4 * r;
      if (a < 27 && b < 27 && a <= b)
      {
        const int pidx = 27 * a - (a * (a - 1)) / 2 + b - a;
        double* K = KS + 9 * pidx;
        const double tr = mu * (X[0][r] + X[4][r] + X[8][r]);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
          {
            double v = lam * X[3 * i + j][r] + mu * X[3 * j + i][r];
            if constexpr (KIN == 0)
              v += i == j ? tr : 0.0;
            else
              v += i == j ? H[i][r] : H[(i + j == 1) ? 3 : ((i + j == 3) ? 4 : 5)][r];
            K[i + 3 * j] = v;
          }
      }
    }
  }
}

// ---------------------------------------------------------------------------------- element
// ASM: 0 = block rows into the incidence scratch (general path, assemble_kernel sums them);
// 1 / 2 = colour-ordered direct assembly, ACCUMULATE / OVERWRITE (hex27 lattice path).
template <int NPE, int KIN, int BLOCK, int MAT = 0, int ASM = 0>
__global__ __launch_bounds__(BLOCK, (NPE == 27 && MAT == 0) ? 3 : 1) void element_kernel(ElementArgs A)
{
  constexpr int NGP = NPE;
  constexpr bool SYM = (NPE == 27);             // hex27: compute a<=b and mirror
  constexpr int NPAIR = SYM ? NPE * (NPE + 1) / 2 : NPE * NPE;
  constexpr int REC = int(record_doubles(NPE));
  constexpr int ROWLEN = 3 * NPE;
  __shared__ ElementShared<NPE, KIN, MAT> sh;
  const int tid = threadIdx.x;
  const double* dNgp = Tables<NPE>::dNgp();
  const double* dNnode = Tables<NPE>::dNnode();
  const double* wgp = Tables<NPE>::w();

  // diagnostic phase timers (library built with -DFCG_ELEMENT_STAMPS, run with FCG_STAMPS=1):
  // wave-uniform s_memtime deltas, summed per workgroup; compiled out of the production library
  // (the counters would cost registers)
#ifdef FCG_ELEMENT_STAMPS
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long st_last = A.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
#define EL_STAMP(i)                                                                                \
  if (A.stamps)                                                                                    \
  {                                                                                                \
    const unsigned long long now = __builtin_amdgcn_s_memtime();                                  \
    st_acc[i] += now - st_last;                                                                    \
    st_last = now;                                                                                 \
  }
#else
#define EL_STAMP(i)
#endif
  const int64_t n_it = ASM ? A.e_end - A.e_begin : A.n_ele;
  for (int64_t it = blockIdx.x; it < n_it; it += gridDim.x)
  {
    const int64_t e = ASM ? int64_t(A.col_ele[A.e_begin + it]) : it;
    const uint32_t ft = ASM ? uint32_t(A.ele_ft[e]) : 0u;
    const int32_t* en = A.ele_nodes + e * NPE;
    // 1. gather reference coordinates and displacements (evaluate_element_nodes, calc_lib.hpp:180-203)
    for (int v = tid; v < 3 * NPE; v += BLOCK)
    {
      const int a = v / 3, d = v - 3 * (v / 3);
      const int node = en[a];
      sh.X[v] = A.node_x[3 * int64_t(node) + d];
      sh.U[v] = A.u_col[A.node_dof_col[node] + d];
    }
    if (NPE == 27 && !ASM && tid < NPE)
    {
      sh.inc[tid] = A.inc_of[e * NPE + tid];
      sh.loc[tid] = c_loc27[tid];
      sh.latnode[tid] = c_latnode27[tid];
    }
    if (NPE == 27 && tid < 9)
    {
      (&sh.L1[0][0])[tid] = (&c_L27gp[0][0])[tid];
      (&sh.dL1[0][0])[tid] = (&c_dL27gp[0][0])[tid];
      (&sh.dLn[0][0])[tid] = (&c_dL27nd[0][0])[tid];
    }
    if (ASM)
    {
      for (int v = tid; v < NPE * NPE; v += BLOCK)
      {
        const int a = v / NPE;
        const int32_t ia = A.inc_of[e * NPE + a];
        sh.ipos[v] = ia >= 0 ? A.inc_pos[int64_t(ia) * NPE + (v - NPE * a)] : uint16_t(0);
        if (v - NPE * a == 0)
        {
          sh.loc[a] = c_loc27[a];
          sh.latnode[a] = c_latnode27[a];
          sh.inc[a] = ia;
          if (ia >= 0)
          {
            const int32_t r0 = A.inc_row0[ia];
            sh.rbase[a] = A.rowptr[r0];
            sh.rlen[a] = int32_t(A.rowptr[r0 + 1] - A.rowptr[r0]);
          }
        }
      }
    }
    if (tid == 0) sh.bad = 0;
    __syncthreads();
    EL_STAMP(0);

    // 2. nodal det J > 0 check (calc_lib.hpp:475-496) and GP Jacobian inverses (calc_lib.hpp:435-448)
    if (NPE == 27 && tid < NPE + NGP)
    {
      // hex27 shape functions are products of 1D quadratic Lagrange factors (the tables of
      // upload_constant_tables are built the same way), so dN comes from 9 + 9 factors instead of
      // 81 table loads; at a node the factors are Kronecker deltas and J reduces to the 3 nodes on
      // each parametric line through it
      const bool at_node = tid < NPE;
      const int g = at_node ? tid : tid - NPE;
      const uint32_t l = sh.loc[g];
      const int p = l & 3, q = (l >> 2) & 3, r = l >> 4;
      double J[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) J[k] = 0.0;
      if (at_node)
      {
#pragma unroll
        for (int m = 0; m < 3; ++m)
        {
          const double* x0 = sh.X + 3 * sh.latnode[m + 3 * q + 9 * r];
          const double* x1 = sh.X + 3 * sh.latnode[p + 3 * m + 9 * r];
          const double* x2 = sh.X + 3 * sh.latnode[p + 3 * q + 9 * m];
          const double d0 = sh.dLn[p][m], d1 = sh.dLn[q][m], d2 = sh.dLn[r][m];
#pragma unroll
          for (int c = 0; c < 3; ++c)
          {
            J[3 * c + 0] += d0 * x0[c];
            J[3 * c + 1] += d1 * x1[c];
            J[3 * c + 2] += d2 * x2[c];
          }
        }
        const double det = invert3x3(J);
        if (det == 0.0) atomicMax(&sh.bad, 2);
        else if (!(det > 0)) atomicMax(&sh.bad, 1);
      }
      else
      {
        double Lx[3], Ly[3], Lz[3], dx[3], dy[3], dz[3];
#pragma unroll
        for (int m = 0; m < 3; ++m)
        {
          Lx[m] = sh.L1[p][m]; dx[m] = sh.dL1[p][m];
          Ly[m] = sh.L1[q][m]; dy[m] = sh.dL1[q][m];
          Lz[m] = sh.L1[r][m]; dz[m] = sh.dL1[r][m];
        }
#pragma unroll
        for (int c = 0; c < 27; ++c)
        {
          const int i = kPos27[c][0], j = kPos27[c][1], k = kPos27[c][2];
          const double d0 = Ly[j] * Lz[k] * dx[i];
          const double d1 = Lx[i] * Lz[k] * dy[j];
          const double d2 = Lx[i] * Ly[j] * dz[k];
          const double x0 = sh.X[3 * c + 0], x1 = sh.X[3 * c + 1], x2 = sh.X[3 * c + 2];
          J[0] += d0 * x0; J[1] += d1 * x0; J[2] += d2 * x0;
          J[3] += d0 * x1; J[4] += d1 * x1; J[5] += d2 * x1;
          J[6] += d0 * x2; J[7] += d1 * x2; J[8] += d2 * x2;
        }
        const double det = invert3x3(J);
        if (det == 0.0) atomicMax(&sh.bad, 2);
#pragma unroll
        for (int k = 0; k < 9; ++k) sh.invJ[9 * g + k] = J[k];
        sh.fac[g] = det * wgp[g];
      }
    }
    else if (NPE == 27)
    {
    }
    else if (tid < NPE)
    {
      double J[9];
      jacobian<NPE>(dNnode + 3 * NPE * tid, sh.X, J);
      const double det = invert3x3(J);
      if (det == 0.0) atomicMax(&sh.bad, 2);
      else if (!(det > 0)) atomicMax(&sh.bad, 1);
    }
    else if (tid < NPE + NGP)
    {
      const int g = tid - NPE;
      double J[9];
      jacobian<NPE>(dNgp + 3 * NPE * g, sh.X, J);
      const double det = invert3x3(J);
      if (det == 0.0) atomicMax(&sh.bad, 2);
#pragma unroll
      for (int k = 0; k < 9; ++k) sh.invJ[9 * g + k] = J[k];
      sh.fac[g] = det * wgp[g];
    }
    __syncthreads();
    EL_STAMP(1);
    if (sh.bad)
    {
      if (tid == 0)
      {
        atomicMax(&A.err[0], sh.bad);
        atomicMin(&A.err[1], int32_t(e));
      }
      __syncthreads();
      continue;
    }

    // 3. N_XYZ = J^-1 dN (multiply(inverse_jacobian, derivatives))
    for (int v = tid; v < NGP * NPE; v += BLOCK)
    {
      const int g = v / NPE, c = v - NPE * (v / NPE);
      const double* iJ = sh.invJ + 9 * g;
      const double* d = dNgp + 3 * (NPE * g + c);
      const double d0 = d[0], d1 = d[1], d2 = d[2];
#pragma unroll
      for (int i = 0; i < 3; ++i) sh.NX[3 * v + i] = iJ[i] * d0 + iJ[i + 3] * d1 + iJ[i + 6] * d2;
    }
    __syncthreads();
    EL_STAMP(2);

    // 4. strains and StVK stress per Gauss point
    if (tid < NGP)
    {
      const int g = tid;
      const double* NX = sh.NX + 3 * NPE * g;
      double E[6];
      if (KIN == 0)
      {
        // evaluate_linear_strain_gradient + evaluate_linear_gl_strain (calc_lib.hpp:682-799)
        for (int k = 0; k < 6; ++k) E[k] = 0.0;
        for (int c = 0; c < NPE; ++c)
        {
          const double n0 = NX[3 * c], n1 = NX[3 * c + 1], n2 = NX[3 * c + 2];
          const double u0 = sh.U[3 * c], u1 = sh.U[3 * c + 1], u2 = sh.U[3 * c + 2];
          E[0] += n0 * u0;
          E[1] += n1 * u1;
          E[2] += n2 * u2;
          E[3] += n1 * u0 + n0 * u1;
          E[4] += n2 * u1 + n1 * u2;
          E[5] += n2 * u0 + n0 * u2;
        }
      }
      else
      {
        // evaluate_deformation_gradient (calc_lib.hpp:579-605): hex8 from current coordinates,
        // hex27 as I + u N_XYZ^T.  F(i,j) column-major.
        double F[9];
        for (int k = 0; k < 9; ++k) F[k] = 0.0;
        for (int c = 0; c < NPE; ++c)
        {
          const double n0 = NX[3 * c], n1 = NX[3 * c + 1], n2 = NX[3 * c + 2];
          double q[3];
#pragma unroll
          for (int i = 0; i < 3; ++i) q[i] = (NPE == 8) ? sh.X[3 * c + i] + sh.U[3 * c + i] : sh.U[3 * c + i];
#pragma unroll
          for (int i = 0; i < 3; ++i)
          {
            F[i + 0] += q[i] * n0;
            F[i + 3] += q[i] * n1;
            F[i + 6] += q[i] * n2;
          }
        }
        if (NPE != 8)
        {
          F[0] += 1.0;
          F[4] += 1.0;
          F[8] += 1.0;
        }
        // inverse of F must exist (evaluate_spatial_material_mapping, calc_lib.hpp:562)
        {
          double Fi[9];
#pragma unroll
          for (int k = 0; k < 9; ++k) Fi[k] = F[k];
          if (invert3x3(Fi) == 0.0) atomicMax(&sh.bad, 2);
        }
        // C = F^T F, E = (C - I)/2 with engineering shear (calc_lib.hpp:639-676)
        double C[9];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            C[i + 3 * j] = F[3 * i] * F[3 * j] + F[3 * i + 1] * F[3 * j + 1] + F[3 * i + 2] * F[3 * j + 2];
        E[0] = 0.5 * (C[0] - 1.0);
        E[1] = 0.5 * (C[4] - 1.0);
        E[2] = 0.5 * (C[8] - 1.0);
        E[3] = C[3];
        E[4] = C[7];
        E[5] = C[2];
        double* Fs = sh.F + 9 * g;
#pragma unroll
        for (int k = 0; k < 9; ++k) Fs[k] = F[k];
        double* Ms = sh.M + 6 * g;  // F F^T: xx yy zz xy yz zx
        Ms[0] = F[0] * F[0] + F[3] * F[3] + F[6] * F[6];
        Ms[1] = F[1] * F[1] + F[4] * F[4] + F[7] * F[7];
        Ms[2] = F[2] * F[2] + F[5] * F[5] + F[8] * F[8];
        Ms[3] = F[0] * F[1] + F[3] * F[4] + F[6] * F[7];
        Ms[4] = F[1] * F[2] + F[4] * F[5] + F[7] * F[8];
        Ms[5] = F[2] * F[0] + F[5] * F[3] + F[8] * F[6];
      }
      // So3Material::evaluate -> S = C E (4C_mat_stvenantkirchhoff.cpp:169-177), or ElastHyper
      double* S = sh.S + 6 * g;
      if (MAT == 1)
        neohooke_stress_cmat(A.nh_c, A.nh_beta, E, S, sh.Cm + 36 * (MAT ? g : 0));
      else
      {
        S[0] = A.cdiag * E[0] + A.lambda * E[1] + A.lambda * E[2];
        S[1] = A.lambda * E[0] + A.cdiag * E[1] + A.lambda * E[2];
        S[2] = A.lambda * E[0] + A.lambda * E[1] + A.cdiag * E[2];
        S[3] = A.mu * E[3];
        S[4] = A.mu * E[4];
        S[5] = A.mu * E[5];
      }
    }
    __syncthreads();
    EL_STAMP(3);
    if (KIN == 1)
    {
      if (sh.bad)
      {
        if (tid == 0)
        {
          atomicMax(&A.err[0], sh.bad);
          atomicMin(&A.err[1], int32_t(e));
        }
        __syncthreads();
        continue;
      }
      // P_c = F N_XYZ_c
      for (int v = tid; v < NGP * NPE; v += BLOCK)
      {
        const int g = v / NPE;
        const double* F = sh.F + 9 * g;
        const double n0 = sh.NX[3 * v], n1 = sh.NX[3 * v + 1], n2 = sh.NX[3 * v + 2];
#pragma unroll
        for (int i = 0; i < 3; ++i) sh.P[3 * v + i] = F[i] * n0 + F[i + 3] * n1 + F[i + 6] * n2;
      }
      __syncthreads();
      EL_STAMP(4);
    }

    const int32_t* inc = A.inc_of + e * NPE;

    // 5. internal force f_a = sum_g fac F S N_XYZ_a  (add_internal_force_vector, calc_lib.hpp:851-860)
    if (tid < NPE)
    {
      const int a = tid;
      const int32_t ia = inc[a];
      if (ia >= 0)
      {
        double f[3] = {0.0, 0.0, 0.0};
        for (int g = 0; g < NGP; ++g)
        {
          const double* S = sh.S + 6 * g;
          const double* n = sh.NX + 3 * (NPE * g + a);
          const double fc = sh.fac[g];
          double t[3];
          t[0] = S[0] * n[0] + S[3] * n[1] + S[5] * n[2];
          t[1] = S[3] * n[0] + S[1] * n[1] + S[4] * n[2];
          t[2] = S[5] * n[0] + S[4] * n[1] + S[2] * n[2];
          if (KIN == 1)
          {
            const double* F = sh.F + 9 * g;
            const double s0 = F[0] * t[0] + F[3] * t[1] + F[6] * t[2];
            const double s1 = F[1] * t[0] + F[4] * t[1] + F[7] * t[2];
            const double s2 = F[2] * t[0] + F[5] * t[1] + F[8] * t[2];
            t[0] = s0;
            t[1] = s1;
            t[2] = s2;
          }
          f[0] += fc * t[0];
          f[1] += fc * t[1];
          f[2] += fc * t[2];
        }
        if (ASM)
        {
          double* dst = A.fint + A.inc_row0[ia];
          if (ASM == 2 && first_touch27(sh.loc, ft, a, a))
          {
            dst[0] = f[0];
            dst[1] = f[1];
            dst[2] = f[2];
          }
          else
          {
            dst[0] += f[0];
            dst[1] += f[1];
            dst[2] += f[2];
          }
        }
        else
        {
          double* rec = A.scratch + int64_t(ia) * REC + 9 * NPE;
          rec[0] = f[0];
          rec[1] = f[1];
          rec[2] = f[2];
        }
      }
    }

    // 6. element stiffness blocks K_ab (add_elastic/geometric_stiffness_matrix, calc_lib.hpp:872-927)
    auto pair_block = [&](int a, int b, double* K) {
      double G[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) G[k] = 0.0;
      double H[6] = {0, 0, 0, 0, 0, 0};
      double geo = 0.0;
      for (int g = 0; g < NGP; ++g)
      {
        const double fc = sh.fac[g];
        const double* na = sh.NX + 3 * (NPE * g + a);
        const double* nb = sh.NX + 3 * (NPE * g + b);
        if (MAT == 1)
        {
          // general material: K_ab += fac (B_a^T cmat B_b + (a.S.b) I)  (calc_lib.hpp:872-927);
          // G holds B_a^T cmat B_b (row-major i, j), geo the geometric part
          const double* F = sh.F + 9 * g;
          const double* cm = sh.Cm + 36 * (MAT ? g : 0);
          double Ba[6][3], Bb[6][3];
          strain_gradient(F, na, Ba);
          strain_gradient(F, nb, Bb);
#pragma unroll
          for (int j = 0; j < 3; ++j)
          {
            double cb[6];
#pragma unroll
            for (int r = 0; r < 6; ++r)
            {
              double t = 0.0;
#pragma unroll
              for (int q = 0; q < 6; ++q) t += cm[r + 6 * q] * Bb[q][j];
              cb[r] = fc * t;
            }
#pragma unroll
            for (int i = 0; i < 3; ++i)
            {
              double t = 0.0;
#pragma unroll
              for (int r = 0; r < 6; ++r) t += Ba[r][i] * cb[r];
              G[i + 3 * j] += t;
            }
          }
          const double* S = sh.S + 6 * g;
          const double c0 = nb[0], c1 = nb[1], c2 = nb[2];
          const double sb0 = S[0] * c0 + S[3] * c1 + S[5] * c2;
          const double sb1 = S[3] * c0 + S[1] * c1 + S[4] * c2;
          const double sb2 = S[5] * c0 + S[4] * c1 + S[2] * c2;
          geo += fc * (na[0] * sb0 + na[1] * sb1 + na[2] * sb2);
        }
        else if (KIN == 0)
        {
          const double fa0 = fc * na[0], fa1 = fc * na[1], fa2 = fc * na[2];
          const double b0 = nb[0], b1 = nb[1], b2 = nb[2];
          G[0] += fa0 * b0; G[3] += fa0 * b1; G[6] += fa0 * b2;
          G[1] += fa1 * b0; G[4] += fa1 * b1; G[7] += fa1 * b2;
          G[2] += fa2 * b0; G[5] += fa2 * b1; G[8] += fa2 * b2;
        }
        else
        {
          const double* pa = sh.P + 3 * (NPE * g + a);
          const double* pb = sh.P + 3 * (NPE * g + b);
          const double fa0 = fc * pa[0], fa1 = fc * pa[1], fa2 = fc * pa[2];
          const double b0 = pb[0], b1 = pb[1], b2 = pb[2];
          G[0] += fa0 * b0; G[3] += fa0 * b1; G[6] += fa0 * b2;
          G[1] += fa1 * b0; G[4] += fa1 * b1; G[7] += fa1 * b2;
          G[2] += fa2 * b0; G[5] += fa2 * b1; G[8] += fa2 * b2;
          const double a0 = na[0], a1 = na[1], a2 = na[2];
          const double c0 = nb[0], c1 = nb[1], c2 = nb[2];
          const double t = fc * (a0 * c0 + a1 * c1 + a2 * c2);
          const double* M = sh.M + 6 * g;
#pragma unroll
          for (int k = 0; k < 6; ++k) H[k] += t * M[k];
          const double* S = sh.S + 6 * g;
          const double sb0 = S[0] * c0 + S[3] * c1 + S[5] * c2;
          const double sb1 = S[3] * c0 + S[1] * c1 + S[4] * c2;
          const double sb2 = S[5] * c0 + S[4] * c1 + S[2] * c2;
          geo += fc * (a0 * sb0 + a1 * sb1 + a2 * sb2);
        }
      }
      // K_ij = lambda G_ij + mu G_ji + mu tr(G) delta_ij      (linear)
      // K_ij = lambda G_ij + mu G_ji + mu H_ij + geo delta_ij (TotLag)
      const double lam = A.lambda, mu = A.mu;
      if (MAT == 1)
      {
#pragma unroll
        for (int i = 0; i < 9; ++i) K[i] = G[i];
        K[0] += geo;
        K[4] += geo;
        K[8] += geo;
      }
      else
      {
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) K[i + 3 * j] = lam * G[i + 3 * j] + mu * G[j + 3 * i];
      }
      if (MAT == 1)
      {
      }
      else if (KIN == 0)
      {
        const double tr = mu * (G[0] + G[4] + G[8]);
        K[0] += tr;
        K[4] += tr;
        K[8] += tr;
      }
      else
      {
        K[0] += mu * H[0] + geo;
        K[4] += mu * H[1] + geo;
        K[8] += mu * H[2] + geo;
        K[1] += mu * H[3]; K[3] += mu * H[3];
        K[5] += mu * H[4]; K[7] += mu * H[4];
        K[2] += mu * H[5]; K[6] += mu * H[5];
      }
    };
    auto pair_of = [&](int p, int& a, int& b) {
      if (SYM)
      {
        const uint16_t pr = c_pairs27[p];
        a = pr & 0xff;
        b = pr >> 8;
      }
      else
      {
        a = p / NPE;
        b = p - NPE * (p / NPE);
      }
    };
    if constexpr (NPE == 27 && (KIN == 0 || ASM != 0 || MAT == 0))
    {
      if (A.want_k)
      {
      // blocks a <= b into registers, then (after every thread's last N_XYZ / P read) into the
      // LDS image KS; then the element's owned block rows leave coalesced: general path (ASM 0)
      // as contiguous incidence records [3][27 nodes][3] of the scratch; colour-ordered path as
      // runs of contiguous CSR columns (element nodes in lattice order) -- written by the first
      // element of the colour order that holds both nodes, added to by the others
      double* KS = sh.ks();
      // matrix cores for the linear blocks and the colour-ordered TotLag path; the TotLag
      // scratch path keeps the VALU loop (its 15 accumulator tiles would spill at three
      // workgroups per CU, and at two the MFMA phase measured slower: DESIGN §7e)
      constexpr bool kMfma = MAT == 0 && !(KIN == 1 && ASM == 0);
      if (kMfma && A.mfma)
        pair_phase_mfma27<KIN>(sh, KS, A.lambda, A.mu, tid);
      else if constexpr (KIN == 0)
      {
        for (int p = tid; p < NPAIR; p += BLOCK)
        {
          int a, b;
          pair_of(p, a, b);
          if (sh.inc[a] >= 0 || sh.inc[b] >= 0) pair_block(a, b, KS + 9 * p);
        }
      }
      else if constexpr (ASM != 0)
      {
        double Kq[2][9];
#pragma unroll
        for (int q = 0; q < 2; ++q)
        {
          const int p = tid + BLOCK * q;
          if (p < NPAIR)
          {
            int a, b;
            pair_of(p, a, b);
            if (sh.inc[a] >= 0 || sh.inc[b] >= 0) pair_block(a, b, Kq[q]);
          }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 2; ++q)
        {
          const int p = tid + BLOCK * q;
          if (p < NPAIR)
#pragma unroll
            for (int k = 0; k < 9; ++k) KS[9 * p + k] = Kq[q][k];
        }
      }
      else
      {
        // TotLag general path without MFMA: each pair thread writes its block rows straight into
        // the scratch records
        for (int p = tid; p < NPAIR; p += BLOCK)
        {
          int a, b;
          pair_of(p, a, b);
          const int32_t ia = inc[a];
          const int32_t ib = inc[b];
          if (ia < 0 && ib < 0) continue;
          double K[9];
          pair_block(a, b, K);
          if (ia >= 0)
          {
            double* rec = A.scratch + int64_t(ia) * REC + 3 * b;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int j = 0; j < 3; ++j) rec[i * ROWLEN + j] = K[i + 3 * j];
          }
          if (a != b && ib >= 0)
          {
            double* rec = A.scratch + int64_t(ib) * REC + 3 * a;
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int j = 0; j < 3; ++j) rec[i * ROWLEN + j] = K[j + 3 * i];
          }
        }
      }
      const bool image = !(KIN == 1 && ASM == 0);
      __syncthreads();
      if (!image)
      {
      }
      else if constexpr (ASM == 0)
      {
        for (int v = tid; v < NPE * 243; v += BLOCK)
        {
          const int a = v / 243;
          if (sh.inc[a] < 0) continue;
          const int r = v - 243 * a;
          const int i = r / 81, c = r - 81 * (r / 81);
          const int b = c / 3, j = c - 3 * (c / 3);
          const int lo = a < b ? a : b, hi = a < b ? b : a;
          const int pidx = 27 * lo - (lo * (lo - 1)) / 2 + hi - lo;
          A.scratch[int64_t(sh.inc[a]) * REC + r] = KS[9 * pidx + (a <= b ? i + 3 * j : j + 3 * i)];
        }
      }
      else
      {
      constexpr int NV = 9;  // entries in flight per thread: all loads before the stores
      for (int v0 = 0; v0 < NPE * 243; v0 += NV * BLOCK)
      {
        uint32_t slot[NV];  // local row node | offset inside its rows << 5; 0xFFFFFFFF = none
        double val[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k)
        {
          const int v = v0 + tid + BLOCK * k;
          slot[k] = 0xFFFFFFFFu;
          val[k] = 0.0;
          if (v >= NPE * 243) continue;
          const int a = v / 243;
          if (sh.inc[a] < 0) continue;
          const int r = v - 243 * a;
          const int i = r / 81, c = r - 81 * (r / 81);
          const int b = sh.latnode[c / 3], j = c - 3 * (c / 3);
          const uint32_t o = uint32_t(i * sh.rlen[a] + sh.ipos[NPE * a + b] + j);
          slot[k] = uint32_t(a) | (o << 5);
          const int lo = a < b ? a : b, hi = a < b ? b : a;
          const int pidx = 27 * lo - (lo * (lo - 1)) / 2 + hi - lo;
          val[k] = KS[9 * pidx + (a <= b ? i + 3 * j : j + 3 * i)];
          if (!(ASM == 2 && first_touch27(sh.loc, ft, a, b))) val[k] += A.K[sh.rbase[a] + o];
        }
#pragma unroll
        for (int k = 0; k < NV; ++k)
          if (slot[k] != 0xFFFFFFFFu)
            __builtin_nontemporal_store(val[k], A.K + sh.rbase[slot[k] & 31u] + (slot[k] >> 5));
      }
      }
      }
    }
    else if (A.want_k)
    {
      for (int p = tid; p < NPAIR; p += BLOCK)
      {
        int a, b;
        pair_of(p, a, b);
        const int32_t ia = inc[a];
        const int32_t ib = inc[b];
        if (ia < 0 && (!SYM || ib < 0)) continue;
        double K[9];
        pair_block(a, b, K);
        if (ia >= 0)
        {
          double* rec = A.scratch + int64_t(ia) * REC + 3 * b;
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) rec[i * ROWLEN + j] = K[i + 3 * j];
        }
        if (SYM && a != b && ib >= 0)
        {
          double* rec = A.scratch + int64_t(ib) * REC + 3 * a;
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) rec[i * ROWLEN + j] = K[j + 3 * i];
        }
      }
    }
    __syncthreads();
    EL_STAMP(5);
  }
#ifdef FCG_ELEMENT_STAMPS
  if (A.stamps && tid == 0)
  {
    for (int i = 0; i < 6; ++i) atomicAdd(&A.stamps[i], st_acc[i]);
    atomicAdd(&A.stamps[6], (unsigned long long)((n_it - blockIdx.x + gridDim.x - 1) / gridDim.x));
    atomicAdd(&A.stamps[7], 1ull);
  }
#endif
#undef EL_STAMP
}

// ---------------------------------------------------------------------------------- hex8, 8 lanes/element
// General (unstructured) hex8 path: 32 elements per 256-thread workgroup, 8 lanes per element
// (fcg_hex8_element.hpp); K_ab goes to the record of incidence (e,a), K_ab^T to (e,b).
constexpr int H8_EPB = 32;  // elements per block

template <int KIN>
__global__ __launch_bounds__(256) void element_kernel_h8(ElementArgs A)
{
  constexpr int REC = 9 * 8 + 3;
  constexpr int ROWLEN = 24;
  __shared__ H8Slot<KIN> slot[H8_EPB];
  __shared__ double dN[8][8][3], dNn[8][8][3];
  __shared__ int bad[H8_EPB];
  const int tid = threadIdx.x;
  const int le = tid >> 3;  // element slot in block
  const int j = tid & 7;    // lane within the element group
  for (int v = tid; v < 192; v += 256)
  {
    (&dN[0][0][0])[v] = c_dN8_gp[v];
    (&dNn[0][0][0])[v] = c_dN8_node[v];
  }
  const StVK mat{A.lambda, A.mu, A.cdiag};
  H8Slot<KIN>& s = slot[le];
  for (int64_t e0 = int64_t(blockIdx.x) * H8_EPB; e0 < A.n_ele; e0 += int64_t(gridDim.x) * H8_EPB)
  {
    const int64_t e = e0 + le;
    const bool active = e < A.n_ele;
    if (active)
    {
      const int node = A.ele_nodes[e * 8 + j];
      const int dof = A.node_dof_col[node];
#pragma unroll
      for (int d = 0; d < 3; ++d)
      {
        s.X[j][d] = A.node_x[3 * int64_t(node) + d];
        s.U[j][d] = A.u_col[dof + d];
      }
    }
    if (j == 0) bad[le] = 0;
    __syncthreads();
    if (active)
    {
      const int b = h8_stage_a<KIN>(j, s, dN, dNn, c_w8[j], mat);
      if (b) atomicMax(&bad[le], b);
    }
    __syncthreads();
    if (active && bad[le] == 0)
    {
      const int a = j;
      double K[5][9], f[3];
      h8_stage_b<KIN>(a, s, mat, A.want_k != 0, K, f);
      const int32_t* inc = A.inc_of + e * 8;
      const int32_t ia = inc[a];
      if (ia >= 0)
      {
        double* rec = A.scratch + int64_t(ia) * REC + 72;
        rec[0] = f[0];
        rec[1] = f[1];
        rec[2] = f[2];
      }
      if (A.want_k)
      {
        const int npair = h8_npair(a);
#pragma unroll
        for (int p = 0; p < 5; ++p)
        {
          if (p >= npair) break;
          const int bb = (a + p) & 7;
          if (ia >= 0)
          {
            double* rec = A.scratch + int64_t(ia) * REC + 3 * bb;
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
              for (int q = 0; q < 3; ++q) rec[r * ROWLEN + q] = K[p][r + 3 * q];
          }
          const int32_t ib = inc[bb];
          if (p > 0 && ib >= 0)
          {
            double* rec = A.scratch + int64_t(ib) * REC + 3 * a;
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
              for (int q = 0; q < 3; ++q) rec[r * ROWLEN + q] = K[p][q + 3 * r];
          }
        }
      }
    }
    if (active && j == 0 && bad[le])
    {
      atomicMax(&A.err[0], bad[le]);
      atomicMin(&A.err[1], int32_t(e));
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------- assembly
struct AssembleArgs {
  int64_t n_rownodes;
  const int64_t* inc_ptr;
  const int32_t* rownode_row0;
  const uint16_t* inc_pos;
  const double* scratch;
  const int64_t* rowptr;
  double* K;
  double* fint;
  // hex27 slab schedule (assemble27_kernel): rows[j_begin, j_end) (NULL: row nodes j directly),
  // the records of row node r at slots rslot0[r] + i (mod ring); ring 0: at the incidence index
  const int32_t* rows;
  int64_t j_begin, j_end;
  const int32_t* rslot0;
  int64_t ring;
};

// hex27 rows: one wavefront per owned row node as assemble_kernel, the incidence records read as
// 16-byte pieces, two records in flight before their sums enter the LDS row image (each
// record adds to distinct columns and a wavefront's LDS operations execute in order: no barrier
// between records).  Summation order per entry = incidence order, as in assemble_kernel.
template <bool WANT_K, bool OVERWRITE>
__global__ __launch_bounds__(64) void assemble27_kernel(AssembleArgs A)
{
#ifndef FCG_A27_NB
#define FCG_A27_NB 2
#endif
  constexpr int NPE = 27, REC = int(record_doubles(NPE)), NB = FCG_A27_NB;
  constexpr int NV2 = 2;  // double2 pieces per lane and record: 122 pieces of the 243 entries
  __shared__ double acc[WANT_K ? 3 * 375 : 1];
  const int lane = threadIdx.x;
  for (int64_t jj = A.j_begin + blockIdx.x; jj < A.j_end; jj += gridDim.x)
  {
    const int64_t r = A.rows ? int64_t(A.rows[jj]) : jj;
    const int32_t row0 = A.rownode_row0[r];
    const int64_t base = A.rowptr[row0];
    const int rowlen = int(A.rowptr[row0 + 1] - base);
    if (WANT_K)
      for (int v = lane; v < 3 * rowlen; v += 64) acc[v] = 0.0;
    double f = 0.0;
    const int64_t k0 = A.inc_ptr[r], k1 = A.inc_ptr[r + 1];
    const int64_t s0 = A.ring ? int64_t(A.rslot0[r]) : k0;  // record slot of incidence k0
    for (int64_t kb = k0; kb < k1; kb += NB)
    {
      double2 val[NB][NV2];
      int dst[NB][NV2][2];
      double fv[NB];
#pragma unroll
      for (int q = 0; q < NB; ++q)
      {
        const int64_t k = kb + q;
        fv[q] = 0.0;
#pragma unroll
        for (int s = 0; s < NV2; ++s)
        {
          val[q][s] = make_double2(0.0, 0.0);
          dst[q][s][0] = dst[q][s][1] = -1;
        }
        if (k >= k1) continue;
        int64_t slot = s0 + (k - k0);
        if (A.ring && slot >= A.ring) slot -= A.ring;
        const double* src = A.scratch + slot * REC;
        if (lane < 3) fv[q] = src[243 + lane];
        if (!WANT_K) continue;
        const uint16_t* pos = A.inc_pos + k * NPE;
#pragma unroll
        for (int s = 0; s < NV2; ++s)
        {
          const int v2 = lane + 64 * s;
          if (v2 >= 122) continue;
          val[q][s] = *reinterpret_cast<const double2*>(src + 2 * v2);
#pragma unroll
          for (int h = 0; h < 2; ++h)
          {
            const int d = 2 * v2 + h;
            if (d >= 243) continue;
            const int i = d / 81, rem = d - 81 * (d / 81);
            const int b = rem / 3, j = rem - 3 * (rem / 3);
            dst[q][s][h] = i * rowlen + pos[b] + j;
          }
        }
      }
#pragma unroll
      for (int q = 0; q < NB; ++q)
      {
        f += fv[q];
        if (WANT_K)
#pragma unroll
          for (int s = 0; s < NV2; ++s)
          {
            if (dst[q][s][0] >= 0) acc[dst[q][s][0]] += val[q][s].x;
            if (dst[q][s][1] >= 0) acc[dst[q][s][1]] += val[q][s].y;
          }
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

template <int NPE, bool WANT_K, bool OVERWRITE>
__global__ __launch_bounds__(64) void assemble_kernel(AssembleArgs A)
{
  constexpr int REC = int(record_doubles(NPE));
  constexpr int ROWLEN = 3 * NPE;
  constexpr int MAXROW = (NPE == 8) ? 81 : 375;
  __shared__ double acc[WANT_K ? 3 * MAXROW : 1];
  const int lane = threadIdx.x;
  for (int64_t r = blockIdx.x; r < A.n_rownodes; r += gridDim.x)
  {
    const int32_t row0 = A.rownode_row0[r];
    const int64_t base = A.rowptr[row0];
    const int rowlen = int(A.rowptr[row0 + 1] - base);
    if (WANT_K)
      for (int v = lane; v < 3 * rowlen; v += 64) acc[v] = 0.0;
    double f = 0.0;
    __syncthreads();
    const int64_t k0 = A.inc_ptr[r], k1 = A.inc_ptr[r + 1];
    // software pipeline: the next incidence's block-row is loaded while the current one is
    // summed into the LDS row image (one wavefront per row node, incidences in element order)
    constexpr int NV = (9 * NPE + 63) / 64;
    double cur[NV], nxt[NV];
    int dst[NV], ndst[NV];
    auto load = [&](int64_t k, double* val, int* off) {
      const double* src = A.scratch + k * REC;
      const uint16_t* pos = A.inc_pos + k * NPE;
#pragma unroll
      for (int s = 0; s < NV; ++s)
      {
        const int v = lane + 64 * s;
        off[s] = -1;
        val[s] = 0.0;
        if (WANT_K && v < 9 * NPE)
        {
          const int i = v / ROWLEN;
          const int rem = v - ROWLEN * i;
          const int b = rem / 3;
          const int j = rem - 3 * b;
          val[s] = src[v];
          off[s] = i * rowlen + pos[b] + j;
        }
      }
    };
    double fcur = 0.0, fnxt = 0.0;
    if (k0 < k1)
    {
      load(k0, cur, dst);
      if (lane < 3) fcur = A.scratch[k0 * REC + 9 * NPE + lane];
    }
    for (int64_t k = k0; k < k1; ++k)
    {
      if (k + 1 < k1)
      {
        load(k + 1, nxt, ndst);
        if (lane < 3) fnxt = A.scratch[(k + 1) * REC + 9 * NPE + lane];
      }
      if (WANT_K)
      {
#pragma unroll
        for (int s = 0; s < NV; ++s)
          if (dst[s] >= 0) acc[dst[s]] += cur[s];
      }
      f += fcur;
      __syncthreads();
#pragma unroll
      for (int s = 0; s < NV; ++s)
      {
        cur[s] = nxt[s];
        dst[s] = ndst[s];
      }
      fcur = fnxt;
    }
    if (WANT_K)
    {
      double* dst = A.K + base;  // the node's 3 rows are contiguous (checked at setup)
      for (int v = lane; v < 3 * rowlen; v += 64)
      {
        if (OVERWRITE)
          dst[v] = acc[v];
        else
          dst[v] += acc[v];
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

// ---------------------------------------------------------------------------------- launchers
static int grid_for(int64_t work, int cap)
{
  return int(work < cap ? (work > 0 ? work : 1) : cap);
}

// hex27 StVK pair phase on the matrix cores unless FCG_H27_MFMA=0 (A/B measurements)
static int h27_mfma()
{
  static const int on = [] {
    const char* e = std::getenv("FCG_H27_MFMA");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on;
}

hipError_t launch_element(const DeviceMesh& m, const double* d_u_col, bool want_k, hipStream_t stream)
{
  if (m.n_ele == 0) return hipSuccess;
  ElementArgs a{};
  a.mfma = h27_mfma();
  a.n_ele = m.n_ele;
  a.ele_nodes = m.ele_nodes;
  a.node_x = m.node_x;
  a.node_dof_col = m.node_dof_col;
  a.u_col = d_u_col;
  a.inc_of = m.inc_of;
  a.scratch = m.scratch;
  a.err = m.err;
  a.lambda = m.lambda;
  a.mu = m.mu;
  a.cdiag = m.cdiag;
  a.want_k = want_k ? 1 : 0;
  a.stamps = m.stamps;
  a.nh_c = m.nh_c;
  a.nh_beta = m.nh_beta;
  if (m.material == FCG_MAT_ELASTHYPER_COUPNEOHOOKE)
  {
    // general constitutive tangent: one workgroup per element (TotLag only, checked at create)
    if (m.npe == 8)
      hipLaunchKernelGGL((element_kernel<8, 1, 64, 1>), dim3(grid_for(m.n_ele, 256 * 32)), dim3(64),
          0, stream, a);
    else
      hipLaunchKernelGGL((element_kernel<27, 1, 256, 1>), dim3(grid_for(m.n_ele, 256 * 8)),
          dim3(256), 0, stream, a);
    return hipGetLastError();
  }
  if (m.npe == 8)
  {
    const int grid = grid_for((m.n_ele + H8_EPB - 1) / H8_EPB, 256 * 16);
    if (m.kinem == 0)
      hipLaunchKernelGGL((element_kernel_h8<0>), dim3(grid), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((element_kernel_h8<1>), dim3(grid), dim3(256), 0, stream, a);
  }
  else
  {
    const int grid = grid_for(m.n_ele, 256 * 8);
    if (m.kinem == 0)
      hipLaunchKernelGGL((element_kernel<27, 0, 256>), dim3(grid), dim3(256), 0, stream, a);
    else
      hipLaunchKernelGGL((element_kernel<27, 1, 256>), dim3(grid), dim3(256), 0, stream, a);
  }
  return hipGetLastError();
}

hipError_t launch_element_colored(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream)
{
  if (m.n_ele == 0 || m.npe != 27) return m.n_ele == 0 ? hipSuccess : hipErrorInvalidValue;
  ElementArgs a{};
  a.mfma = h27_mfma();
  a.n_ele = m.n_ele;
  a.ele_nodes = m.ele_nodes;
  a.node_x = m.node_x;
  a.node_dof_col = m.node_dof_col;
  a.u_col = d_u_col;
  a.inc_of = m.inc_of;
  a.scratch = nullptr;
  a.err = m.err;
  a.lambda = m.lambda;
  a.mu = m.mu;
  a.cdiag = m.cdiag;
  a.want_k = want_k ? 1 : 0;
  a.stamps = m.stamps;
  a.nh_c = m.nh_c;
  a.nh_beta = m.nh_beta;
  a.col_ele = m.col_ele;
  a.ele_ft = m.ele_ft;
  a.inc_row0 = m.inc_row0;
  a.inc_pos = m.inc_pos;
  a.rowptr = m.rowptr;
  a.K = d_K;
  a.fint = d_fint;
  for (int c = 0; c < 8; ++c)
  {
    a.e_begin = m.color_ptr[c];
    a.e_end = m.color_ptr[c + 1];
    if (a.e_end == a.e_begin) continue;
    const dim3 grid(grid_for(a.e_end - a.e_begin, 256 * 8)), block(256);
#define FCG_COL(KIN, MAT)                                                                          \
  if (overwrite)                                                                                   \
    hipLaunchKernelGGL((element_kernel<27, KIN, 256, MAT, 2>), grid, block, 0, stream, a);         \
  else                                                                                             \
    hipLaunchKernelGGL((element_kernel<27, KIN, 256, MAT, 1>), grid, block, 0, stream, a);
    if (m.material == FCG_MAT_ELASTHYPER_COUPNEOHOOKE)
    {
      FCG_COL(1, 1)
    }
    else if (m.kinem == 0)
    {
      FCG_COL(0, 0)
    }
    else
    {
      FCG_COL(1, 0)
    }
#undef FCG_COL
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_assemble(const DeviceMesh& m, bool want_k, bool overwrite, double* d_K,
    double* d_fint, hipStream_t stream)
{
  if (m.n_rownodes == 0) return hipSuccess;
  AssembleArgs a;
  a.n_rownodes = m.n_rownodes;
  a.inc_ptr = m.inc_ptr;
  a.rownode_row0 = m.rownode_row0;
  a.inc_pos = m.inc_pos;
  a.scratch = m.scratch;
  a.rowptr = m.rowptr;
  a.K = d_K;
  a.fint = d_fint;
  a.rows = nullptr;
  a.j_begin = 0;
  a.j_end = m.n_rownodes;
  a.rslot0 = nullptr;
  a.ring = 0;
  const int grid = grid_for(m.n_rownodes, 256 * 32);
#define FCG_ASM(NPE)                                                                               \
  if (want_k && overwrite)                                                                         \
    hipLaunchKernelGGL((assemble_kernel<NPE, true, true>), dim3(grid), dim3(64), 0, stream, a);    \
  else if (want_k)                                                                                 \
    hipLaunchKernelGGL((assemble_kernel<NPE, true, false>), dim3(grid), dim3(64), 0, stream, a);   \
  else if (overwrite)                                                                              \
    hipLaunchKernelGGL((assemble_kernel<NPE, false, true>), dim3(grid), dim3(64), 0, stream, a);   \
  else                                                                                             \
    hipLaunchKernelGGL((assemble_kernel<NPE, false, false>), dim3(grid), dim3(64), 0, stream, a);
  if (m.npe == 8)
  {
    FCG_ASM(8)
  }
  else
  {
    if (want_k && overwrite)
      hipLaunchKernelGGL((assemble27_kernel<true, true>), dim3(grid), dim3(64), 0, stream, a);
    else if (want_k)
      hipLaunchKernelGGL((assemble27_kernel<true, false>), dim3(grid), dim3(64), 0, stream, a);
    else if (overwrite)
      hipLaunchKernelGGL((assemble27_kernel<false, true>), dim3(grid), dim3(64), 0, stream, a);
    else
      hipLaunchKernelGGL((assemble27_kernel<false, false>), dim3(grid), dim3(64), 0, stream, a);
  }
#undef FCG_ASM
  return hipGetLastError();
}

// hex27 slab schedule: the row nodes completed by slab s (m.h27_asm_ptr), records in the ring
hipError_t launch_assemble27_slab(const DeviceMesh& m, int64_t s, bool want_k, bool overwrite,
    double* d_K, double* d_fint, hipStream_t stream)
{
  AssembleArgs a;
  a.n_rownodes = m.n_rownodes;
  a.inc_ptr = m.inc_ptr;
  a.rownode_row0 = m.rownode_row0;
  a.inc_pos = m.inc_pos;
  a.scratch = m.scratch;
  a.rowptr = m.rowptr;
  a.K = d_K;
  a.fint = d_fint;
  a.rows = m.h27_rows;
  a.j_begin = m.h27_asm_ptr[s];
  a.j_end = m.h27_asm_ptr[s + 1];
  a.rslot0 = m.h27_rslot0;
  a.ring = m.h27_ring;
  if (a.j_end <= a.j_begin) return hipSuccess;
  const int grid = grid_for(a.j_end - a.j_begin, 256 * 32);
  if (want_k && overwrite)
    hipLaunchKernelGGL((assemble27_kernel<true, true>), dim3(grid), dim3(64), 0, stream, a);
  else if (want_k)
    hipLaunchKernelGGL((assemble27_kernel<true, false>), dim3(grid), dim3(64), 0, stream, a);
  else if (overwrite)
    hipLaunchKernelGGL((assemble27_kernel<false, true>), dim3(grid), dim3(64), 0, stream, a);
  else
    hipLaunchKernelGGL((assemble27_kernel<false, false>), dim3(grid), dim3(64), 0, stream, a);
  return hipGetLastError();
}

}  // namespace fcg
