// fcg_hex8_element.hpp -- hex8 element math for the 8-lanes-per-element kernels (device code).
//
// One element is handled by 8 consecutive lanes.  Stage A: lane j = Gauss point g (J, J^-1, fac,
// N_XYZ of all 8 nodes, strain or F, StVK stress), plus the det J > 0 check at node j
// (4C_solid_3D_ele_calc_lib.hpp:380-496, 579-676, 682-799; 4C_mat_stvenantkirchhoff.cpp:169-177).
// Stage B: lane j = node row a: f_a = sum_g fac F S N_XYZ_a (calc_lib.hpp:851-860) and the pair
// blocks K_ab of a tournament schedule -- (a,a), (a,a+1), (a,a+2), (a,a+3) mod 8 and (a,a+4) for
// a < 4 -- that covers the 36 symmetric pairs of the element exactly once:
//   linear:  K_ab = sum_g fac [lambda a b^T + mu b a^T + mu (a.b) I]
//   TotLag:  K_ab = sum_g fac [lambda (Fa)(Fb)^T + mu (Fb)(Fa)^T + mu (a.b) F F^T + (a.S.b) I]
// (= B_a^T C B_b + K_geo of calc_lib.hpp:872-927 for the isotropic C of fill_cmat).
#pragma once

#include <hip/hip_runtime.h>

namespace fcg {

// LDS image of one element slot
template <int KIN>
struct H8Slot {
  double X[8][3];
  double U[8][3];
  double NX[8][8][3];  // [g][node][d]
  double fac[8];
  double S[8][6];      // PK2, Voigt xx yy zz xy yz zx
  double F[KIN ? 8 : 1][9];
  double pad[4];       // slot stride = 600 / 744 dwords: consecutive slots start in different banks
};

__device__ inline double h8_invert3x3(double* m)
{
  // invert3x3 of 4C_linalg_fixedsizematrix.hpp:1382-1409 (column-major m[r + 3c])
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
  m[3] = r3; m[4] = r4; m[7] = r7; m[5] = r5; m[6] = r6; m[8] = r8;
  m[0] = id * t00;
  m[1] = id * t10;
  m[2] = id * t20;
  return det;
}

struct StVK {
  double lambda, mu, cdiag;
};

// hex8 shape derivatives at a point (xi, eta, zeta) without a table: dN_n/dxi = sx (1 + sy eta)
// (1 + sz zeta) / 8 etc. (sx, sy, sz = the corner's parametric signs), from the 12 distinct
// products; with n a compile-time constant the sign is a negation modifier.
struct H8dN {
  double pyz[2][2], pxz[2][2], pxy[2][2];  // [sign index][sign index], 1 = +
};
__device__ inline H8dN h8_dn_products(double x, double y, double z)
{
  const double xp = 1.0 + x, xm = 1.0 - x, yp = 1.0 + y, ym = 1.0 - y, zp = 1.0 + z, zm = 1.0 - z;
  const double hyp = 0.125 * yp, hym = 0.125 * ym, hxp = 0.125 * xp, hxm = 0.125 * xm;
  H8dN p;
  p.pyz[0][0] = hym * zm; p.pyz[0][1] = hym * zp; p.pyz[1][0] = hyp * zm; p.pyz[1][1] = hyp * zp;
  p.pxz[0][0] = hxm * zm; p.pxz[0][1] = hxm * zp; p.pxz[1][0] = hxp * zm; p.pxz[1][1] = hxp * zp;
  p.pxy[0][0] = hxm * ym; p.pxy[0][1] = hxm * yp; p.pxy[1][0] = hxp * ym; p.pxy[1][1] = hxp * yp;
  return p;
}
// node n in 4C order: x sign (n & 3) in {1, 2}, y sign (n & 3) >= 2, z sign n >= 4
__device__ inline void h8_dn(const H8dN& p, int n, double& d0, double& d1, double& d2)
{
  const int ix = ((n & 3) == 1 || (n & 3) == 2), iy = (n & 3) >= 2, iz = n >= 4;
  d0 = ix ? p.pyz[iy][iz] : -p.pyz[iy][iz];
  d1 = iy ? p.pxz[ix][iz] : -p.pxz[ix][iz];
  d2 = iz ? p.pxy[ix][iy] : -p.pxy[ix][iy];
}

// Stage A for Gauss point g = j.  Returns 0, 1 (nodal det J <= 0) or 2 (singular).
template <int KIN>
__device__ inline int h8_stage_a(int j, H8Slot<KIN>& s, const double (*dN)[8][3],
    const double (*dNn)[8][3], double wg, const StVK& mat)
{
  double J[9], Jn[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) J[k] = Jn[k] = 0.0;
#pragma unroll
  for (int c = 0; c < 8; ++c)
  {
    const double x0 = s.X[c][0], x1 = s.X[c][1], x2 = s.X[c][2];
    const double d0 = dN[j][c][0], d1 = dN[j][c][1], d2 = dN[j][c][2];
    J[0] += d0 * x0; J[1] += d1 * x0; J[2] += d2 * x0;
    J[3] += d0 * x1; J[4] += d1 * x1; J[5] += d2 * x1;
    J[6] += d0 * x2; J[7] += d1 * x2; J[8] += d2 * x2;
    const double n0 = dNn[j][c][0], n1 = dNn[j][c][1], n2 = dNn[j][c][2];
    Jn[0] += n0 * x0; Jn[1] += n1 * x0; Jn[2] += n2 * x0;
    Jn[3] += n0 * x1; Jn[4] += n1 * x1; Jn[5] += n2 * x1;
    Jn[6] += n0 * x2; Jn[7] += n1 * x2; Jn[8] += n2 * x2;
  }
  int bad = 0;
  const double detn = h8_invert3x3(Jn);
  if (detn == 0.0) bad = 2;
  else if (!(detn > 0)) bad = 1;
  const double det = h8_invert3x3(J);
  if (det == 0.0) bad = 2;
  s.fac[j] = det * wg;
  double E[6] = {0, 0, 0, 0, 0, 0};
  double F[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 8; ++c)
  {
    const double d0 = dN[j][c][0], d1 = dN[j][c][1], d2 = dN[j][c][2];
    const double n0 = J[0] * d0 + J[3] * d1 + J[6] * d2;
    const double n1 = J[1] * d0 + J[4] * d1 + J[7] * d2;
    const double n2 = J[2] * d0 + J[5] * d1 + J[8] * d2;
    s.NX[j][c][0] = n0;
    s.NX[j][c][1] = n1;
    s.NX[j][c][2] = n2;
    const double u0 = s.U[c][0], u1 = s.U[c][1], u2 = s.U[c][2];
    if (KIN == 0)
    {
      E[0] += n0 * u0;
      E[1] += n1 * u1;
      E[2] += n2 * u2;
      E[3] += n1 * u0 + n0 * u1;
      E[4] += n2 * u1 + n1 * u2;
      E[5] += n2 * u0 + n0 * u2;
    }
    else
    {
      // hex8: F = x N_XYZ^T from current coordinates (calc_lib.hpp:585-595)
      const double q0 = s.X[c][0] + u0, q1 = s.X[c][1] + u1, q2 = s.X[c][2] + u2;
      F[0] += q0 * n0; F[1] += q1 * n0; F[2] += q2 * n0;
      F[3] += q0 * n1; F[4] += q1 * n1; F[5] += q2 * n1;
      F[6] += q0 * n2; F[7] += q1 * n2; F[8] += q2 * n2;
    }
  }
  if (KIN == 1)
  {
    double Fi[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) Fi[k] = F[k];
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
#pragma unroll
    for (int k = 0; k < 9; ++k) s.F[j][k] = F[k];
  }
  double* S = s.S[j];
  S[0] = mat.cdiag * E[0] + mat.lambda * E[1] + mat.lambda * E[2];
  S[1] = mat.lambda * E[0] + mat.cdiag * E[1] + mat.lambda * E[2];
  S[2] = mat.lambda * E[0] + mat.lambda * E[1] + mat.cdiag * E[2];
  S[3] = mat.mu * E[3];
  S[4] = mat.mu * E[4];
  S[5] = mat.mu * E[5];
  return bad;
}

__device__ inline int h8_npair(int a) { return a < 4 ? 5 : 4; }

// Stage B for node row a: K[p] (column-major 3x3) of pair (a, (a+p)&7), p < h8_npair(a); f_a.
template <int KIN>
__device__ inline void h8_stage_b(int a, const H8Slot<KIN>& s, const StVK& mat, bool want_k,
    double (&K)[5][9], double (&f)[3])
{
  double G[5][9];
  double H[KIN ? 5 : 1][6];
  double geo[KIN ? 5 : 1];
  const int npair = h8_npair(a);
#pragma unroll
  for (int p = 0; p < 5; ++p)
#pragma unroll
    for (int k = 0; k < 9; ++k) G[p][k] = 0.0;
  if (KIN == 1)
  {
#pragma unroll
    for (int p = 0; p < 5; ++p)
    {
#pragma unroll
      for (int k = 0; k < 6; ++k) H[p][k] = 0.0;
      geo[p] = 0.0;
    }
  }
  double f0 = 0.0, f1 = 0.0, f2 = 0.0;
#pragma unroll 1
  for (int g = 0; g < 8; ++g)
  {
    const double fc = s.fac[g];
    const double* S = s.S[g];
    const double a0 = s.NX[g][a][0], a1 = s.NX[g][a][1], a2 = s.NX[g][a][2];
    double t0 = S[0] * a0 + S[3] * a1 + S[5] * a2;
    double t1 = S[3] * a0 + S[1] * a1 + S[4] * a2;
    double t2 = S[5] * a0 + S[4] * a1 + S[2] * a2;
    double pa0 = a0, pa1 = a1, pa2 = a2;
    double M[6];
    const double* F = s.F[KIN ? g : 0];
    if (KIN == 1)
    {
      const double s0 = F[0] * t0 + F[3] * t1 + F[6] * t2;
      const double s1 = F[1] * t0 + F[4] * t1 + F[7] * t2;
      const double s2 = F[2] * t0 + F[5] * t1 + F[8] * t2;
      t0 = s0;
      t1 = s1;
      t2 = s2;
      pa0 = F[0] * a0 + F[3] * a1 + F[6] * a2;
      pa1 = F[1] * a0 + F[4] * a1 + F[7] * a2;
      pa2 = F[2] * a0 + F[5] * a1 + F[8] * a2;
      M[0] = F[0] * F[0] + F[3] * F[3] + F[6] * F[6];
      M[1] = F[1] * F[1] + F[4] * F[4] + F[7] * F[7];
      M[2] = F[2] * F[2] + F[5] * F[5] + F[8] * F[8];
      M[3] = F[0] * F[1] + F[3] * F[4] + F[6] * F[7];
      M[4] = F[1] * F[2] + F[4] * F[5] + F[7] * F[8];
      M[5] = F[2] * F[0] + F[5] * F[3] + F[8] * F[6];
    }
    f0 += fc * t0;
    f1 += fc * t1;
    f2 += fc * t2;
    if (!want_k) continue;
    const double fa0 = fc * pa0, fa1 = fc * pa1, fa2 = fc * pa2;
#pragma unroll
    for (int p = 0; p < 5; ++p)
    {
      if (p >= npair) break;
      const int b = (a + p) & 7;
      const double b0 = s.NX[g][b][0], b1 = s.NX[g][b][1], b2 = s.NX[g][b][2];
      double q0 = b0, q1 = b1, q2 = b2;
      if (KIN == 1)
      {
        q0 = F[0] * b0 + F[3] * b1 + F[6] * b2;
        q1 = F[1] * b0 + F[4] * b1 + F[7] * b2;
        q2 = F[2] * b0 + F[5] * b1 + F[8] * b2;
      }
      G[p][0] += fa0 * q0; G[p][3] += fa0 * q1; G[p][6] += fa0 * q2;
      G[p][1] += fa1 * q0; G[p][4] += fa1 * q1; G[p][7] += fa1 * q2;
      G[p][2] += fa2 * q0; G[p][5] += fa2 * q1; G[p][8] += fa2 * q2;
      if (KIN == 1)
      {
        const double t = fc * (a0 * b0 + a1 * b1 + a2 * b2);
#pragma unroll
        for (int k = 0; k < 6; ++k) H[p][k] += t * M[k];
        const double sb0 = S[0] * b0 + S[3] * b1 + S[5] * b2;
        const double sb1 = S[3] * b0 + S[1] * b1 + S[4] * b2;
        const double sb2 = S[5] * b0 + S[4] * b1 + S[2] * b2;
        geo[p] += fc * (a0 * sb0 + a1 * sb1 + a2 * sb2);
      }
    }
  }
  f[0] = f0;
  f[1] = f1;
  f[2] = f2;
  if (!want_k) return;
  const double lam = mat.lambda, mu = mat.mu;
#pragma unroll
  for (int p = 0; p < 5; ++p)
  {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int q = 0; q < 3; ++q) K[p][r + 3 * q] = lam * G[p][r + 3 * q] + mu * G[p][q + 3 * r];
    if (KIN == 0)
    {
      const double tr = mu * (G[p][0] + G[p][4] + G[p][8]);
      K[p][0] += tr;
      K[p][4] += tr;
      K[p][8] += tr;
    }
    else
    {
      K[p][0] += mu * H[p][0] + geo[p];
      K[p][4] += mu * H[p][1] + geo[p];
      K[p][8] += mu * H[p][2] + geo[p];
      K[p][1] += mu * H[p][3]; K[p][3] += mu * H[p][3];
      K[p][5] += mu * H[p][4]; K[p][7] += mu * H[p][4];
      K[p][2] += mu * H[p][5]; K[p][6] += mu * H[p][5];
    }
  }
}

}  // namespace fcg
