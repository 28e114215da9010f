/*
 * fourc_oracle.c -- CPU restatement of 4C's SOLID hex8/hex27 + StVK evaluation and the
 * Epetra-style global assembly.  TEST INFRASTRUCTURE ONLY (see fourc_oracle.h).
 *
 * Conventions follow Core::LinAlg::Matrix (column-major, 4C_linalg_fixedsizematrix.hpp):
 *   A(r, c) of an R x C matrix lives at A[r + R*c].
 * The dense kernels below reproduce the summation order of the reference's fixed-size
 * multiply_nn / multiply_nt / multiply_tn (4C_linalg_fixedsizematrix.hpp:907-1000,1224-1245):
 * every dot product starts with its first product and accumulates in index order, and the
 * "update" forms compute out = out*outfac + infac*tmp.
 */
#include "fourc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXN 27
#define MAXDOF 81

int orc_num_nodes(int celltype) { return celltype == ORC_HEX27 ? 27 : 8; }
int orc_num_gp(int celltype) { return celltype == ORC_HEX27 ? 27 : 8; }

/* ---------------------------------------------------------------------------------------
 * Gauss rules: 4C_fem_general_utils_integration.cpp:74-106 (hex_8point) and :130-245
 * (hex_27point).  hex27 uses the truncated constants xi3 = 0.7745966692415 and
 * w = 0.5555555555556 / 0.8888888888889 exactly as the reference does.
 * ------------------------------------------------------------------------------------- */
void orc_gauss_points(int celltype, double* xi, double* w)
{
  if (celltype == ORC_HEX8)
  {
    const double xi2 = 1.0 / sqrt(3.0);
    static const int sgn[8][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1},
        {-1, -1, 1}, {1, -1, 1}, {1, 1, 1}, {-1, 1, 1}};
    for (int g = 0; g < 8; ++g)
    {
      for (int d = 0; d < 3; ++d) xi[3 * g + d] = sgn[g][d] * xi2;
      w[g] = 1.0;
    }
    return;
  }
  /* hex_27point: point order :134-214, weights :215-243 */
  const double xi3 = 0.7745966692415;
  static const int pos[27][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1}, {-1, -1, 1},
      {1, -1, 1}, {1, 1, 1}, {-1, 1, 1}, {0, -1, -1}, {1, 0, -1}, {0, 1, -1}, {-1, 0, -1},
      {-1, -1, 0}, {1, -1, 0}, {1, 1, 0}, {-1, 1, 0}, {0, -1, 1}, {1, 0, 1}, {0, 1, 1}, {-1, 0, 1},
      {0, 0, -1}, {0, -1, 0}, {1, 0, 0}, {0, 1, 0}, {-1, 0, 0}, {0, 0, 1}, {0, 0, 0}};
  const double w1 = 0.5555555555556;
  const double w2 = 0.8888888888889;
  const double w3 = w1;
  for (int g = 0; g < 27; ++g)
    for (int d = 0; d < 3; ++d) xi[3 * g + d] = pos[g][d] * xi3;
  /* qwgt[g] = wa*wb*wc, multiplied left to right as in the reference */
  const double* wt[27][3] = {{&w1, &w1, &w1}, {&w3, &w1, &w1}, {&w3, &w3, &w1}, {&w1, &w3, &w1},
      {&w1, &w1, &w3}, {&w3, &w1, &w3}, {&w3, &w3, &w3}, {&w1, &w3, &w3}, {&w2, &w1, &w1},
      {&w3, &w2, &w1}, {&w2, &w3, &w1}, {&w1, &w2, &w1}, {&w1, &w1, &w2}, {&w3, &w1, &w2},
      {&w3, &w3, &w2}, {&w1, &w3, &w2}, {&w2, &w1, &w3}, {&w3, &w2, &w3}, {&w2, &w3, &w3},
      {&w1, &w2, &w3}, {&w2, &w2, &w1}, {&w2, &w1, &w2}, {&w3, &w2, &w2}, {&w2, &w3, &w2},
      {&w1, &w2, &w2}, {&w2, &w2, &w3}, {&w2, &w2, &w2}};
  for (int g = 0; g < 27; ++g) w[g] = *wt[g][0] * *wt[g][1] * *wt[g][2];
}

/* Parameter-space nodes (4C_fem_general_utils_local_connectivity_matrices.hpp:291-297). */
static const double hex27_nodes_ref[27][3] = {{-1.0, -1.0, -1.0}, {1.0, -1.0, -1.0},
    {1.0, 1.0, -1.0}, {-1.0, 1.0, -1.0}, {-1.0, -1.0, 1.0}, {1.0, -1.0, 1.0}, {1.0, 1.0, 1.0},
    {-1.0, 1.0, 1.0}, {0.0, -1.0, -1.0}, {1.0, 0.0, -1.0}, {0.0, 1.0, -1.0}, {-1.0, 0.0, -1.0},
    {-1.0, -1.0, 0.0}, {1.0, -1.0, 0.0}, {1.0, 1.0, 0.0}, {-1.0, 1.0, 0.0}, {0.0, -1.0, 1.0},
    {1.0, 0.0, 1.0}, {0.0, 1.0, 1.0}, {-1.0, 0.0, 1.0}, {0.0, 0.0, -1.0}, {0.0, -1.0, 0.0},
    {1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {-1.0, 0.0, 0.0}, {0.0, 0.0, 1.0}, {0.0, 0.0, 0.0}};

void orc_node_param_coords(int celltype, double* xi)
{
  const int n = orc_num_nodes(celltype);
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d) xi[3 * i + d] = hex27_nodes_ref[i][d];
}

/* ---------------------------------------------------------------------------------------
 * Shape functions (4C_fem_general_utils_fem_shapefunctions.hpp:53-72 hex8, :190-229 hex27)
 * ------------------------------------------------------------------------------------- */
void orc_shape(int celltype, const double* xi, double* funct)
{
  const double r = xi[0], s = xi[1], t = xi[2];
  if (celltype == ORC_HEX8)
  {
    const double Q18 = 1.0 / 8.0;
    const double rp = 1.0 + r, rm = 1.0 - r, sp = 1.0 + s, sm = 1.0 - s, tp = 1.0 + t,
                 tm = 1.0 - t;
    funct[0] = Q18 * rm * sm * tm;
    funct[1] = Q18 * rp * sm * tm;
    funct[2] = Q18 * rp * sp * tm;
    funct[3] = Q18 * rm * sp * tm;
    funct[4] = Q18 * rm * sm * tp;
    funct[5] = Q18 * rp * sm * tp;
    funct[6] = Q18 * rp * sp * tp;
    funct[7] = Q18 * rm * sp * tp;
    return;
  }
  const double rm1 = 0.5 * r * (r - 1.0), r00 = (1.0 - r * r), rp1 = 0.5 * r * (r + 1.0);
  const double sm1 = 0.5 * s * (s - 1.0), s00 = (1.0 - s * s), sp1 = 0.5 * s * (s + 1.0);
  const double tm1 = 0.5 * t * (t - 1.0), t00 = (1.0 - t * t), tp1 = 0.5 * t * (t + 1.0);
  funct[0] = rm1 * sm1 * tm1;
  funct[1] = rp1 * sm1 * tm1;
  funct[2] = rp1 * sp1 * tm1;
  funct[3] = rm1 * sp1 * tm1;
  funct[4] = rm1 * sm1 * tp1;
  funct[5] = rp1 * sm1 * tp1;
  funct[6] = rp1 * sp1 * tp1;
  funct[7] = rm1 * sp1 * tp1;
  funct[8] = r00 * sm1 * tm1;
  funct[9] = s00 * tm1 * rp1;
  funct[10] = r00 * tm1 * sp1;
  funct[11] = s00 * rm1 * tm1;
  funct[12] = t00 * rm1 * sm1;
  funct[13] = t00 * sm1 * rp1;
  funct[14] = t00 * rp1 * sp1;
  funct[15] = t00 * rm1 * sp1;
  funct[16] = r00 * sm1 * tp1;
  funct[17] = s00 * rp1 * tp1;
  funct[18] = r00 * sp1 * tp1;
  funct[19] = s00 * rm1 * tp1;
  funct[20] = r00 * s00 * tm1;
  funct[21] = r00 * t00 * sm1;
  funct[22] = s00 * t00 * rp1;
  funct[23] = r00 * t00 * sp1;
  funct[24] = s00 * t00 * rm1;
  funct[25] = r00 * s00 * tp1;
  funct[26] = r00 * s00 * t00;
}

/* First derivatives (:386-426 hex8, :683-788 hex27); deriv1(d, node) -> dN[3*node + d]. */
void orc_shape_deriv1(int celltype, const double* xi, double* dN)
{
  const double r = xi[0], s = xi[1], t = xi[2];
#define D(d, n) dN[3 * (n) + (d)]
  if (celltype == ORC_HEX8)
  {
    const double Q18 = 1.0 / 8.0;
    const double rp = 1.0 + r, rm = 1.0 - r, sp = 1.0 + s, sm = 1.0 - s, tp = 1.0 + t,
                 tm = 1.0 - t;
    D(0, 0) = -Q18 * sm * tm;
    D(1, 0) = -Q18 * tm * rm;
    D(2, 0) = -Q18 * rm * sm;
    D(0, 1) = Q18 * sm * tm;
    D(1, 1) = -Q18 * tm * rp;
    D(2, 1) = -Q18 * rp * sm;
    D(0, 2) = Q18 * sp * tm;
    D(1, 2) = Q18 * tm * rp;
    D(2, 2) = -Q18 * rp * sp;
    D(0, 3) = -Q18 * sp * tm;
    D(1, 3) = Q18 * tm * rm;
    D(2, 3) = -Q18 * rm * sp;
    D(0, 4) = -Q18 * sm * tp;
    D(1, 4) = -Q18 * tp * rm;
    D(2, 4) = Q18 * rm * sm;
    D(0, 5) = Q18 * sm * tp;
    D(1, 5) = -Q18 * tp * rp;
    D(2, 5) = Q18 * rp * sm;
    D(0, 6) = Q18 * sp * tp;
    D(1, 6) = Q18 * tp * rp;
    D(2, 6) = Q18 * rp * sp;
    D(0, 7) = -Q18 * sp * tp;
    D(1, 7) = Q18 * tp * rm;
    D(2, 7) = Q18 * rm * sp;
    return;
  }
  const double rm1 = 0.5 * r * (r - 1.0), r00 = (1.0 - r * r), rp1 = 0.5 * r * (r + 1.0);
  const double sm1 = 0.5 * s * (s - 1.0), s00 = (1.0 - s * s), sp1 = 0.5 * s * (s + 1.0);
  const double tm1 = 0.5 * t * (t - 1.0), t00 = (1.0 - t * t), tp1 = 0.5 * t * (t + 1.0);
  const double drm1 = r - 0.5, dr00 = -2.0 * r, drp1 = r + 0.5;
  const double dsm1 = s - 0.5, ds00 = -2.0 * s, dsp1 = s + 0.5;
  const double dtm1 = t - 0.5, dt00 = -2.0 * t, dtp1 = t + 0.5;
  D(0, 0) = sm1 * tm1 * drm1;
  D(0, 1) = sm1 * tm1 * drp1;
  D(0, 2) = tm1 * sp1 * drp1;
  D(0, 3) = tm1 * sp1 * drm1;
  D(0, 4) = sm1 * tp1 * drm1;
  D(0, 5) = sm1 * tp1 * drp1;
  D(0, 6) = sp1 * tp1 * drp1;
  D(0, 7) = sp1 * tp1 * drm1;
  D(0, 8) = sm1 * tm1 * dr00;
  D(0, 9) = s00 * tm1 * drp1;
  D(0, 10) = tm1 * sp1 * dr00;
  D(0, 11) = s00 * tm1 * drm1;
  D(0, 12) = t00 * sm1 * drm1;
  D(0, 13) = t00 * sm1 * drp1;
  D(0, 14) = t00 * sp1 * drp1;
  D(0, 15) = t00 * sp1 * drm1;
  D(0, 16) = sm1 * tp1 * dr00;
  D(0, 17) = s00 * tp1 * drp1;
  D(0, 18) = sp1 * tp1 * dr00;
  D(0, 19) = s00 * tp1 * drm1;
  D(0, 20) = s00 * tm1 * dr00;
  D(0, 21) = t00 * sm1 * dr00;
  D(0, 22) = s00 * t00 * drp1;
  D(0, 23) = t00 * sp1 * dr00;
  D(0, 24) = s00 * t00 * drm1;
  D(0, 25) = s00 * tp1 * dr00;
  D(0, 26) = s00 * t00 * dr00;

  D(1, 0) = rm1 * tm1 * dsm1;
  D(1, 1) = tm1 * rp1 * dsm1;
  D(1, 2) = tm1 * rp1 * dsp1;
  D(1, 3) = rm1 * tm1 * dsp1;
  D(1, 4) = rm1 * tp1 * dsm1;
  D(1, 5) = rp1 * tp1 * dsm1;
  D(1, 6) = rp1 * tp1 * dsp1;
  D(1, 7) = rm1 * tp1 * dsp1;
  D(1, 8) = r00 * tm1 * dsm1;
  D(1, 9) = tm1 * rp1 * ds00;
  D(1, 10) = r00 * tm1 * dsp1;
  D(1, 11) = rm1 * tm1 * ds00;
  D(1, 12) = t00 * rm1 * dsm1;
  D(1, 13) = t00 * rp1 * dsm1;
  D(1, 14) = t00 * rp1 * dsp1;
  D(1, 15) = t00 * rm1 * dsp1;
  D(1, 16) = r00 * tp1 * dsm1;
  D(1, 17) = rp1 * tp1 * ds00;
  D(1, 18) = r00 * tp1 * dsp1;
  D(1, 19) = rm1 * tp1 * ds00;
  D(1, 20) = r00 * tm1 * ds00;
  D(1, 21) = r00 * t00 * dsm1;
  D(1, 22) = t00 * rp1 * ds00;
  D(1, 23) = r00 * t00 * dsp1;
  D(1, 24) = t00 * rm1 * ds00;
  D(1, 25) = r00 * tp1 * ds00;
  D(1, 26) = r00 * t00 * ds00;

  D(2, 0) = rm1 * sm1 * dtm1;
  D(2, 1) = sm1 * rp1 * dtm1;
  D(2, 2) = rp1 * sp1 * dtm1;
  D(2, 3) = rm1 * sp1 * dtm1;
  D(2, 4) = rm1 * sm1 * dtp1;
  D(2, 5) = sm1 * rp1 * dtp1;
  D(2, 6) = rp1 * sp1 * dtp1;
  D(2, 7) = rm1 * sp1 * dtp1;
  D(2, 8) = r00 * sm1 * dtm1;
  D(2, 9) = s00 * rp1 * dtm1;
  D(2, 10) = r00 * sp1 * dtm1;
  D(2, 11) = s00 * rm1 * dtm1;
  D(2, 12) = rm1 * sm1 * dt00;
  D(2, 13) = sm1 * rp1 * dt00;
  D(2, 14) = rp1 * sp1 * dt00;
  D(2, 15) = rm1 * sp1 * dt00;
  D(2, 16) = r00 * sm1 * dtp1;
  D(2, 17) = s00 * rp1 * dtp1;
  D(2, 18) = r00 * sp1 * dtp1;
  D(2, 19) = s00 * rm1 * dtp1;
  D(2, 20) = r00 * s00 * dtm1;
  D(2, 21) = r00 * sm1 * dt00;
  D(2, 22) = s00 * rp1 * dt00;
  D(2, 23) = r00 * sp1 * dt00;
  D(2, 24) = s00 * rm1 * dt00;
  D(2, 25) = r00 * s00 * dtp1;
  D(2, 26) = r00 * s00 * dt00;
#undef D
}

/* ---------------------------------------------------------------------------------------
 * Fixed-size dense kernels with the reference's summation order
 * (4C_linalg_fixedsizematrix.hpp:907-1000 plain, :1224-1245 "out*outfac + infac*tmp").
 * ------------------------------------------------------------------------------------- */
/* out(i x k) = outfac*out + infac * left(i x j) * right(j x k) */
static void mm_nn(double* out, double outfac, double infac, const double* l, const double* r,
    int i, int j, int k, int update)
{
  for (int c1 = 0; c1 < k; ++c1)
    for (int c2 = 0; c2 < i; ++c2)
    {
      double tmp = l[c2] * r[j * c1];
      for (int c3 = 1; c3 < j; ++c3) tmp += l[c2 + c3 * i] * r[j * c1 + c3];
      double* o = &out[c2 + i * c1];
      *o = update ? (*o) * outfac + infac * tmp : infac * tmp;
    }
}
/* out(i x k) = outfac*out + infac * left(i x j) * right(k x j)^T */
static void mm_nt(double* out, double outfac, double infac, const double* l, const double* r,
    int i, int j, int k, int update)
{
  for (int c1 = 0; c1 < k; ++c1)
    for (int c2 = 0; c2 < i; ++c2)
    {
      double tmp = l[c2] * r[c1];
      for (int c3 = 1; c3 < j; ++c3) tmp += l[c2 + c3 * i] * r[c1 + c3 * k];
      double* o = &out[c2 + i * c1];
      *o = update ? (*o) * outfac + infac * tmp : infac * tmp;
    }
}
/* out(i x k) = outfac*out + infac * left(j x i)^T * right(j x k) */
static void mm_tn(double* out, double outfac, double infac, const double* l, const double* r,
    int i, int j, int k, int update)
{
  for (int c1 = 0; c1 < k; ++c1)
    for (int c2 = 0; c2 < i; ++c2)
    {
      double tmp = l[j * c2] * r[j * c1];
      for (int c3 = 1; c3 < j; ++c3) tmp += l[j * c2 + c3] * r[j * c1 + c3];
      double* o = &out[c2 + i * c1];
      *o = update ? (*o) * outfac + infac * tmp : infac * tmp;
    }
}

/* invert3x3 (4C_linalg_fixedsizematrix.hpp:1382-1409); returns det, 0 if singular. */
static double invert3x3(double* mat)
{
  const double tmp00 = mat[1 + 1 * 3] * mat[2 + 2 * 3] - mat[2 + 1 * 3] * mat[1 + 2 * 3];
  const double tmp10 = mat[2] * mat[1 + 2 * 3] - mat[1] * mat[2 + 2 * 3];
  const double tmp20 = mat[1] * mat[2 + 1 * 3] - mat[2] * mat[1 + 1 * 3];
  const double det = mat[0] * tmp00 + mat[1 * 3] * tmp10 + mat[2 * 3] * tmp20;
  if (det == 0.0) return 0.0;
  const double invdet = 1.0 / det;
  const double tmp01 = mat[1 * 3];
  const double tmp11 = mat[1 + 1 * 3];
  const double tmp12 = mat[1 + 2 * 3];
  mat[1 * 3] = invdet * (mat[2 + 1 * 3] * mat[2 * 3] - tmp01 * mat[2 + 2 * 3]);
  mat[1 + 1 * 3] = invdet * (mat[0] * mat[2 + 2 * 3] - mat[2] * mat[2 * 3]);
  mat[1 + 2 * 3] = invdet * (mat[1] * mat[2 * 3] - mat[0] * tmp12);
  mat[2 + 1 * 3] = invdet * (mat[2] * tmp01 - mat[0] * mat[2 + 1 * 3]);
  mat[2 * 3] = invdet * (tmp01 * tmp12 - tmp11 * mat[2 * 3]);
  mat[2 + 2 * 3] = invdet * (mat[0] * tmp11 - mat[1] * tmp01);
  mat[0] = invdet * tmp00;
  mat[1] = invdet * tmp10;
  mat[2] = invdet * tmp20;
  return det;
}

/* ---------------------------------------------------------------------------------------
 * StVenantKirchhoff (4C_mat_stvenantkirchhoff.cpp)
 * ------------------------------------------------------------------------------------- */
void orc_stvk_cmat(double Emod, double nu, double* cmat)
{
  /* fill_cmat :115-145 */
  const double mfac = Emod / ((1.0 + nu) * (1.0 - 2.0 * nu));
  for (int i = 0; i < 36; ++i) cmat[i] = 0.0;
#define C(i, j) cmat[(i) + 6 * (j)]
  C(0, 0) = mfac * (1.0 - nu);
  C(0, 1) = mfac * nu;
  C(0, 2) = mfac * nu;
  C(1, 0) = mfac * nu;
  C(1, 1) = mfac * (1.0 - nu);
  C(1, 2) = mfac * nu;
  C(2, 0) = mfac * nu;
  C(2, 1) = mfac * nu;
  C(2, 2) = mfac * (1.0 - nu);
  C(3, 3) = mfac * 0.5 * (1.0 - 2.0 * nu);
  C(4, 4) = mfac * 0.5 * (1.0 - 2.0 * nu);
  C(5, 5) = mfac * 0.5 * (1.0 - 2.0 * nu);
#undef C
}

void orc_stvk_evaluate(double E, double nu, const double* glstrain, double* stress, double* cmat)
{
  /* :169-177: setup_cmat; stress = C . E (multiply_nn) */
  double c[36];
  orc_stvk_cmat(E, nu, c);
  if (cmat) memcpy(cmat, c, sizeof(c));
  mm_nn(stress, 0.0, 1.0, c, glstrain, 6, 6, 1, 0);
}

double orc_stvk_strain_energy(double E, double nu, const double* glstrain)
{
  /* :184-194 */
  double c[36], stress[6];
  orc_stvk_cmat(E, nu, c);
  mm_nn(stress, 0.0, 1.0, c, glstrain, 6, 6, 1, 0);
  double psi = 0.0;
  for (int k = 0; k < 6; ++k) psi += glstrain[k] * stress[k];
  psi /= 2.0;
  return psi;
}

/* ---------------------------------------------------------------------------------------
 * Mat::ElastHyper with one ELAST_CoupNeoHooke summand (isotropic, principal invariants):
 * elast_hyper_evaluate (4C_mat_elasthyper_service.cpp:19-78) -> right Cauchy-Green (:80-88),
 * Voigt inverse / principal invariants (4C_linalg_fixedsizematrix_voigt_notation.hpp:76-101,
 * .cpp:188-207), CoupNeoHooke::add_derivatives_principal (4C_mat_elast_coupneohooke.cpp),
 * calculate_gamma_delta (:413-432), elast_hyper_add_isotropic_stress_cmat (:162-215) with
 * add_holzapfel_product (4C_linalg_fixedsizematrix_tensor_products.cpp:264-312).
 * Strain-like Voigt vectors carry doubled shears; stress-like ones do not.
 * ------------------------------------------------------------------------------------- */
static const double voigt_unscale_strain[6] = {1.0, 1.0, 1.0, 0.5, 0.5, 0.5};
static const double voigt_scale_strain[6] = {1.0, 1.0, 1.0, 2.0, 2.0, 2.0};

static double voigt_triple(const double* v, int i, int j, int k)
{
  return v[i] * voigt_unscale_strain[i] * v[j] * voigt_unscale_strain[j] * v[k] *
         voigt_unscale_strain[k];
}

static double voigt_det_strain(const double* v)
{
  return voigt_triple(v, 0, 1, 2) + 2 * voigt_triple(v, 3, 4, 5) - voigt_triple(v, 1, 5, 5) -
         voigt_triple(v, 2, 3, 3) - voigt_triple(v, 0, 4, 4);
}

void orc_elasthyper_coupneohooke(double E, double nu, const double* glstrain, double* stress,
    double* cmat)
{
  const double* us = voigt_unscale_strain;
  const double* sc = voigt_scale_strain;
  /* Mat::Elastic::PAR::CoupNeoHooke: c = E / (4 (1 + nu)), beta = nu / (1 - 2 nu) */
  const double c = E / (4.0 * (1.0 + nu));
  const double beta = nu / (1.0 - 2.0 * nu);
  const double id2[6] = {1.0, 1.0, 1.0, 0.0, 0.0, 0.0};
  double C[6], iC[6], prinv[3], dPI[3] = {0, 0, 0}, ddPII[6] = {0, 0, 0, 0, 0, 0};
  /* C = 2 E + I (strain-like) */
  for (int i = 0; i < 6; ++i) C[i] = 2.0 * glstrain[i];
  for (int i = 0; i < 3; ++i) C[i] += 1.0;
  /* VoigtUtils<strain>::inverse_tensor */
  const double det = voigt_det_strain(C);
  iC[0] = (C[1] * C[2] - us[4] * us[4] * C[4] * C[4]) / det * sc[0];
  iC[1] = (C[0] * C[2] - us[5] * us[5] * C[5] * C[5]) / det * sc[1];
  iC[2] = (C[0] * C[1] - us[3] * us[3] * C[3] * C[3]) / det * sc[2];
  iC[3] = (us[5] * us[4] * C[5] * C[4] - us[3] * us[2] * C[3] * C[2]) / det * sc[3];
  iC[4] = (us[3] * us[5] * C[3] * C[5] - us[0] * us[4] * C[0] * C[4]) / det * sc[4];
  iC[5] = (us[3] * us[4] * C[3] * C[4] - us[5] * us[1] * C[5] * C[1]) / det * sc[5];
  /* invariants_principal */
  prinv[0] = C[0] + C[1] + C[2];
  prinv[1] = 0.5 * (prinv[0] * prinv[0] - C[0] * C[0] - C[1] * C[1] - C[2] * C[2]) -
             C[3] * C[3] * us[3] * us[3] - C[4] * C[4] * us[4] * us[4] - C[5] * C[5] * us[5] * us[5];
  prinv[2] = voigt_det_strain(C);
  /* CoupNeoHooke::add_derivatives_principal */
  dPI[0] += c;
  if (prinv[2] > 0)
  {
    const double p = exp(log(prinv[2]) * (-beta - 1.));
    dPI[2] -= c * p;
    ddPII[2] += c * (beta + 1.) * p / prinv[2];
  }
  else
    dPI[2] = ddPII[2] = NAN;
  /* calculate_gamma_delta (Holzapfel p. 216, 261) */
  double gamma[3], delta[8];
  gamma[0] = 2. * (dPI[0] + prinv[0] * dPI[1]);
  gamma[1] = -2. * dPI[1];
  gamma[2] = 2. * prinv[2] * dPI[2];
  delta[0] = 4. * (ddPII[0] + 2. * prinv[0] * ddPII[5] + dPI[1] + prinv[0] * prinv[0] * ddPII[1]);
  delta[1] = -4. * (ddPII[5] + prinv[0] * ddPII[1]);
  delta[2] = 4. * (prinv[2] * ddPII[4] + prinv[0] * prinv[2] * ddPII[3]);
  delta[3] = 4. * ddPII[1];
  delta[4] = -4. * prinv[2] * ddPII[3];
  delta[5] = 4. * (prinv[2] * dPI[2] + prinv[2] * prinv[2] * ddPII[2]);
  delta[6] = -4. * prinv[2] * dPI[2];
  delta[7] = -4. * dPI[1];
  /* stress-like C and C^-1 */
  double Cs[6], iCs[6];
  for (int i = 0; i < 6; ++i)
  {
    Cs[i] = us[i] * C[i];
    iCs[i] = us[i] * iC[i];
  }
  for (int i = 0; i < 6; ++i) stress[i] = 0.0;
  for (int i = 0; i < 36; ++i) cmat[i] = 0.0;
  for (int i = 0; i < 6; ++i) stress[i] = 1.0 * stress[i] + gamma[0] * id2[i];
  for (int i = 0; i < 6; ++i) stress[i] = 1.0 * stress[i] + gamma[1] * Cs[i];
  for (int i = 0; i < 6; ++i) stress[i] = 1.0 * stress[i] + gamma[2] * iCs[i];
  mm_nt(cmat, 1.0, delta[0], id2, id2, 6, 1, 6, 1);
  mm_nt(cmat, 1.0, delta[1], id2, Cs, 6, 1, 6, 1);
  mm_nt(cmat, 1.0, delta[1], Cs, id2, 6, 1, 6, 1);
  mm_nt(cmat, 1.0, delta[2], id2, iCs, 6, 1, 6, 1);
  mm_nt(cmat, 1.0, delta[2], iCs, id2, 6, 1, 6, 1);
  mm_nt(cmat, 1.0, delta[3], Cs, Cs, 6, 1, 6, 1);
  mm_nt(cmat, 1.0, delta[4], Cs, iCs, 6, 1, 6, 1);
  mm_nt(cmat, 1.0, delta[4], iCs, Cs, 6, 1, 6, 1);
  mm_nt(cmat, 1.0, delta[5], iCs, iCs, 6, 1, 6, 1);
  /* add_holzapfel_product(cmat, iC_stress, delta[6]) */
  {
    const double* v = iCs;
    const double sc6 = delta[6];
#define CM(i, j) cmat[(i) + 6 * (j)]
    CM(0, 0) += sc6 * v[0] * v[0]; CM(0, 1) += sc6 * v[3] * v[3]; CM(0, 2) += sc6 * v[5] * v[5];
    CM(0, 3) += sc6 * v[0] * v[3]; CM(0, 4) += sc6 * v[3] * v[5]; CM(0, 5) += sc6 * v[0] * v[5];
    CM(1, 0) += sc6 * v[3] * v[3]; CM(1, 1) += sc6 * v[1] * v[1]; CM(1, 2) += sc6 * v[4] * v[4];
    CM(1, 3) += sc6 * v[3] * v[1]; CM(1, 4) += sc6 * v[1] * v[4]; CM(1, 5) += sc6 * v[3] * v[4];
    CM(2, 0) += sc6 * v[5] * v[5]; CM(2, 1) += sc6 * v[4] * v[4]; CM(2, 2) += sc6 * v[2] * v[2];
    CM(2, 3) += sc6 * v[5] * v[4]; CM(2, 4) += sc6 * v[4] * v[2]; CM(2, 5) += sc6 * v[5] * v[2];
    CM(3, 0) += sc6 * v[0] * v[3]; CM(3, 1) += sc6 * v[3] * v[1]; CM(3, 2) += sc6 * v[5] * v[4];
    CM(3, 3) += sc6 * 0.5 * (v[0] * v[1] + v[3] * v[3]);
    CM(3, 4) += sc6 * 0.5 * (v[3] * v[4] + v[5] * v[1]);
    CM(3, 5) += sc6 * 0.5 * (v[0] * v[4] + v[5] * v[3]);
    CM(4, 0) += sc6 * v[3] * v[5]; CM(4, 1) += sc6 * v[1] * v[4]; CM(4, 2) += sc6 * v[4] * v[2];
    CM(4, 3) += sc6 * 0.5 * (v[3] * v[4] + v[5] * v[1]);
    CM(4, 4) += sc6 * 0.5 * (v[1] * v[2] + v[4] * v[4]);
    CM(4, 5) += sc6 * 0.5 * (v[3] * v[2] + v[4] * v[5]);
    CM(5, 0) += sc6 * v[0] * v[5]; CM(5, 1) += sc6 * v[3] * v[4]; CM(5, 2) += sc6 * v[5] * v[2];
    CM(5, 3) += sc6 * 0.5 * (v[0] * v[4] + v[5] * v[3]);
    CM(5, 4) += sc6 * 0.5 * (v[3] * v[2] + v[4] * v[5]);
    CM(5, 5) += sc6 * 0.5 * (v[0] * v[2] + v[5] * v[5]);
    /* cmat.update(delta[7], id4sharp<stress, stress>, 1.0): diag 1 (normal), 0.5 (shear) */
    for (int i = 0; i < 6; ++i) CM(i, i) = 1.0 * CM(i, i) + delta[7] * (i < 3 ? 1.0 : 0.5);
#undef CM
  }
}

/* ---------------------------------------------------------------------------------------
 * Element evaluation: SolidEleCalc::evaluate_nonlinear_force_stiffness_mass
 * (4C_solid_3D_ele_calc.cpp:110-240) with the helpers of 4C_solid_3D_ele_calc_lib.hpp.
 * ------------------------------------------------------------------------------------- */
typedef struct
{
  double det;
  double J[9];    /* jacobian_ (3x3) */
  double invJ[9]; /* inverse_jacobian_ */
  double N_XYZ[3 * MAXN];
} jac_map;

/* evaluate_jacobian_mapping (calc_lib.hpp:435-448) */
static int jacobian_mapping(int n, const double* dN, const double* X, jac_map* jm)
{
  mm_nt(jm->J, 0.0, 1.0, dN, X, 3, n, 3, 0); /* J = deriv * X^T */
  memcpy(jm->invJ, jm->J, sizeof(jm->J));
  jm->det = invert3x3(jm->invJ);
  if (jm->det == 0.0) return ORC_ERR_SINGULAR;
  mm_nn(jm->N_XYZ, 0.0, 1.0, jm->invJ, dN, 3, 3, n, 0); /* N_XYZ = invJ * deriv */
  return ORC_OK;
}

int orc_solid_evaluate(int celltype, int kinem, double E, double nu, const double* X,
    const double* u, double* Ke, double* fe)
{
  return orc_solid_evaluate_mat(celltype, kinem, ORC_MAT_STVK, E, nu, X, u, Ke, fe);
}

int orc_solid_evaluate_mat(int celltype, int kinem, int material, double E, double nu,
    const double* X, const double* u, double* Ke, double* fe)
{
  if (material != ORC_MAT_STVK && material != ORC_MAT_NEOHOOKE) return ORC_ERR_ARG;
  if (celltype != ORC_HEX8 && celltype != ORC_HEX27) return ORC_ERR_ARG;
  const int n = orc_num_nodes(celltype);
  const int ndof = 3 * n;
  const int ngp = orc_num_gp(celltype);

  /* evaluate_element_nodes (calc_lib.hpp:152-173): reference, displacement, current (3 x n) */
  double xref[3 * MAXN], disp[3 * MAXN], xcur[3 * MAXN];
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d)
    {
      xref[d + 3 * i] = X[3 * i + d];
      disp[d + 3 * i] = u[3 * i + d];
      xcur[d + 3 * i] = xref[d + 3 * i] + 1.0 * disp[d + 3 * i];
    }

  /* ensure_positive_jacobian_determinant_at_element_nodes (calc_lib.hpp:475-496) */
  {
    double xin[3 * MAXN], dN[3 * MAXN];
    orc_node_param_coords(celltype, xin);
    for (int i = 0; i < n; ++i)
    {
      jac_map jm;
      orc_shape_deriv1(celltype, &xin[3 * i], dN);
      int err = jacobian_mapping(n, dN, xref, &jm);
      if (err) return ORC_ERR_SINGULAR;
      if (!(jm.det > 0)) return ORC_ERR_NODAL_DETJ;
    }
  }

  double cmat[36];
  orc_stvk_cmat(E, nu, cmat);

  double gxi[3 * 27], gw[27];
  orc_gauss_points(celltype, gxi, gw);

  /* for_each_gauss_point (calc_lib.hpp:974-993) */
  for (int gp = 0; gp < ngp; ++gp)
  {
    double dN[3 * MAXN];
    orc_shape_deriv1(celltype, &gxi[3 * gp], dN);
    jac_map jm;
    if (jacobian_mapping(n, dN, xref, &jm)) return ORC_ERR_SINGULAR;
    const double fac = jm.det * gw[gp];
    const double* NX = jm.N_XYZ;

    double Bop[6 * MAXDOF];
    double gl[6];
    double F[9];
    memset(Bop, 0, sizeof(double) * 6 * ndof);
#define B(r, c) Bop[(r) + 6 * (c)]
#define NXYZ(d, i) NX[(d) + 3 * (i)]
    if (kinem == ORC_LINEAR)
    {
      /* evaluate_linear_strain_gradient (calc_lib.hpp:770-799) */
      for (int i = 0; i < n; ++i)
      {
        for (int d = 0; d < 3; ++d) B(d, 3 * i + d) = NXYZ(d, i);
        B(3, 3 * i + 0) = NXYZ(1, i);
        B(3, 3 * i + 1) = NXYZ(0, i);
        B(3, 3 * i + 2) = 0;
        B(4, 3 * i + 0) = 0;
        B(4, 3 * i + 1) = NXYZ(2, i);
        B(4, 3 * i + 2) = NXYZ(1, i);
        B(5, 3 * i + 0) = NXYZ(2, i);
        B(5, 3 * i + 1) = 0;
        B(5, 3 * i + 2) = NXYZ(0, i);
      }
      /* evaluate_linear_gl_strain (:682-695): gl = B * u_vec */
      mm_nn(gl, 0.0, 1.0, Bop, disp, 6, ndof, 1, 0);
    }
    else
    {
      /* evaluate_deformation_gradient (:579-605) */
      if (celltype == ORC_HEX8)
        mm_nt(F, 0.0, 1.0, xcur, NX, 3, n, 3, 0); /* F = x * N_XYZ^T */
      else
      {
        for (int k = 0; k < 9; ++k) F[k] = 0.0;
        F[0] = F[4] = F[8] = 1.0;
        mm_nt(F, 1.0, 1.0, disp, NX, 3, n, 3, 1); /* F = I + u * N_XYZ^T */
      }
      /* evaluate_spatial_material_mapping (:549-568): inverse of F (throws if singular) */
      {
        double Finv[9];
        memcpy(Finv, F, sizeof(F));
        if (invert3x3(Finv) == 0.0) return ORC_ERR_SINGULAR;
      }
      /* evaluate_cauchy_green (:664-676) and evaluate_green_lagrange_strain (:639-652) */
      double Cg[9];
      mm_tn(Cg, 0.0, 1.0, F, F, 3, 3, 3, 0);
      gl[0] = 0.5 * (Cg[0] - 1.0);
      gl[1] = 0.5 * (Cg[4] - 1.0);
      gl[2] = 0.5 * (Cg[8] - 1.0);
      gl[3] = Cg[0 + 3 * 1];
      gl[4] = Cg[1 + 3 * 2];
      gl[5] = Cg[2 + 3 * 0];
      /* evaluate_strain_gradient (:708-760) */
#define FF(i, j) F[(i) + 3 * (j)]
      for (int i = 0; i < n; ++i)
      {
        for (int d = 0; d < 3; ++d)
          for (int e = 0; e < 3; ++e) B(d, 3 * i + e) = FF(e, d) * NXYZ(d, i);
        B(3, 3 * i + 0) = FF(0, 0) * NXYZ(1, i) + FF(0, 1) * NXYZ(0, i);
        B(3, 3 * i + 1) = FF(1, 0) * NXYZ(1, i) + FF(1, 1) * NXYZ(0, i);
        B(3, 3 * i + 2) = FF(2, 0) * NXYZ(1, i) + FF(2, 1) * NXYZ(0, i);
        B(4, 3 * i + 0) = FF(0, 1) * NXYZ(2, i) + FF(0, 2) * NXYZ(1, i);
        B(4, 3 * i + 1) = FF(1, 1) * NXYZ(2, i) + FF(1, 2) * NXYZ(1, i);
        B(4, 3 * i + 2) = FF(2, 1) * NXYZ(2, i) + FF(2, 2) * NXYZ(1, i);
        B(5, 3 * i + 0) = FF(0, 2) * NXYZ(0, i) + FF(0, 0) * NXYZ(2, i);
        B(5, 3 * i + 1) = FF(1, 2) * NXYZ(0, i) + FF(1, 0) * NXYZ(2, i);
        B(5, 3 * i + 2) = FF(2, 2) * NXYZ(0, i) + FF(2, 0) * NXYZ(2, i);
      }
#undef FF
    }

    /* So3Material::evaluate -> StVK: S = C . E (4C_mat_stvenantkirchhoff.cpp:169-177), or
     * ElastHyper/CoupNeoHooke (cmat and S from the principal invariants of C = 2E + I) */
    double pk2[6];
    if (material == ORC_MAT_NEOHOOKE)
      orc_elasthyper_coupneohooke(E, nu, gl, pk2, cmat);
    else
      mm_nn(pk2, 0.0, 1.0, cmat, gl, 6, 6, 1, 0);

    /* add_internal_force_vector (calc_lib.hpp:851-860): f += fac * B^T S */
    if (fe) mm_tn(fe, 1.0, fac, Bop, pk2, ndof, 6, 1, 1);

    if (Ke)
    {
      /* add_elastic_stiffness_matrix (:872-885): cb = C B; K += fac * B^T cb */
      double cb[6 * MAXDOF];
      mm_nn(cb, 0.0, 1.0, cmat, Bop, 6, 6, ndof, 0);
      mm_tn(Ke, 1.0, fac, Bop, cb, ndof, 6, ndof, 1);

      if (kinem == ORC_TOTLAG)
      {
        /* add_geometric_stiffness_matrix (:898-927) */
        for (int inod = 0; inod < n; ++inod)
        {
          double SmB_L[3];
          SmB_L[0] = pk2[0] * NXYZ(0, inod) + pk2[3] * NXYZ(1, inod) + pk2[5] * NXYZ(2, inod);
          SmB_L[1] = pk2[3] * NXYZ(0, inod) + pk2[1] * NXYZ(1, inod) + pk2[4] * NXYZ(2, inod);
          SmB_L[2] = pk2[5] * NXYZ(0, inod) + pk2[4] * NXYZ(1, inod) + pk2[2] * NXYZ(2, inod);
          for (int jnod = 0; jnod < n; ++jnod)
          {
            double bopstrbop = 0.0;
            for (int idim = 0; idim < 3; ++idim) bopstrbop += NXYZ(idim, jnod) * SmB_L[idim];
            for (int d = 0; d < 3; ++d) Ke[(3 * inod + d) + ndof * (3 * jnod + d)] += fac * bopstrbop;
          }
        }
      }
    }
#undef B
#undef NXYZ
  }
  return ORC_OK;
}

/* ---------------------------------------------------------------------------------------
 * GridGenerator (4C_io_gridgenerator.cpp)
 * ------------------------------------------------------------------------------------- */
void orc_hex_element_nodeids(int celltype, int64_t eleid, const int32_t* interval,
    int64_t nodeOffset, int64_t* nodeids)
{
  /* create_hex_element :329-392 */
  const int64_t ex = 2 * (eleid % interval[0]);
  const int64_t ey = 2 * ((eleid / interval[0]) % interval[1]);
  const int64_t ez = 2 * (eleid / ((int64_t)interval[0] * interval[1]));
  const int64_t nx = 2 * (int64_t)interval[0] + 1;
  const int64_t ny = 2 * (int64_t)interval[1] + 1;
  if (celltype == ORC_HEX27)
  {
    nodeids[20] = nodeOffset + (ez * ny + ey + 1) * nx + ex + 1;
    nodeids[21] = nodeOffset + ((ez + 1) * ny + ey) * nx + ex + 1;
    nodeids[22] = nodeOffset + ((ez + 1) * ny + ey + 1) * nx + ex + 2;
    nodeids[23] = nodeOffset + ((ez + 1) * ny + ey + 2) * nx + ex + 1;
    nodeids[24] = nodeOffset + ((ez + 1) * ny + ey + 1) * nx + ex;
    nodeids[25] = nodeOffset + ((ez + 2) * ny + ey + 1) * nx + ex + 1;
    nodeids[26] = nodeOffset + ((ez + 1) * ny + ey + 1) * nx + ex + 1;
    nodeids[8] = nodeOffset + (ez * ny + ey) * nx + ex + 1;
    nodeids[9] = nodeOffset + (ez * ny + ey + 1) * nx + ex + 2;
    nodeids[10] = nodeOffset + (ez * ny + ey + 2) * nx + ex + 1;
    nodeids[11] = nodeOffset + (ez * ny + ey + 1) * nx + ex;
    nodeids[12] = nodeOffset + ((ez + 1) * ny + ey) * nx + ex;
    nodeids[13] = nodeOffset + ((ez + 1) * ny + ey) * nx + ex + 2;
    nodeids[14] = nodeOffset + ((ez + 1) * ny + ey + 2) * nx + ex + 2;
    nodeids[15] = nodeOffset + ((ez + 1) * ny + ey + 2) * nx + ex;
    nodeids[16] = nodeOffset + ((ez + 2) * ny + ey) * nx + ex + 1;
    nodeids[17] = nodeOffset + ((ez + 2) * ny + ey + 1) * nx + ex + 2;
    nodeids[18] = nodeOffset + ((ez + 2) * ny + ey + 2) * nx + ex + 1;
    nodeids[19] = nodeOffset + ((ez + 2) * ny + ey + 1) * nx + ex;
  }
  nodeids[0] = nodeOffset + (ez * ny + ey) * nx + ex;
  nodeids[1] = nodeOffset + (ez * ny + ey) * nx + ex + 2;
  nodeids[2] = nodeOffset + (ez * ny + ey + 2) * nx + ex + 2;
  nodeids[3] = nodeOffset + (ez * ny + ey + 2) * nx + ex;
  nodeids[4] = nodeOffset + ((ez + 2) * ny + ey) * nx + ex;
  nodeids[5] = nodeOffset + ((ez + 2) * ny + ey) * nx + ex + 2;
  nodeids[6] = nodeOffset + ((ez + 2) * ny + ey + 2) * nx + ex + 2;
  nodeids[7] = nodeOffset + ((ez + 2) * ny + ey + 2) * nx + ex;
}

void orc_lattice_node_coords(int64_t gid, const int32_t* interval, int64_t node_offset,
    const double* lo, const double* hi, const double* rot, double* coords)
{
  /* :254-323 */
  const int64_t nx = 2 * (int64_t)interval[0] + 1;
  const int64_t ny = 2 * (int64_t)interval[1] + 1;
  double coordm[3] = {0.0, 0.0, 0.0};
  if (rot[0] != 0.0 || rot[1] != 0.0 || rot[2] != 0.0)
  {
    coordm[0] = (hi[0] + lo[0]) / 2.;
    coordm[1] = (hi[1] + lo[1]) / 2.;
    coordm[2] = (hi[2] + lo[2]) / 2.;
  }
  const int64_t posid = gid - node_offset;
  const int64_t i = posid % nx;
  const int64_t j = (posid / nx) % ny;
  const int64_t k = posid / (nx * ny);
  coords[0] = (double)i / (2 * interval[0]) * (hi[0] - lo[0]) + lo[0];
  coords[1] = (double)j / (2 * interval[1]) * (hi[1] - lo[1]) + lo[1];
  coords[2] = (double)k / (2 * interval[2]) * (hi[2] - lo[2]) + lo[2];
  for (int rotaxis = 0; rotaxis < 3; ++rotaxis)
  {
    if (rot[rotaxis] != 0.0)
    {
      double dx[3];
      dx[0] = coords[0] - coordm[0];
      dx[1] = coords[1] - coordm[1];
      dx[2] = coords[2] - coordm[2];
      const double calpha = cos(rot[rotaxis] * M_PI / 180);
      const double salpha = sin(rot[rotaxis] * M_PI / 180);
      coords[0] = coordm[0];
      coords[1] = coordm[1];
      coords[2] = coordm[2];
      coords[(rotaxis + 1) % 3] += calpha * dx[(rotaxis + 1) % 3] + salpha * dx[(rotaxis + 2) % 3];
      coords[(rotaxis + 2) % 3] += calpha * dx[(rotaxis + 2) % 3] - salpha * dx[(rotaxis + 1) % 3];
      coords[rotaxis] += dx[rotaxis];
    }
  }
}

int orc_box_section(const int32_t* interval, int nproc, int rank, int32_t* range)
{
  /* element row map "fancy final box map", :87-153 */
  int factors[64];
  int nf = 0;
  int np = nproc;
  for (int fac = 2; fac < np + 1;)
  {
    if (np % fac == 0)
    {
      factors[nf++] = fac;
      np /= fac;
    }
    else
      fac++;
  }
  if (np != 1) return -1;
  unsigned sub[3] = {1, 1, 1};
  const double dint[3] = {(double)interval[0], (double)interval[1], (double)interval[2]};
  for (int f = nf - 1; f >= 0; --f)
  {
    const double ratios[3] = {dint[0] / sub[0], dint[1] / sub[1], dint[2] / sub[2]};
    if (ratios[0] >= ratios[1] && ratios[0] >= ratios[2])
      sub[0] *= factors[f];
    else if (ratios[1] >= ratios[0] && ratios[1] >= ratios[2])
      sub[1] *= factors[f];
    else if (ratios[2] >= ratios[0] && ratios[2] >= ratios[1])
      sub[2] *= factors[f];
  }
  const unsigned sec[3] = {rank % sub[0], (rank / sub[0]) % sub[1], rank / (sub[0] * sub[1])};
  for (int d = 0; d < 3; ++d)
  {
    for (int b = 0; b < 2; ++b)
    {
      const unsigned idx = sec[d] + b;
      long v = lround(idx * dint[d] / sub[d]);
      if (v < 0) v = 0;
      if (v > interval[d]) v = interval[d];
      range[2 * d + b] = (int32_t)v;
    }
  }
  return 0;
}

/* ---------------------------------------------------------------------------------------
 * Assembly
 * ------------------------------------------------------------------------------------- */
static int* lower_bound_int(int* first, int* last, int value)
{
  int64_t count = last - first;
  while (count > 0)
  {
    int64_t step = count / 2;
    int* it = first + step;
    if (*it < value)
    {
      first = it + 1;
      count -= step + 1;
    }
    else
      count = step;
  }
  return first;
}

int orc_sparse_assemble(orc_csr* A, int myrank, int numnode, const int* lmstride, int lcoldim,
    const double* Aele, const int* lmrow, const int* lmrowowner, const int* lmcol)
{
  return orc_sparse_assemble_rect(A, myrank, numnode, lmstride, lcoldim, lcoldim, Aele, lmrow,
      lmrowowner, lmcol);
}

int orc_sparse_assemble_rect(orc_csr* A, int myrank, int numnode, const int* lmstride, int lrowdim,
    int lcoldim, const double* Aele, const int* lmrow, const int* lmrowowner, const int* lmcol)
{
  /* SparseMatrix::assemble, Filled() branch (4C_linalg_sparsematrix.cpp:444-576): lrowdim rows x
   * lcoldim columns (rectangular for TSI's coupling blocks, AssembleStrategy(0, 1, k_st));
   * numnode / lmstride describe the column nodes.  Aele is column-major with leading dimension
   * lrowdim. */
  int localcol[MAXDOF];
  for (int lcol = 0; lcol < lcoldim; ++lcol)
  {
    const int cgid = lmcol[lcol];
    localcol[lcol] = (cgid >= 0 && cgid <= A->max_gid) ? A->col_lid_of_gid[cgid] : -1;
    if (localcol[lcol] < 0) return -1;
  }
  for (int lrow = 0; lrow < lrowdim; ++lrow)
  {
    if (lmrowowner[lrow] != myrank) continue;
    const int rgid = lmrow[lrow];
    const int rlid = A->row_lid_of_gid[rgid];
    if (rlid < 0) return -2;
    /* ExtractMyRowView */
    const int64_t start = A->rowptr[rlid];
    const int length = (int)(A->rowptr[rlid + 1] - start);
    double* valview = A->vals + start;
    int* indices = (int*)(A->col_lid + start);
    int dofcount = 0;
    int pos = 0;
    for (int node = 0; node < numnode; ++node)
    {
      if (pos >= length || indices[pos] != localcol[dofcount])
      {
        int* loc = lower_bound_int(indices, indices + length, localcol[dofcount]);
        if (loc == indices + length || *loc != localcol[dofcount]) return -3;
        pos = (int)(loc - indices);
      }
      const int stride = lmstride[node];
      int reachedlength = 0;
      int continuous = 1;
      if (stride + pos > length)
        continuous = 0;
      else
      {
        for (int j = 1; j < stride; ++j)
          if (indices[pos + j] != localcol[dofcount + j])
          {
            continuous = 0;
            break;
          }
      }
      if (continuous)
      {
        for (int j = 0; j < stride; ++j)
        {
          valview[pos++] += Aele[lrow + lrowdim * dofcount];
          dofcount++;
          if (dofcount == lcoldim)
          {
            reachedlength = 1;
            break;
          }
        }
      }
      else
      {
        /* SumIntoMyValues fallback: search each column individually */
        for (int j = 0; j < stride; ++j)
        {
          int* loc = lower_bound_int(indices, indices + length, localcol[dofcount]);
          if (loc == indices + length || *loc != localcol[dofcount]) return -3;
          valview[loc - indices] += Aele[lrow + lrowdim * dofcount];
          dofcount++;
          if (dofcount == lcoldim)
          {
            reachedlength = 1;
            break;
          }
        }
      }
      if (reachedlength) break;
    }
  }
  return 0;
}

int orc_vector_assemble(double* V, const int32_t* lid_of_gid, int64_t max_gid, int ldim,
    const double* Vele, const int* lm, const int* lmowner, int myrank)
{
  /* 4C_linalg_utils_sparse_algebra_assemble.cpp:72-92 */
  for (int lrow = 0; lrow < ldim; ++lrow)
  {
    if (lmowner[lrow] != myrank) continue;
    const int rgid = lm[lrow];
    if (rgid < 0 || rgid > max_gid || lid_of_gid[rgid] < 0) return -1;
    V[lid_of_gid[rgid]] += Vele[lrow];
  }
  return 0;
}

int orc_discretization_evaluate(int celltype, int kinem, double E, double nu, int64_t n_ele,
    const int64_t* ele_nodes, int64_t n_nodes, const double* node_x, const int64_t* node_gid,
    const int32_t* node_owner, int64_t min_node_gid, int nworkers, const double* u, orc_csr* K,
    double* fint, int64_t* bad_ele)
{
  return orc_discretization_evaluate_mat(celltype, kinem, ORC_MAT_STVK, E, nu, n_ele, ele_nodes,
      n_nodes, node_x, node_gid, node_owner, min_node_gid, nworkers, u, K, fint, bad_ele);
}

int orc_discretization_evaluate_mat(int celltype, int kinem, int material, double E, double nu,
    int64_t n_ele, const int64_t* ele_nodes, int64_t n_nodes, const double* node_x,
    const int64_t* node_gid, const int32_t* node_owner, int64_t min_node_gid, int nworkers,
    const double* u, orc_csr* K, double* fint, int64_t* bad_ele)
{
  const int n = orc_num_nodes(celltype);
  const int ndof = 3 * n;
  int result = 0;
  if (!K) return ORC_ERR_ARG;
  int64_t first_bad = -1;
  (void)n_nodes;
  if (nworkers < 1) nworkers = 1;

#pragma omp parallel for num_threads(nworkers) schedule(static, 1)
  for (int w = 0; w < nworkers; ++w)
  {
    /* per-"rank" element storage, AssembleStrategy::clear_element_storage */
    double* Ke = (double*)malloc(sizeof(double) * ndof * ndof);
    double fe[MAXDOF], X[3 * MAXN], ue[3 * MAXN];
    int lm[MAXDOF], lmowner[MAXDOF], lmstride[MAXN];
    /* Discretization::evaluate loops over the rank's column elements
     * (4C_fem_discretization_evaluate.cpp:83-102) */
    for (int64_t e = 0; e < n_ele; ++e)
    {
      const int64_t* en = ele_nodes + (int64_t)n * e;
      int touches = 0;
      for (int a = 0; a < n; ++a)
        if (node_owner[en[a]] == w)
        {
          touches = 1;
          break;
        }
      if (!touches) continue; /* not a column element of rank w */
      /* location_vector (4C_fem_general_element.cpp:474-542) */
      for (int a = 0; a < n; ++a)
      {
        const int64_t nd = en[a];
        const int dof0 = (int)(3 * (node_gid[nd] - min_node_gid));
        for (int d = 0; d < 3; ++d)
        {
          lm[3 * a + d] = dof0 + d;
          lmowner[3 * a + d] = node_owner[nd];
          X[3 * a + d] = node_x[3 * nd + d];
          /* extract_values_as_array: u[col LID(gid)] */
          ue[3 * a + d] = u[K->col_lid_of_gid[dof0 + d]];
        }
        lmstride[a] = 3;
      }
      const int want_k = K->vals != NULL;
      if (want_k) memset(Ke, 0, sizeof(double) * ndof * ndof);
      memset(fe, 0, sizeof(fe));
      int err = orc_solid_evaluate_mat(celltype, kinem, material, E, nu, X, ue, want_k ? Ke : NULL, fe);
      if (err)
      {
#pragma omp critical
        {
          if (!result || e < first_bad)
          {
            result = err;
            first_bad = e;
          }
        }
        break;
      }
      if (want_k)
      {
        if (orc_sparse_assemble(K, w, n, lmstride, ndof, Ke, lm, lmowner, lm))
        {
#pragma omp critical
          result = ORC_ERR_ARG;
          break;
        }
      }
      if (fint)
        orc_vector_assemble(fint, K->row_lid_of_gid, K->max_gid, ndof, fe, lm, lmowner, w);
    }
    free(Ke);
  }
  if (bad_ele) *bad_ele = first_bad;
  return result;
}

/* =======================================================================================
 * Thermo-structure interaction, geometrically linear (BASELINE config 5)
 * ===================================================================================== */

double orc_thermo_stvk_st_modulus(double E, double nu, double alpha)
{
  /* ThermoStVenantKirchhoff::st_modulus (4C_mat_thermostvenantkirchhoff.cpp:331-369) */
  const double c1 = E / (1.0 + nu);
  const double b1 = c1 * nu / (1.0 - 2.0 * nu);
  const double mu = 0.5 * c1;
  const double lambda = b1;
  return (-1.0) * (2.0 * mu + 3.0 * lambda) * alpha;
}

/* linear B operator (evaluate_linear_strain_gradient, calc_lib.hpp:770-799; identical to the
 * thermo element's calculate_boplin, 4C_thermo_ele_impl.cpp:2829-2869) */
static void boplin(int n, const double* NX, double* Bop)
{
  memset(Bop, 0, sizeof(double) * 6 * 3 * n);
#define B(r, c) Bop[(r) + 6 * (c)]
#define NXYZ(d, i) NX[(d) + 3 * (i)]
  for (int i = 0; i < n; ++i)
  {
    for (int d = 0; d < 3; ++d) B(d, 3 * i + d) = NXYZ(d, i);
    B(3, 3 * i + 0) = NXYZ(1, i);
    B(3, 3 * i + 1) = NXYZ(0, i);
    B(4, 3 * i + 1) = NXYZ(2, i);
    B(4, 3 * i + 2) = NXYZ(1, i);
    B(5, 3 * i + 0) = NXYZ(2, i);
    B(5, 3 * i + 2) = NXYZ(0, i);
  }
#undef B
#undef NXYZ
}

/* Core::LinAlg::Matrix::dot (shape functions . nodal values), index order */
static double dotn(const double* a, const double* b, int n)
{
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

int orc_tsi_solid_evaluate(int celltype, double E, double nu, double alpha, double T0,
    const double* X, const double* u, const double* T, double* Ke, double* fe, double* Kst)
{
  if (celltype != ORC_HEX8 && celltype != ORC_HEX27) return ORC_ERR_ARG;
  const int n = orc_num_nodes(celltype);
  const int ndof = 3 * n;
  const int ngp = orc_num_gp(celltype);
  double xref[3 * MAXN], disp[3 * MAXN];
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d)
    {
      xref[d + 3 * i] = X[3 * i + d];
      disp[d + 3 * i] = u[3 * i + d];
    }
  /* struct_calc_stifftemp checks the nodal Jacobians (4C_solid_scatra_3D_ele_calc.cpp:441);
   * struct_calc_nlnstiff of the solid-scatra element does not (:272-403). */
  if (Kst)
  {
    double xin[3 * MAXN], dN[3 * MAXN];
    orc_node_param_coords(celltype, xin);
    for (int i = 0; i < n; ++i)
    {
      jac_map jm;
      orc_shape_deriv1(celltype, &xin[3 * i], dN);
      if (jacobian_mapping(n, dN, xref, &jm)) return ORC_ERR_SINGULAR;
      if (!(jm.det > 0)) return ORC_ERR_NODAL_DETJ;
    }
  }
  double cmat[36];
  orc_stvk_cmat(E, nu, cmat); /* ThermoStVenantKirchhoff::setup_cmat (:308-326), constant E */
  const double m = orc_thermo_stvk_st_modulus(E, nu, alpha);
  double gxi[3 * 27], gw[27];
  orc_gauss_points(celltype, gxi, gw);
  for (int gp = 0; gp < ngp; ++gp)
  {
    double dN[3 * MAXN], N[MAXN];
    orc_shape(celltype, &gxi[3 * gp], N);
    orc_shape_deriv1(celltype, &gxi[3 * gp], dN);
    jac_map jm;
    if (jacobian_mapping(n, dN, xref, &jm)) return ORC_ERR_SINGULAR;
    const double fac = jm.det * gw[gp];
    double Bop[6 * MAXDOF];
    boplin(n, jm.N_XYZ, Bop);
    /* prepare_scalar_in_parameter_list("temperature"): T_gp = N . T
     * (4C_solid_scatra_3D_ele_calc.cpp:172-182) */
    const double Tgp = dotn(N, T, n);
    if (fe || Ke)
    {
      double gl[6], pk2[6];
      mm_nn(gl, 0.0, 1.0, Bop, disp, 6, ndof, 1, 0); /* evaluate_linear_gl_strain */
      /* ThermoStVenantKirchhoff::evaluate (:141-174): S = C E, S_ii += m (T - T_ref) */
      mm_nn(pk2, 0.0, 1.0, cmat, gl, 6, 6, 1, 0);
      for (int i = 0; i < 3; ++i) pk2[i] += m * (Tgp - T0);
      if (fe) mm_tn(fe, 1.0, fac, Bop, pk2, ndof, 6, 1, 1);
      if (Ke)
      {
        double cb[6 * MAXDOF];
        mm_nn(cb, 0.0, 1.0, cmat, Bop, 6, 6, ndof, 0);
        mm_tn(Ke, 1.0, fac, Bop, cb, ndof, 6, ndof, 1);
      }
    }
    if (Kst)
    {
      /* evaluate_d_stress_d_scalar (4C_mat_thermostvenantkirchhoff.cpp:250-295) with constant E:
       * dS/dT = C_T E + (T - T0) ctemp_T + ctemp = (m, m, m, 0, 0, 0) */
      double dSdT[6] = {m, m, m, 0.0, 0.0, 0.0};
      /* k_dS = B^T dS/dT fac N^T (4C_solid_scatra_3D_ele_calc.cpp:472-487) */
      double BdSdc[MAXDOF];
      mm_tn(BdSdc, 0.0, fac, Bop, dSdT, ndof, 6, 1, 0);
      for (int r = 0; r < ndof; ++r)
        for (int c = 0; c < n; ++c) Kst[r + ndof * c] += BdSdc[r] * N[c];
    }
  }
  return ORC_OK;
}

int orc_tsi_thermo_evaluate(int celltype, double conduct, double m, const double* X,
    const double* T, const double* v, double timefac, double timefac_d, double* Ktt,
    double* fT, double* Kts)
{
  if (celltype != ORC_HEX8 && celltype != ORC_HEX27) return ORC_ERR_ARG;
  const int n = orc_num_nodes(celltype);
  const int ndof = 3 * n;
  const int ngp = orc_num_gp(celltype); /* DisTypeToOptGaussRule: hex_8point / hex_27point */
  double xyze[3 * MAXN], evel[3 * MAXN];
  for (int i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d)
    {
      xyze[d + 3 * i] = X[3 * i + d];
      evel[d + 3 * i] = v[3 * i + d];
    }
  double gxi[3 * 27], gw[27];
  orc_gauss_points(celltype, gxi, gw);
  double ctemp[6] = {m, m, m, 0.0, 0.0, 0.0}; /* setup_cthermo / fill_cthermo (:376-402) */
  for (int gp = 0; gp < ngp; ++gp)
  {
    /* eval_shape_func_and_derivs_at_int_point (4C_thermo_ele_impl.cpp:2613-2671) */
    double N[MAXN], deriv[3 * MAXN], xjm[9], derxy[3 * MAXN];
    orc_shape(celltype, &gxi[3 * gp], N);
    orc_shape_deriv1(celltype, &gxi[3 * gp], deriv);
    mm_nt(xjm, 0.0, 1.0, deriv, xyze, 3, n, 3, 0);
    const double det = invert3x3(xjm);
    if (det < 1e-16) return det == 0.0 ? ORC_ERR_SINGULAR : ORC_ERR_NODAL_DETJ;
    const double fac = gw[gp] * det;
    mm_nn(derxy, 0.0, 1.0, xjm, deriv, 3, 3, n, 0);
    const double NT = dotn(N, T, n); /* NT.multiply_tn(funct_, etempn_) */

    /* linear_thermo_contribution (:802-891); Fourier: cmat = k I, heatflux = cmat gradT
     * (4C_mat_fourier.cpp:147-192); the dercmat term vanishes for a constant conductivity */
    if (fT || Ktt)
    {
      double gradtemp[3], heatflux[3], cm[9] = {conduct, 0, 0, 0, conduct, 0, 0, 0, conduct};
      mm_nn(gradtemp, 0.0, 1.0, derxy, T, 3, n, 1, 0);
      mm_nn(heatflux, 0.0, 1.0, cm, gradtemp, 3, 3, 1, 0);
      if (fT) mm_tn(fT, 1.0, fac, derxy, heatflux, n, 3, 1, 1);
      if (Ktt)
      {
        double aop[3 * MAXN];
        mm_nn(aop, 0.0, 1.0, cm, derxy, 3, 3, n, 0);
        mm_tn(Ktt, 1.0, fac, derxy, aop, n, 3, n, 1);
      }
      /* linear_disp_contribution (:899-1043): thermoelastic term with e' = B_L v */
      double Bop[6 * MAXDOF], strainvel[6], Nctemp[6 * MAXN], ncBv[MAXN];
      boplin(n, derxy, Bop);
      mm_nn(strainvel, 0.0, 1.0, Bop, evel, 6, ndof, 1, 0);
      mm_nt(Nctemp, 0.0, 1.0, N, ctemp, n, 1, 6, 0);
      mm_nn(ncBv, 0.0, 1.0, Nctemp, strainvel, n, 6, 1, 0);
      if (fT) mm_nn(fT, 1.0, -fac, ncBv, &NT, n, 1, 1, 1);
      if (Ktt) mm_nt(Ktt, 1.0, -fac, ncBv, N, n, 1, n, 1);
    }
    /* linear_coupled_tang (:1046-1194): k_Td += -timefac fac timefac_d (N N.T ctemp^T) B_L */
    if (Kts)
    {
      double Bop[6 * MAXDOF], NNT[MAXN], NNTC[6 * MAXN];
      boplin(n, derxy, Bop);
      mm_nn(NNT, 0.0, 1.0, N, &NT, n, 1, 1, 0);
      mm_nt(NNTC, 0.0, 1.0, NNT, ctemp, n, 1, 6, 0);
      mm_nn(Kts, 1.0, -timefac * fac * timefac_d, NNTC, Bop, n, 6, ndof, 1);
    }
  }
  return ORC_OK;
}

/* TSI::Monolithic's four element evaluates per element and their assembly (owned rows, the
 * reference's MPI semantics with `nworkers` ranks as threads, as orc_discretization_evaluate):
 * struct_calc_nlnstiff with the temperature state -> K_ss, f_s; struct_calc_stifftemp -> K_st
 * (AssembleStrategy(0, 1, k_st), 4C_tsi_monolithic.cpp:1694-1767); calc_thermo_fintcond -> K_tt,
 * f_t; calc_thermo_coupltang -> K_ts (:1773-1869).  Structural DOF gid 3 (node gid - min) + d,
 * thermo DOF gid node gid - min (one DOF per node; only the maps of the four CSRs use them). */
int orc_tsi_discretization_evaluate(int celltype, double E, double nu, double alpha, double T0,
    double conduct, double timefac, double timefac_d, int64_t n_ele, const int64_t* ele_nodes,
    const double* node_x, const int64_t* node_gid, const int32_t* node_owner, int64_t min_node_gid,
    int nworkers, const double* u, const double* v, const double* T, orc_csr* Kss, orc_csr* Kst,
    orc_csr* Kts, orc_csr* Ktt, double* fs, double* ft, int64_t* bad_ele)
{
  const int n = orc_num_nodes(celltype);
  const int ndof = 3 * n;
  const double m = orc_thermo_stvk_st_modulus(E, nu, alpha);
  int result = 0;
  int64_t first_bad = -1;
  if (nworkers < 1) nworkers = 1;
#pragma omp parallel for num_threads(nworkers) schedule(static, 1)
  for (int w = 0; w < nworkers; ++w)
  {
    double* Ke = (double*)malloc(sizeof(double) * ndof * ndof);
    double* Kst_e = (double*)malloc(sizeof(double) * ndof * n);
    double* Kts_e = (double*)malloc(sizeof(double) * ndof * n);
    double* Ktt_e = (double*)malloc(sizeof(double) * n * n);
    double fe[MAXDOF], fte[MAXN], X[3 * MAXN], ue[3 * MAXN], ve[3 * MAXN], Te[MAXN];
    int lm[MAXDOF], lmowner[MAXDOF], lmstride[MAXN], lmt[MAXN], lmtowner[MAXN], lmtstride[MAXN];
    for (int64_t e = 0; e < n_ele; ++e)
    {
      const int64_t* en = ele_nodes + (int64_t)n * e;
      int touches = 0;
      for (int a = 0; a < n; ++a)
        if (node_owner[en[a]] == w)
        {
          touches = 1;
          break;
        }
      if (!touches) continue;
      for (int a = 0; a < n; ++a)
      {
        const int64_t nd = en[a];
        const int g = (int)(node_gid[nd] - min_node_gid);
        for (int d = 0; d < 3; ++d)
        {
          lm[3 * a + d] = 3 * g + d;
          lmowner[3 * a + d] = node_owner[nd];
          X[3 * a + d] = node_x[3 * nd + d];
          ue[3 * a + d] = u[Kss->col_lid_of_gid[3 * g + d]];
          ve[3 * a + d] = v[Kss->col_lid_of_gid[3 * g + d]];
        }
        lmt[a] = g;
        lmtowner[a] = node_owner[nd];
        Te[a] = T[Ktt->col_lid_of_gid[g]];
        lmstride[a] = 3;
        lmtstride[a] = 1;
      }
      memset(Ke, 0, sizeof(double) * ndof * ndof);
      memset(Kst_e, 0, sizeof(double) * ndof * n);
      memset(Kts_e, 0, sizeof(double) * ndof * n);
      memset(Ktt_e, 0, sizeof(double) * n * n);
      memset(fe, 0, sizeof(fe));
      memset(fte, 0, sizeof(fte));
      int err = orc_tsi_solid_evaluate(celltype, E, nu, alpha, T0, X, ue, Te, Ke, fe, Kst_e);
      if (!err) err = orc_tsi_thermo_evaluate(celltype, conduct, m, X, Te, ve, timefac, timefac_d,
                    Ktt_e, fte, Kts_e);
      if (err)
      {
#pragma omp critical
        {
          if (!result || e < first_bad)
          {
            result = err;
            first_bad = e;
          }
        }
        break;
      }
      int rc = orc_sparse_assemble_rect(Kss, w, n, lmstride, ndof, ndof, Ke, lm, lmowner, lm);
      if (!rc) rc = orc_sparse_assemble_rect(Kst, w, n, lmtstride, ndof, n, Kst_e, lm, lmowner, lmt);
      if (!rc) rc = orc_sparse_assemble_rect(Kts, w, n, lmstride, n, ndof, Kts_e, lmt, lmtowner, lm);
      if (!rc) rc = orc_sparse_assemble_rect(Ktt, w, n, lmtstride, n, n, Ktt_e, lmt, lmtowner, lmt);
      if (!rc) rc = orc_vector_assemble(fs, Kss->row_lid_of_gid, Kss->max_gid, ndof, fe, lm, lmowner, w);
      if (!rc) rc = orc_vector_assemble(ft, Ktt->row_lid_of_gid, Ktt->max_gid, n, fte, lmt, lmtowner, w);
      if (rc)
      {
#pragma omp critical
        result = ORC_ERR_ARG;
        break;
      }
    }
    free(Ke);
    free(Kst_e);
    free(Kts_e);
    free(Ktt_e);
  }
  if (bad_ele) *bad_ele = first_bad;
  return result;
}
