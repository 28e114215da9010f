// fcg_neumann.cpp -- external load vectors of the Newton step: surface and
// volume Neumann conditions of SOLID hex8/hex27 elements, assembled into the owned DOF rows.
//
// Live surface loads on the material configuration (Solid surface evaluate_neumann,
// src/solid_3D_ele/4C_solid_3D_ele_surface_evaluate.cpp:262-320): at every point of the
// quad_4point / quad_9point rule (4C_fem_general_utils_integration.cpp, with the reference's
// truncated constants) f_a += N_a w detA val_d funct_d(x_gp, t), detA = sqrt(det(dxdr dxdr^T)),
// quad4 / quad9 shape functions of 4C_fem_general_utils_fem_shapefunctions.hpp:2003-2087,
// 2148-2274.  Volume loads (4C_solid_3D_ele_neumann_evaluator.cpp:45-110): the element's
// stiffness Gauss rule, f_a += N_a w det J val_d funct_d(x_gp, t).
// These loads do not depend on the displacements, so the Newton driver evaluates them once per
// load step on the host (the caller's function manager supplies funct through a callback) and
// keeps the vector in HBM.
#include <cmath>
#include <cstdint>

#include "fcg_shape.hpp"
#include "fourc_gpu.h"

namespace {

void quad_rule(int nfn, double (*xg)[2], double* w)
{
  if (nfn == 4)
  {
    const double a = 0.5773502691896;
    const double p[4][2] = {{-a, -a}, {a, -a}, {a, a}, {-a, a}};
    for (int g = 0; g < 4; ++g)
    {
      xg[g][0] = p[g][0];
      xg[g][1] = p[g][1];
      w[g] = 1.0;
    }
    return;
  }
  const double b = 0.7745966692415, w1 = 0.5555555555556, w2 = 0.8888888888889;
  const double p[9][2] = {{-b, -b}, {b, -b}, {b, b}, {-b, b}, {0.0, -b}, {b, 0.0}, {0.0, b},
      {-b, 0.0}, {0.0, 0.0}};
  const double ww[9] = {w1 * w1, w1 * w1, w1 * w1, w1 * w1, w2 * w1, w1 * w2, w2 * w1, w1 * w2,
      w2 * w2};
  for (int g = 0; g < 9; ++g)
  {
    xg[g][0] = p[g][0];
    xg[g][1] = p[g][1];
    w[g] = ww[g];
  }
}

void quad_shape(int nfn, double r, double s, double* N, double (*dN)[9])
{
  const double rp = 1.0 + r, rm = 1.0 - r, sp = 1.0 + s, sm = 1.0 - s;
  if (nfn == 4)
  {
    N[0] = 0.25 * rm * sm;
    N[1] = 0.25 * rp * sm;
    N[2] = 0.25 * rp * sp;
    N[3] = 0.25 * rm * sp;
    dN[0][0] = -0.25 * sm; dN[0][1] = 0.25 * sm; dN[0][2] = 0.25 * sp; dN[0][3] = -0.25 * sp;
    dN[1][0] = -0.25 * rm; dN[1][1] = -0.25 * rp; dN[1][2] = 0.25 * rp; dN[1][3] = 0.25 * rm;
    return;
  }
  const double r2 = 1.0 - r * r, s2 = 1.0 - s * s;
  const double rh = 0.5 * r, sh = 0.5 * s, rs = rh * sh;
  const double rhp = r + 0.5, rhm = r - 0.5, shp = s + 0.5, shm = s - 0.5;
  N[0] = rs * rm * sm;
  N[1] = -rs * rp * sm;
  N[2] = rs * rp * sp;
  N[3] = -rs * rm * sp;
  N[4] = -sh * sm * r2;
  N[5] = rh * rp * s2;
  N[6] = sh * sp * r2;
  N[7] = -rh * rm * s2;
  N[8] = r2 * s2;
  const double d0[9] = {-rhm * sh * sm, -rhp * sh * sm, rhp * sh * sp, rhm * sh * sp,
      2.0 * r * sh * sm, rhp * s2, -2.0 * r * sh * sp, rhm * s2, -2.0 * r * s2};
  const double d1[9] = {-shm * rh * rm, shm * rh * rp, shp * rh * rp, -shp * rh * rm, shm * r2,
      -2.0 * s * rh * rp, shp * r2, 2.0 * s * rh * rm, -2.0 * s * r2};
  for (int i = 0; i < 9; ++i)
  {
    dN[0][i] = d0[i];
    dN[1][i] = d1[i];
  }
}

bool args_ok(int celltype, int64_t n, const int32_t* nodes, const double* node_x,
    const int32_t* node_dof_row, const int32_t* onoff, const double* val, double* f)
{
  return (celltype == FCG_HEX8 || celltype == FCG_HEX27) && n >= 0 &&
         (n == 0 || (nodes && node_x && node_dof_row && onoff && val && f));
}

double funct_factor(const int32_t* funct, int d, fcg_funct_fn fn, void* user, const double* x,
    double t)
{
  if (!funct || funct[d] <= 0) return 1.0;
  return fn ? fn(funct[d], x, t, user) : 1.0;
}

}  // namespace

extern "C" {

int fcg_neumann_surface(int celltype, int64_t n_faces, const int32_t* face_nodes,
    const double* node_x, const int32_t* node_dof_row, const int32_t* onoff, const double* val,
    const int32_t* funct, fcg_funct_fn fn, void* user, double time, double* fext_row)
{
  if (!args_ok(celltype, n_faces, face_nodes, node_x, node_dof_row, onoff, val, fext_row))
    return FCG_ERR_ARG;
  if (funct && !fn)
    for (int d = 0; d < 3; ++d)
      if (funct[d] > 0) return FCG_ERR_ARG;
  const int nfn = celltype == FCG_HEX27 ? 9 : 4;
  double xg[9][2], wg[9];
  quad_rule(nfn, xg, wg);
  for (int64_t f = 0; f < n_faces; ++f)
  {
    const int32_t* fnod = face_nodes + f * nfn;
    for (int g = 0; g < nfn; ++g)
    {
      double N[9], dN[2][9];
      quad_shape(nfn, xg[g][0], xg[g][1], N, dN);
      double dx[2][3] = {{0, 0, 0}, {0, 0, 0}}, xgp[3] = {0, 0, 0};
      for (int i = 0; i < nfn; ++i)
        for (int d = 0; d < 3; ++d)
        {
          const double xi = node_x[3 * int64_t(fnod[i]) + d];
          dx[0][d] += dN[0][i] * xi;
          dx[1][d] += dN[1][i] * xi;
          xgp[d] += N[i] * xi;
        }
      double gm[2][2];
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) gm[a][b] = dx[a][0] * dx[b][0] + dx[a][1] * dx[b][1] + dx[a][2] * dx[b][2];
      const double detA = std::sqrt(gm[0][0] * gm[1][1] - gm[0][1] * gm[1][0]);
      for (int d = 0; d < 3; ++d)
      {
        if (!onoff[d]) continue;
        const double fac = wg[g] * detA * val[d] * funct_factor(funct, d, fn, user, xgp, time);
        for (int i = 0; i < nfn; ++i)
        {
          const int32_t r = node_dof_row[fnod[i]];
          if (r >= 0) fext_row[r + d] += N[i] * fac;
        }
      }
    }
  }
  return FCG_OK;
}

int fcg_neumann_volume(int celltype, int64_t n_ele, const int32_t* ele_nodes, const double* node_x,
    const int32_t* node_dof_row, const int32_t* onoff, const double* val, const int32_t* funct,
    fcg_funct_fn fn, void* user, double time, double* fext_row)
{
  if (!args_ok(celltype, n_ele, ele_nodes, node_x, node_dof_row, onoff, val, fext_row))
    return FCG_ERR_ARG;
  if (funct && !fn)
    for (int d = 0; d < 3; ++d)
      if (funct[d] > 0) return FCG_ERR_ARG;
  const int ct = celltype == FCG_HEX27 ? fcg::kHex27 : fcg::kHex8;
  const int npe = fcg::num_nodes(ct);
  const int ngp = ct == fcg::kHex27 ? 27 : 8;
  double xi[81], w[27];
  fcg::gauss_rule(ct, xi, w);
  for (int64_t e = 0; e < n_ele; ++e)
  {
    const int32_t* en = ele_nodes + e * npe;
    for (int g = 0; g < ngp; ++g)
    {
      double N[27], dN[81];
      fcg::shape_values(ct, &xi[3 * g], N);
      fcg::shape_deriv(ct, &xi[3 * g], dN);
      double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, xgp[3] = {0, 0, 0};
      for (int i = 0; i < npe; ++i)
        for (int d = 0; d < 3; ++d)
        {
          const double x = node_x[3 * int64_t(en[i]) + d];
          for (int k = 0; k < 3; ++k) J[k][d] += dN[3 * i + k] * x;
          xgp[d] += N[i] * x;
        }
      const double det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                         J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                         J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
      const double fac = det * w[g];
      for (int d = 0; d < 3; ++d)
      {
        if (!onoff[d]) continue;
        const double v = val[d] * funct_factor(funct, d, fn, user, xgp, time) * fac;
        for (int i = 0; i < npe; ++i)
        {
          const int32_t r = node_dof_row[en[i]];
          if (r >= 0) fext_row[r + d] += N[i] * v;
        }
      }
    }
  }
  return FCG_OK;
}

}  // extern "C"
