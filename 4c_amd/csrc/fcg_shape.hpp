// fcg_shape.hpp -- hex8 / hex27 Lagrange shape-function derivatives and Gauss rules used to build
// the constant tables of the element kernels (host side, once per context).
//
// Follows 4C's definitions:
//   hex_8point / hex_27point rules  src/core/fem/src/general/utils/4C_fem_general_utils_integration.cpp:74-106,130-245
//     (hex27 keeps the reference's truncated constants xi = 0.7745966692415, w = 0.5555555555556 /
//      0.8888888888889 so that results match 4C, not the exact Gauss-Legendre values)
//   derivatives  src/core/fem/src/general/utils/4C_fem_general_utils_fem_shapefunctions.hpp:386-426,683-788
//   node parameter coordinates  .../4C_fem_general_utils_local_connectivity_matrices.hpp:291-297
// The hex27 functions are tensor products of the 1-D quadratic Lagrange polynomials on
// {-1, 0, 1}; we evaluate them through that factorisation (per-node index triple) instead of the
// reference's 27 hand-written lines -- same polynomials, products taken in the reference's order.
#pragma once

#include <cmath>

namespace fcg {

constexpr int kHex8 = 0;
constexpr int kHex27 = 1;

// Position index (-1, 0, +1 -> 0, 1, 2) of every hex27 node in parameter space.
static const int kHex27NodePos[27][3] = {{0, 0, 0}, {2, 0, 0}, {2, 2, 0}, {0, 2, 0}, {0, 0, 2},
    {2, 0, 2}, {2, 2, 2}, {0, 2, 2}, {1, 0, 0}, {2, 1, 0}, {1, 2, 0}, {0, 1, 0}, {0, 0, 1},
    {2, 0, 1}, {2, 2, 1}, {0, 2, 1}, {1, 0, 2}, {2, 1, 2}, {1, 2, 2}, {0, 1, 2}, {1, 1, 0},
    {1, 0, 1}, {2, 1, 1}, {1, 2, 1}, {0, 1, 1}, {1, 1, 2}, {1, 1, 1}};

// Gauss-point position indices of hex_27point (same table as the nodes: the reference lists the
// 27 points in node order) and of hex_8point (corner order).
inline int num_nodes(int celltype) { return celltype == kHex27 ? 27 : 8; }

inline void gauss_rule(int celltype, double* xi, double* w)
{
  if (celltype == kHex8)
  {
    const double a = 1.0 / std::sqrt(3.0);
    for (int g = 0; g < 8; ++g)
    {
      for (int d = 0; d < 3; ++d) xi[3 * g + d] = (kHex27NodePos[g][d] == 0 ? -a : a);
      w[g] = 1.0;
    }
    return;
  }
  const double a = 0.7745966692415;
  const double w1 = 0.5555555555556, w2 = 0.8888888888889;
  for (int g = 0; g < 27; ++g)
  {
    double wg[3];
    for (int d = 0; d < 3; ++d)
    {
      const int p = kHex27NodePos[g][d];
      xi[3 * g + d] = (p == 0 ? -a : (p == 2 ? a : 0.0));
      wg[d] = (p == 1 ? w2 : w1);
    }
    w[g] = wg[0] * wg[1] * wg[2];
  }
}

inline void node_param_coords(int celltype, double* xi)
{
  for (int i = 0; i < num_nodes(celltype); ++i)
    for (int d = 0; d < 3; ++d) xi[3 * i + d] = double(kHex27NodePos[i][d] - 1);
}

// dN[3*node + d] = dN_node / dxi_d at xi.
inline void shape_deriv(int celltype, const double* xi, double* dN)
{
  if (celltype == kHex8)
  {
    for (int n = 0; n < 8; ++n)
    {
      double s[3], p[3];
      for (int d = 0; d < 3; ++d)
      {
        s[d] = (kHex27NodePos[n][d] == 0 ? -1.0 : 1.0);
        p[d] = 1.0 + s[d] * xi[d];
      }
      // reference: deriv(0,n) = +-Q18 * (1+-s)(1+-t), etc.
      dN[3 * n + 0] = 0.125 * s[0] * p[1] * p[2];
      dN[3 * n + 1] = 0.125 * s[1] * p[2] * p[0];
      dN[3 * n + 2] = 0.125 * s[2] * p[0] * p[1];
    }
    return;
  }
  double L[3][3], dL[3][3];
  for (int d = 0; d < 3; ++d)
  {
    const double r = xi[d];
    L[d][0] = 0.5 * r * (r - 1.0);
    L[d][1] = 1.0 - r * r;
    L[d][2] = 0.5 * r * (r + 1.0);
    dL[d][0] = r - 0.5;
    dL[d][1] = -2.0 * r;
    dL[d][2] = r + 0.5;
  }
  for (int n = 0; n < 27; ++n)
  {
    const int i = kHex27NodePos[n][0], j = kHex27NodePos[n][1], k = kHex27NodePos[n][2];
    dN[3 * n + 0] = L[1][j] * L[2][k] * dL[0][i];
    dN[3 * n + 1] = L[0][i] * L[2][k] * dL[1][j];
    dN[3 * n + 2] = L[0][i] * L[1][j] * dL[2][k];
  }
}

// N[node] at xi (shape_function_3d, 4C_fem_general_utils_fem_shapefunctions.hpp:53-72,190-229).
inline void shape_values(int celltype, const double* xi, double* N)
{
  if (celltype == kHex8)
  {
    for (int n = 0; n < 8; ++n)
    {
      double p[3];
      for (int d = 0; d < 3; ++d) p[d] = 1.0 + (kHex27NodePos[n][d] == 0 ? -1.0 : 1.0) * xi[d];
      N[n] = 0.125 * p[0] * p[1] * p[2];
    }
    return;
  }
  double L[3][3];
  for (int d = 0; d < 3; ++d)
  {
    const double r = xi[d];
    L[d][0] = 0.5 * r * (r - 1.0);
    L[d][1] = 1.0 - r * r;
    L[d][2] = 0.5 * r * (r + 1.0);
  }
  for (int n = 0; n < 27; ++n)
    N[n] = L[0][kHex27NodePos[n][0]] * L[1][kHex27NodePos[n][1]] * L[2][kHex27NodePos[n][2]];
}

}  // namespace fcg
