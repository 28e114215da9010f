// fcg_tsi.hip -- thermo-structure interaction (TSI), geometrically linear, on the device: the
// temperature-dependent blocks of 4C's monolithic TSI tangent and the temperature-dependent parts
// of both residuals (BASELINE config 5).
//
// Reference (paths relative to the 4C tree):
//   f_S thermal stress   SolidScatraEleCalc::evaluate_nonlinear_force_stiffness_mass with a
//                        "temperature" state (4C_solid_scatra_3D_ele_calc.cpp:272-403) and
//                        Mat::ThermoStVenantKirchhoff::evaluate (4C_mat_thermostvenantkirchhoff.cpp:141-174)
//   k_ST                 struct_calc_stifftemp -> evaluate_d_stress_d_scalar
//                        (4C_solid_scatra_3D_ele_calc.cpp:405-490; dS/dT :250-295), assembled with
//                        AssembleStrategy(0, 1, k_st) by TSI::Monolithic::apply_str_coupl_matrix
//                        (4C_tsi_monolithic.cpp:1694-1767)
//   k_TT, f_T            calc_thermo_fintcond: linear_thermo_contribution (4C_thermo_ele_impl.cpp:802-891,
//                        Fourier conduction 4C_mat_fourier.cpp:147-192) + linear_disp_contribution (:899-1043)
//   k_TS                 calc_thermo_coupltang: linear_coupled_tang (4C_thermo_ele_impl.cpp:1046-1194)
// With a constant Young's modulus the stress-temperature modulus m = -(2 mu + 3 lambda) alpha_T
// (st_modulus, 4C_mat_thermostvenantkirchhoff.cpp:331-369) is constant, B_L^T (m,m,m,0,0,0) =
// m N_XYZ(a), and every block reduces to Gauss-point scalars:
//   f_S(a)   += sum_g fac m (T_g - T_0) N_XYZ(a)
//   K_ST(a,b) = sum_g fac m N_XYZ(a) N_b                                   (3 x 1 per node pair)
//   K_TS(a,b) = -timefac timefac_d sum_g fac N_a T_g m N_XYZ(b)^T            (1 x 3)
//   K_TT(a,b) = sum_g fac (k N_XYZ(a).N_XYZ(b) - m tr(e')_g N_a N_b)
//   f_T(a)    = sum_g fac (k N_XYZ(a).grad T_g - m tr(e')_g N_a T_g)
// with T_g = N.T, grad T_g = N_XYZ T and tr(e')_g = sum_b N_XYZ(b).v_b (e' = B_L v).
//
// Kernels: tsi_element_kernel (one wavefront per element: Gauss-point stage into LDS, then the
// node pairs; the block rows of every owned node go to an incidence-ordered scratch record) and
// tsi_assemble_kernel (one wavefront per owned node: its 3 k_ST rows, its k_TS row and its k_TT row
// are summed in element order in an LDS row image and written once, coalesced).  Owned rows only,
// no atomics, bitwise reproducible -- the contract of the structural path.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <climits>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "fcg_hex8_element.hpp"
#include "fcg_internal.hpp"
#include "fcg_status.hpp"
#include "fcg_shape.hpp"

namespace fcg {
namespace {

// scratch record of incidence (e, a): K_ST rows [3][npe] | K_TS row [npe][3] | K_TT row [npe] |
// f_S thermal part [3] | f_T [1]
__host__ __device__ constexpr int tsi_rec(int npe) { return 7 * npe + 4; }

struct TsiDevice {
  int npe = 8;
  int64_t n_ele = 0, n_node = 0, n_rownodes = 0, n_inc = 0;
  int64_t n_rows_s = 0, n_cols_s = 0, n_rows_t = 0, n_cols_t = 0;
  int64_t nnz_st = 0, nnz_ts = 0, nnz_tt = 0;
  double m = 0, T0 = 0, conduct = 0;
  int32_t* ele_nodes = nullptr;
  int32_t* ele_gid = nullptr;
  double* node_x = nullptr;
  int32_t* dof_col_s = nullptr;
  int32_t* dof_col_t = nullptr;
  int32_t* inc_of = nullptr;     // [n_ele][npe]
  int64_t* inc_ptr = nullptr;    // [n_rownodes + 1]
  int32_t* rn_srow = nullptr;    // [n_rownodes] first structural row
  int32_t* rn_trow = nullptr;    // [n_rownodes] thermo row
  uint16_t* pos_st = nullptr;    // [n_inc][npe] position of node b's thermo column in the k_ST rows
  uint16_t* pos_ts = nullptr;    // [n_inc][npe] position of node b's displacement triple in the k_TS row
  uint16_t* pos_tt = nullptr;    // [n_inc][npe] position of node b's thermo column in the k_TT row
  int64_t* rowptr_st = nullptr;
  int64_t* rowptr_ts = nullptr;
  int64_t* rowptr_tt = nullptr;
  double* tables = nullptr;      // dN at GPs [npe][npe][3] | N at GPs [npe][npe] | dN at nodes | w
  double* scratch = nullptr;     // [n_inc][tsi_rec(npe)]
  int32_t* err = nullptr;        // [2]
  // fused path (fcg_tsi_evaluate_fused): node-consistent numbering verified at create, the
  // structural context it was last verified against, the k_TT graph on the device for that check
  bool fusable = false;
  double lambda = 0, mu = 0;
  int32_t* col_tt = nullptr;
  const void* fused_with = nullptr;
};

template <int NPE>
struct TsiShared {
  double X[NPE * 3];
  double V[NPE * 3];
  double T[NPE];
  double N[NPE * NPE];        // [g][n]
  double NX[NPE * NPE * 3];   // [g][n][d]
  double fac[NPE], Tg[NPE], tr[NPE], gT[NPE * 3];
  int bad;
};

struct TsiElementArgs {
  int64_t n_ele;
  const int32_t* ele_nodes;
  const double* node_x;
  const int32_t* dof_col_s;
  const int32_t* dof_col_t;
  const double* v_col;
  const double* T_col;
  const int32_t* inc_of;
  const double* tables;
  double* scratch;
  int32_t* err;
  double m, T0, conduct, kts_fac;
  int want;  // fcg_tsi_part bits
};

template <int NPE>
__global__ __launch_bounds__(64) void tsi_element_kernel(TsiElementArgs A)
{
  constexpr int NGP = NPE;
  constexpr int REC = tsi_rec(NPE);
  __shared__ TsiShared<NPE> sh;
  const int lane = threadIdx.x;
  const double* dNgp = A.tables;
  const double* Ngp = A.tables + NGP * NPE * 3;
  const double* dNnode = Ngp + NGP * NPE;
  const double* wgp = dNnode + NPE * NPE * 3;
  for (int v = lane; v < NGP * NPE; v += 64) sh.N[v] = Ngp[v];
  const bool want_st = A.want & FCG_TSI_STIFFTEMP;
  const bool want_fs = A.want & FCG_TSI_STRUCT_FORCE;
  const bool want_t = A.want & FCG_TSI_THERMO_FINTCOND;
  const bool want_ts = A.want & FCG_TSI_COUPLTANG;

  for (int64_t e = blockIdx.x; e < A.n_ele; e += gridDim.x)
  {
    const int32_t* en = A.ele_nodes + e * NPE;
    for (int v = lane; v < 3 * NPE; v += 64)
    {
      const int a = v / 3, d = v - 3 * (v / 3);
      const int node = en[a];
      sh.X[v] = A.node_x[3 * int64_t(node) + d];
      sh.V[v] = want_t ? A.v_col[A.dof_col_s[node] + d] : 0.0;
    }
    for (int a = lane; a < NPE; a += 64) sh.T[a] = A.T_col[A.dof_col_t[en[a]]];
    if (lane == 0) sh.bad = 0;
    __syncthreads();

    // Gauss-point stage (eval_shape_func_and_derivs_at_int_point, 4C_thermo_ele_impl.cpp:2613-2671;
    // evaluate_jacobian_mapping, 4C_solid_3D_ele_calc_lib.hpp:435-448) and the nodal det J check
    // of struct_calc_stifftemp (4C_solid_scatra_3D_ele_calc.cpp:441, calc_lib.hpp:475-496)
    for (int t = lane; t < NGP + (want_st ? NPE : 0); t += 64)
    {
      const bool gp = t < NGP;
      const int g = gp ? t : t - NGP;
      const double* dN = (gp ? dNgp : dNnode) + 3 * NPE * g;
      double J[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) J[k] = 0.0;
      for (int c = 0; c < NPE; ++c)
      {
        const double d0 = dN[3 * c], d1 = dN[3 * c + 1], d2 = dN[3 * c + 2];
        const double x0 = sh.X[3 * c], x1 = sh.X[3 * c + 1], x2 = sh.X[3 * c + 2];
        J[0] += d0 * x0; J[1] += d1 * x0; J[2] += d2 * x0;
        J[3] += d0 * x1; J[4] += d1 * x1; J[5] += d2 * x1;
        J[6] += d0 * x2; J[7] += d1 * x2; J[8] += d2 * x2;
      }
      const double det = h8_invert3x3(J);
      if (!gp)
      {
        if (det == 0.0) atomicMax(&sh.bad, int(FCG_ERR_SINGULAR));
        else if (!(det > 0)) atomicMax(&sh.bad, int(FCG_ERR_NODAL_DETJ));
        continue;
      }
      // the thermo element throws for det < 1e-16 (4C_thermo_ele_impl.cpp:2663-2664)
      if (det == 0.0) atomicMax(&sh.bad, int(FCG_ERR_SINGULAR));
      else if (want_t && det < 1e-16) atomicMax(&sh.bad, int(FCG_ERR_NODAL_DETJ));
      const double fac = det * wgp[g];
      double Tg = 0.0, tr = 0.0, g0 = 0.0, g1 = 0.0, g2 = 0.0;
      for (int c = 0; c < NPE; ++c)
      {
        const double d0 = dN[3 * c], d1 = dN[3 * c + 1], d2 = dN[3 * c + 2];
        const double n0 = J[0] * d0 + J[3] * d1 + J[6] * d2;
        const double n1 = J[1] * d0 + J[4] * d1 + J[7] * d2;
        const double n2 = J[2] * d0 + J[5] * d1 + J[8] * d2;
        double* nx = sh.NX + 3 * (NPE * g + c);
        nx[0] = n0;
        nx[1] = n1;
        nx[2] = n2;
        const double Tc = sh.T[c];
        Tg += sh.N[NPE * g + c] * Tc;
        g0 += n0 * Tc;
        g1 += n1 * Tc;
        g2 += n2 * Tc;
        tr += n0 * sh.V[3 * c] + n1 * sh.V[3 * c + 1] + n2 * sh.V[3 * c + 2];
      }
      sh.fac[g] = fac;
      sh.Tg[g] = Tg;
      sh.tr[g] = tr;
      sh.gT[3 * g] = g0;
      sh.gT[3 * g + 1] = g1;
      sh.gT[3 * g + 2] = g2;
    }
    __syncthreads();
    if (sh.bad)
    {
      if (lane == 0)
      {
        atomicMax(&A.err[0], sh.bad);
        atomicMin(&A.err[1], int32_t(e));
      }
      __syncthreads();
      continue;
    }
    const int32_t* inc = A.inc_of + e * NPE;
    const double m = A.m, k = A.conduct;

    // node pairs (a, b): K_ST(a,b) [3], K_TS(a,b) [3], K_TT(a,b)
    if (want_st || want_ts || want_t)
      for (int p = lane; p < NPE * NPE; p += 64)
      {
        const int a = p / NPE, b = p - NPE * (p / NPE);
        const int32_t ia = inc[a];
        if (ia < 0) continue;
        double st0 = 0, st1 = 0, st2 = 0, ts0 = 0, ts1 = 0, ts2 = 0, tt = 0;
        for (int g = 0; g < NGP; ++g)
        {
          const double fac = sh.fac[g];
          const double* na = sh.NX + 3 * (NPE * g + a);
          const double* nb = sh.NX + 3 * (NPE * g + b);
          const double Na = sh.N[NPE * g + a], Nb = sh.N[NPE * g + b];
          const double cst = fac * m * Nb;
          st0 += cst * na[0];
          st1 += cst * na[1];
          st2 += cst * na[2];
          const double cts = fac * Na * sh.Tg[g] * m;
          ts0 += cts * nb[0];
          ts1 += cts * nb[1];
          ts2 += cts * nb[2];
          tt += fac * (k * (na[0] * nb[0] + na[1] * nb[1] + na[2] * nb[2]) - m * sh.tr[g] * Na * Nb);
        }
        double* rec = A.scratch + int64_t(ia) * REC;
        rec[b] = st0;
        rec[NPE + b] = st1;
        rec[2 * NPE + b] = st2;
        rec[3 * NPE + 3 * b] = A.kts_fac * ts0;
        rec[3 * NPE + 3 * b + 1] = A.kts_fac * ts1;
        rec[3 * NPE + 3 * b + 2] = A.kts_fac * ts2;
        rec[6 * NPE + b] = tt;
      }
    // per node: f_S thermal part [3], f_T
    if (want_fs || want_t)
      for (int a = lane; a < NPE; a += 64)
      {
        const int32_t ia = inc[a];
        if (ia < 0) continue;
        double f0 = 0, f1 = 0, f2 = 0, ft = 0;
        for (int g = 0; g < NGP; ++g)
        {
          const double fac = sh.fac[g];
          const double* na = sh.NX + 3 * (NPE * g + a);
          const double c = fac * m * (sh.Tg[g] - A.T0);
          f0 += c * na[0];
          f1 += c * na[1];
          f2 += c * na[2];
          const double* gt = sh.gT + 3 * g;
          ft += fac * (k * (na[0] * gt[0] + na[1] * gt[1] + na[2] * gt[2]) -
                          m * sh.tr[g] * sh.N[NPE * g + a] * sh.Tg[g]);
        }
        double* rec = A.scratch + int64_t(ia) * REC + 7 * NPE;
        rec[0] = f0;
        rec[1] = f1;
        rec[2] = f2;
        rec[3] = ft;
      }
    __syncthreads();
  }
}

struct TsiAssembleArgs {
  int64_t n_rownodes;
  const int64_t* inc_ptr;
  const int32_t* rn_srow;
  const int32_t* rn_trow;
  const uint16_t* pos_st;
  const uint16_t* pos_ts;
  const uint16_t* pos_tt;
  const double* scratch;
  const int64_t* rowptr_st;
  const int64_t* rowptr_ts;
  const int64_t* rowptr_tt;
  double* Kst;
  double* Kts;
  double* Ktt;
  double* fs;
  double* fT;
  int want;
  int overwrite;
};

template <int NPE>
__global__ __launch_bounds__(64) void tsi_assemble_kernel(TsiAssembleArgs A)
{
  constexpr int REC = tsi_rec(NPE);
  constexpr int MAXN = NPE == 8 ? 27 : 125;  // node neighbours of a row
  __shared__ double img_st[3 * MAXN];
  __shared__ double img_ts[3 * MAXN];
  __shared__ double img_tt[MAXN];
  const int lane = threadIdx.x;
  const bool st = A.want & FCG_TSI_STIFFTEMP;
  const bool ts = A.want & FCG_TSI_COUPLTANG;
  const bool tt = A.want & FCG_TSI_THERMO_FINTCOND;
  const bool fs = A.want & FCG_TSI_STRUCT_FORCE;
  for (int64_t r = blockIdx.x; r < A.n_rownodes; r += gridDim.x)
  {
    const int32_t srow = A.rn_srow[r], trow = A.rn_trow[r];
    const int lst = st ? int(A.rowptr_st[srow + 1] - A.rowptr_st[srow]) : 0;
    const int64_t bts = ts ? A.rowptr_ts[trow] : 0;
    const int lts = ts ? int(A.rowptr_ts[trow + 1] - bts) : 0;
    const int64_t btt = tt ? A.rowptr_tt[trow] : 0;
    const int ltt = tt ? int(A.rowptr_tt[trow + 1] - btt) : 0;
    for (int v = lane; v < 3 * MAXN; v += 64)
    {
      img_st[v] = 0.0;
      img_ts[v] = 0.0;
    }
    for (int v = lane; v < MAXN; v += 64) img_tt[v] = 0.0;
    double facc = 0.0;
    __syncthreads();
    for (int64_t q = A.inc_ptr[r]; q < A.inc_ptr[r + 1]; ++q)
    {
      const double* rec = A.scratch + q * REC;
      // 7 npe matrix entries of one incidence: distinct LDS targets
      for (int v = lane; v < 7 * NPE; v += 64)
      {
        if (v < 3 * NPE)
        {
          if (!st) continue;
          const int i = v / NPE, b = v - NPE * i;
          img_st[i * MAXN + A.pos_st[q * NPE + b]] += rec[v];
        }
        else if (v < 6 * NPE)
        {
          if (!ts) continue;
          const int w = v - 3 * NPE, b = w / 3, j = w - 3 * b;
          img_ts[A.pos_ts[q * NPE + b] + j] += rec[v];
        }
        else
        {
          if (!tt) continue;
          const int b = v - 6 * NPE;
          img_tt[A.pos_tt[q * NPE + b]] += rec[v];
        }
      }
      if (lane < 4) facc += rec[7 * NPE + lane];
      __syncthreads();
    }
    if (st)
      for (int v = lane; v < 3 * lst; v += 64)
      {
        const int i = v / lst, c = v - lst * i;
        double* dst = A.Kst + A.rowptr_st[srow + i] + c;
        if (A.overwrite)
          *dst = img_st[i * MAXN + c];
        else
          *dst += img_st[i * MAXN + c];
      }
    if (ts)
      for (int v = lane; v < lts; v += 64)
      {
        if (A.overwrite)
          A.Kts[bts + v] = img_ts[v];
        else
          A.Kts[bts + v] += img_ts[v];
      }
    if (tt)
      for (int v = lane; v < ltt; v += 64)
      {
        if (A.overwrite)
          A.Ktt[btt + v] = img_tt[v];
        else
          A.Ktt[btt + v] += img_tt[v];
      }
    // f_S: the thermal-stress part is added to the structural residual (its mechanical part comes
    // from fcg_evaluate_device); f_T follows the mode
    if (fs && lane < 3) A.fs[srow + lane] += facc;
    if (tt && lane == 3)
    {
      if (A.overwrite)
        A.fT[trow] = facc;
      else
        A.fT[trow] += facc;
    }
    __syncthreads();
  }
}

template <class T>
hipError_t upload(T** dst, const T* src, int64_t n, int64_t& bytes)
{
  *dst = nullptr;
  if (n <= 0) return hipSuccess;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(dst), sizeof(T) * n);
  if (e != hipSuccess) return e;
  bytes += int64_t(sizeof(T)) * n;
  if (src) return hipMemcpy(*dst, src, sizeof(T) * n, hipMemcpyHostToDevice);
  return hipMemset(*dst, 0, sizeof(T) * n);
}

// The structural context of a fused call describes the same mesh with the node graph of the TSI
// context: same elements, node coordinates and column DOFs, K rows = the 3 x 3 expansion of the k_TT rows.
struct FusedCheckArgs {
  int64_t n_node, n_ele8, n_rows_s;
  const int32_t* s_dof_col;
  const int32_t* t_dof_col_s;
  const int32_t* s_ele;
  const int32_t* t_ele;
  const double* s_x;
  const double* t_x;
  const int64_t* rp_ss;
  const int32_t* col_ss;
  const int64_t* rp_tt;
  const int32_t* col_tt;
  int32_t* flag;
};

__global__ __launch_bounds__(256) void tsi_fused_check_kernel(FusedCheckArgs A)
{
  const int64_t i0 = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t st = int64_t(gridDim.x) * blockDim.x;
  int bad = 0;
  for (int64_t i = i0; i < A.n_node; i += st)
    if (A.s_dof_col[i] != A.t_dof_col_s[i] || A.s_x[3 * i] != A.t_x[3 * i] ||
        A.s_x[3 * i + 1] != A.t_x[3 * i + 1] || A.s_x[3 * i + 2] != A.t_x[3 * i + 2])
      bad = 1;
  for (int64_t i = i0; i < A.n_ele8; i += st)
    if (A.s_ele[i] != A.t_ele[i]) bad = 1;
  for (int64_t r = i0; r < A.n_rows_s; r += st)
  {
    const int64_t t = r / 3, d = r - 3 * t;
    const int64_t b = A.rp_tt[t], lt = A.rp_tt[t + 1] - b;
    const int64_t rb = A.rp_ss[r];
    if (rb != 9 * b + 3 * d * lt || A.rp_ss[r + 1] - rb != 3 * lt)
    {
      bad = 1;
      continue;
    }
    for (int64_t j = 0; j < 3 * lt; ++j)
      if (A.col_ss[rb + j] != 3 * A.col_tt[b + j / 3] + int32_t(j % 3)) bad = 1;
  }
  if (bad) atomicOr(A.flag, 1);
}

std::mutex g_tsi_err_mutex;
std::string g_tsi_create_error;

void set_tsi_create_error(const std::string& s)
{
  std::lock_guard<std::mutex> lk(g_tsi_err_mutex);
  g_tsi_create_error = s;
}

int grid_for(int64_t work, int cap) { return int(work < cap ? (work > 0 ? work : 1) : cap); }

}  // namespace
}  // namespace fcg

struct fcg_tsi_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  fcg::TsiDevice d;
  std::string last_error;
  int64_t device_bytes = 0;
};

extern "C" {

const char* fcg_tsi_last_error(const fcg_tsi_ctx* ctx)
{
  if (ctx) return ctx->last_error.c_str();
  std::lock_guard<std::mutex> lk(fcg::g_tsi_err_mutex);
  return fcg::g_tsi_create_error.c_str();
}

int fcg_tsi_destroy(fcg_tsi_ctx* ctx)
{
  if (!ctx) return FCG_OK;
  (void)hipSetDevice(ctx->device);
  fcg::TsiDevice& d = ctx->d;
  void* ptrs[] = {d.ele_nodes, d.ele_gid, d.node_x, d.dof_col_s, d.dof_col_t, d.inc_of, d.inc_ptr,
      d.rn_srow, d.rn_trow, d.pos_st, d.pos_ts, d.pos_tt, d.rowptr_st, d.rowptr_ts, d.rowptr_tt,
      d.tables, d.scratch, d.err, d.col_tt};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return FCG_OK;
}

int fcg_tsi_create(const fcg_tsi_desc* D, fcg_tsi_ctx** out)
{
  using fcg::set_tsi_create_error;
  if (!D || !out) return FCG_ERR_ARG;
  *out = nullptr;
  if (D->abi_version != FCG_ABI_VERSION)
  {
    set_tsi_create_error("abi_version mismatch");
    return FCG_ERR_ARG;
  }
  if (D->celltype != FCG_HEX8 && D->celltype != FCG_HEX27)
  {
    set_tsi_create_error("unsupported celltype");
    return FCG_ERR_ARG;
  }
  // Mat::PAR::ThermoStVenantKirchhoff (4C_mat_thermostvenantkirchhoff.cpp:35-36)
  if (!(D->youngs > 0.0) || D->poisson >= 0.5 || D->poisson < -1.0)
  {
    set_tsi_create_error("Poisson's ratio must be in [-1;0.5) and Young's modulus > 0");
    return FCG_ERR_ARG;
  }
  const int npe = D->celltype == FCG_HEX27 ? 27 : 8;
  const int maxn = npe == 8 ? 27 : 125;
  if (D->n_ele < 0 || D->n_node < 0 || D->n_ele >= (int64_t(1) << 31) ||
      (D->n_ele > 0 && (!D->ele_nodes || !D->node_x || !D->node_dof_col_s || !D->node_dof_col_t ||
                           !D->node_dof_row_s || !D->node_dof_row_t)) ||
      (D->n_rows_s > 0 && (!D->rowptr_st || !D->col_st)) ||
      (D->n_rows_t > 0 && (!D->rowptr_ts || !D->col_ts || !D->rowptr_tt || !D->col_tt)))
  {
    set_tsi_create_error("invalid descriptor arrays/sizes");
    return FCG_ERR_ARG;
  }
  for (int64_t i = 0; i < D->n_ele * npe; ++i)
    if (D->ele_nodes[i] < 0 || D->ele_nodes[i] >= D->n_node)
    {
      set_tsi_create_error("element references a node outside [0, n_node)");
      return FCG_ERR_ARG;
    }
  // owned nodes: the structural rows and the thermo row are owned together
  std::vector<int32_t> rownodes;
  for (int64_t n = 0; n < D->n_node; ++n)
  {
    const int32_t rs = D->node_dof_row_s[n], rt = D->node_dof_row_t[n];
    const int32_t cs = D->node_dof_col_s[n], ct = D->node_dof_col_t[n];
    if ((rs >= 0) != (rt >= 0) || cs < 0 || cs + 3 > D->n_cols_s || ct < 0 || ct >= D->n_cols_t ||
        rs + 3 > D->n_rows_s || rt >= D->n_rows_t)
    {
      set_tsi_create_error("node DOF maps out of range, or a node owned in one field only");
      return FCG_ERR_ARG;
    }
    if (rs >= 0) rownodes.push_back(int32_t(n));
  }
  std::sort(rownodes.begin(), rownodes.end(),
      [&](int32_t a, int32_t b) { return D->node_dof_row_s[a] < D->node_dof_row_s[b]; });
  const int64_t nrn = int64_t(rownodes.size());
  std::vector<int32_t> rn_of_node(D->n_node, -1), srow(nrn), trow(nrn);
  for (int64_t r = 0; r < nrn; ++r)
  {
    rn_of_node[rownodes[r]] = int32_t(r);
    srow[r] = D->node_dof_row_s[rownodes[r]];
    trow[r] = D->node_dof_row_t[rownodes[r]];
  }
  // the 3 k_ST rows of a node share one list of at most maxn thermo columns
  for (int64_t r = 0; r < nrn; ++r)
  {
    const int64_t* p = D->rowptr_st + srow[r];
    const int64_t l = p[1] - p[0];
    if (l > maxn || p[2] - p[1] != l || p[3] - p[2] != l ||
        std::memcmp(D->col_st + p[0], D->col_st + p[1], sizeof(int32_t) * l) != 0 ||
        std::memcmp(D->col_st + p[0], D->col_st + p[2], sizeof(int32_t) * l) != 0 ||
        D->rowptr_ts[trow[r] + 1] - D->rowptr_ts[trow[r]] > 3 * maxn ||
        D->rowptr_tt[trow[r] + 1] - D->rowptr_tt[trow[r]] > maxn)
    {
      set_tsi_create_error("k_ST/k_TS/k_TT rows do not have the node-graph layout");
      return FCG_ERR_ARG;
    }
  }
  // incidences grouped by owned node, element order
  std::vector<int64_t> inc_ptr(nrn + 1, 0);
  for (int64_t i = 0; i < D->n_ele * npe; ++i)
  {
    const int32_t rn = rn_of_node[D->ele_nodes[i]];
    if (rn >= 0) inc_ptr[rn + 1]++;
  }
  for (int64_t r = 0; r < nrn; ++r) inc_ptr[r + 1] += inc_ptr[r];
  const int64_t n_inc = inc_ptr[nrn];
  if (n_inc >= (int64_t(1) << 31))
  {
    set_tsi_create_error("too many incidences for one context (> 2^31)");
    return FCG_ERR_ARG;
  }
  std::vector<int32_t> inc_of(D->n_ele * npe, -1), inc_ele(n_inc);
  {
    std::vector<int64_t> fill(inc_ptr.begin(), inc_ptr.end() - 1);
    for (int64_t e = 0; e < D->n_ele; ++e)
      for (int a = 0; a < npe; ++a)
      {
        const int32_t rn = rn_of_node[D->ele_nodes[e * npe + a]];
        if (rn < 0) continue;
        const int64_t k = fill[rn]++;
        inc_of[e * npe + a] = int32_t(k);
        inc_ele[k] = int32_t(e);
      }
  }
  // column positions (SparseMatrix::assemble's row search, 4C_linalg_sparsematrix.cpp:471-543,
  // resolved once)
  std::vector<uint16_t> pos_st(n_inc * npe), pos_ts(n_inc * npe), pos_tt(n_inc * npe);
  for (int64_t r = 0; r < nrn; ++r)
  {
    const int32_t* cst = D->col_st + D->rowptr_st[srow[r]];
    const int64_t lst = D->rowptr_st[srow[r] + 1] - D->rowptr_st[srow[r]];
    const int32_t* cts = D->col_ts + D->rowptr_ts[trow[r]];
    const int64_t lts = D->rowptr_ts[trow[r] + 1] - D->rowptr_ts[trow[r]];
    const int32_t* ctt = D->col_tt + D->rowptr_tt[trow[r]];
    const int64_t ltt = D->rowptr_tt[trow[r] + 1] - D->rowptr_tt[trow[r]];
    for (int64_t k = inc_ptr[r]; k < inc_ptr[r + 1]; ++k)
    {
      const int32_t* en = D->ele_nodes + int64_t(inc_ele[k]) * npe;
      for (int b = 0; b < npe; ++b)
      {
        const int32_t tc = D->node_dof_col_t[en[b]], sc = D->node_dof_col_s[en[b]];
        const int32_t* i1 = std::lower_bound(cst, cst + lst, tc);
        const int32_t* i2 = std::lower_bound(cts, cts + lts, sc);
        const int32_t* i3 = std::lower_bound(ctt, ctt + ltt, tc);
        if (i1 == cst + lst || *i1 != tc || i3 == ctt + ltt || *i3 != tc ||
            i2 + 3 > cts + lts || i2[0] != sc || i2[1] != sc + 1 || i2[2] != sc + 2)
        {
          set_tsi_create_error("a TSI block graph lacks an element coupling, or a node's "
                               "displacement columns are not contiguous");
          return FCG_ERR_ARG;
        }
        pos_st[k * npe + b] = uint16_t(i1 - cst);
        pos_ts[k * npe + b] = uint16_t(i2 - cts);
        pos_tt[k * npe + b] = uint16_t(i3 - ctt);
      }
    }
  }
  // tables: dN at GPs | N at GPs | dN at nodes | weights (hex_8point / hex_27point: the thermo
  // element's DisTypeToOptGaussRule, 4C_thermo_ele_impl_utils.hpp:28-50, is the solid's rule)
  const int ct = D->celltype == FCG_HEX27 ? fcg::kHex27 : fcg::kHex8;
  std::vector<double> tab(npe * npe * 3 * 2 + npe * npe + npe);
  {
    double xi[81], w[27], xn[81];
    fcg::gauss_rule(ct, xi, w);
    fcg::node_param_coords(ct, xn);
    double* dNg = tab.data();
    double* Ng = dNg + npe * npe * 3;
    double* dNn = Ng + npe * npe;
    double* wg = dNn + npe * npe * 3;
    for (int g = 0; g < npe; ++g)
    {
      fcg::shape_deriv(ct, &xi[3 * g], dNg + 3 * npe * g);
      fcg::shape_values(ct, &xi[3 * g], Ng + npe * g);
      fcg::shape_deriv(ct, &xn[3 * g], dNn + 3 * npe * g);
      wg[g] = w[g];
    }
  }

  // node-consistent numbering (what fcg_tsi_evaluate_fused requires): thermo DOF LIDs are the
  // structural ones / 3 and the three block graphs are expansions of one node graph (the k_TT graph)
  bool fusable = npe == 8 && D->n_rows_s == 3 * D->n_rows_t && D->n_cols_s == 3 * D->n_cols_t;
  for (int64_t n = 0; fusable && n < D->n_node; ++n)
    fusable = D->node_dof_col_s[n] == 3 * D->node_dof_col_t[n] &&
              D->node_dof_row_s[n] == (D->node_dof_row_t[n] < 0 ? D->node_dof_row_s[n] : 3 * D->node_dof_row_t[n]);
  for (int64_t t = 0; fusable && t < D->n_rows_t; ++t)
  {
    const int64_t b = D->rowptr_tt[t], lt = D->rowptr_tt[t + 1] - b;
    fusable = D->rowptr_ts[t] == 3 * b && D->rowptr_ts[t + 1] - D->rowptr_ts[t] == 3 * lt;
    for (int d = 0; fusable && d < 3; ++d)
      fusable = D->rowptr_st[3 * t + d] == 3 * b + d * lt &&
                std::memcmp(D->col_st + D->rowptr_st[3 * t + d], D->col_tt + b, sizeof(int32_t) * lt) == 0;
    for (int64_t j = 0; fusable && j < 3 * lt; ++j)
      fusable = D->col_ts[3 * b + j] == 3 * D->col_tt[b + j / 3] + int32_t(j % 3);
  }
  if (fusable && D->n_rows_t > 0)
    fusable = D->rowptr_st[D->n_rows_s] == 3 * D->rowptr_tt[D->n_rows_t] &&
              D->rowptr_ts[D->n_rows_t] == 3 * D->rowptr_tt[D->n_rows_t];

  auto* ctx = new fcg_tsi_ctx();
  ctx->device = D->device;
  hipError_t he = hipSetDevice(D->device);
  if (he == hipSuccess) he = hipStreamCreateWithFlags(&ctx->stream, hipStreamDefault);  // ordered with the null stream (torch's default)
  if (he != hipSuccess)
  {
    set_tsi_create_error(std::string("HIP: ") + hipGetErrorString(he));
    delete ctx;
    return fcg_device_error();
  }
  fcg::TsiDevice& d = ctx->d;
  d.npe = npe;
  d.n_ele = D->n_ele;
  d.n_node = D->n_node;
  d.n_rownodes = nrn;
  d.n_inc = n_inc;
  d.n_rows_s = D->n_rows_s;
  d.n_cols_s = D->n_cols_s;
  d.n_rows_t = D->n_rows_t;
  d.n_cols_t = D->n_cols_t;
  d.nnz_st = D->n_rows_s ? D->rowptr_st[D->n_rows_s] : 0;
  d.nnz_ts = D->n_rows_t ? D->rowptr_ts[D->n_rows_t] : 0;
  d.nnz_tt = D->n_rows_t ? D->rowptr_tt[D->n_rows_t] : 0;
  // st_modulus (4C_mat_thermostvenantkirchhoff.cpp:331-369)
  {
    const double c1 = D->youngs / (1.0 + D->poisson);
    const double b1 = c1 * D->poisson / (1.0 - 2.0 * D->poisson);
    const double mu = 0.5 * c1, lambda = b1;
    d.m = (-1.0) * (2.0 * mu + 3.0 * lambda) * D->thexpans;
    d.lambda = lambda;
    d.mu = mu;
  }
  d.fusable = fusable;
  d.T0 = D->inittemp;
  d.conduct = D->conduct;
  std::vector<int32_t> eg;
  if (!D->ele_gid)
  {
    eg.resize(D->n_ele);
    for (int64_t e = 0; e < D->n_ele; ++e) eg[e] = int32_t(e);
  }
  int64_t& bytes = ctx->device_bytes;
  he = hipSuccess;
  auto chk = [&](hipError_t x) {
    if (he == hipSuccess) he = x;
  };
  using fcg::upload;
  chk(upload(&d.ele_nodes, D->ele_nodes, D->n_ele * npe, bytes));
  chk(upload(&d.ele_gid, D->ele_gid ? D->ele_gid : eg.data(), D->n_ele, bytes));
  chk(upload(&d.node_x, D->node_x, D->n_node * 3, bytes));
  chk(upload(&d.dof_col_s, D->node_dof_col_s, D->n_node, bytes));
  chk(upload(&d.dof_col_t, D->node_dof_col_t, D->n_node, bytes));
  chk(upload(&d.inc_of, inc_of.data(), D->n_ele * npe, bytes));
  chk(upload(&d.inc_ptr, inc_ptr.data(), nrn + 1, bytes));
  chk(upload(&d.rn_srow, srow.data(), nrn, bytes));
  chk(upload(&d.rn_trow, trow.data(), nrn, bytes));
  chk(upload(&d.pos_st, pos_st.data(), n_inc * npe, bytes));
  chk(upload(&d.pos_ts, pos_ts.data(), n_inc * npe, bytes));
  chk(upload(&d.pos_tt, pos_tt.data(), n_inc * npe, bytes));
  chk(upload(&d.rowptr_st, D->rowptr_st, D->n_rows_s + 1, bytes));
  chk(upload(&d.rowptr_ts, D->rowptr_ts, D->n_rows_t + 1, bytes));
  chk(upload(&d.rowptr_tt, D->rowptr_tt, D->n_rows_t + 1, bytes));
  chk(upload(&d.tables, tab.data(), int64_t(tab.size()), bytes));
  chk(upload<double>(&d.scratch, nullptr, n_inc * fcg::tsi_rec(npe), bytes));
  chk(upload<int32_t>(&d.err, nullptr, 2, bytes));
  if (fusable) chk(upload(&d.col_tt, D->col_tt, d.nnz_tt, bytes));
  if (he != hipSuccess)
  {
    set_tsi_create_error(std::string("HIP allocation/copy failed: ") + hipGetErrorString(he));
    fcg_tsi_destroy(ctx);
    return fcg_device_error();
  }
  *out = ctx;
  return FCG_OK;
}

int fcg_tsi_evaluate_device(fcg_tsi_ctx* ctx, int parts, int mode, const double* d_v_col,
    const double* d_T_col, double timefac, double timefac_d, double* d_fs_row, double* d_Kst,
    double* d_fT_row, double* d_Ktt, double* d_Kts, void* stream_ptr, int32_t* bad_ele_gid)
{
  if (!ctx) return FCG_ERR_ARG;
  fcg::TsiDevice& d = ctx->d;
  const bool st = parts & FCG_TSI_STIFFTEMP, ts = parts & FCG_TSI_COUPLTANG;
  const bool tt = parts & FCG_TSI_THERMO_FINTCOND, fs = parts & FCG_TSI_STRUCT_FORCE;
  if ((parts & ~0xF) || !parts || (mode != FCG_ACCUMULATE && mode != FCG_OVERWRITE) ||
      (d.n_ele > 0 && !d_T_col) || (tt && d.n_ele > 0 && !d_v_col) ||
      (fs && d.n_rows_s > 0 && !d_fs_row) || (st && d.nnz_st > 0 && !d_Kst) ||
      (tt && d.n_rows_t > 0 && (!d_fT_row || (d.nnz_tt > 0 && !d_Ktt))) ||
      (ts && d.nnz_ts > 0 && !d_Kts))
  {
    ctx->last_error = "invalid TSI evaluate arguments";
    return FCG_ERR_ARG;
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream_ptr ? static_cast<hipStream_t>(stream_ptr) : ctx->stream;
  const int32_t init[2] = {0, INT32_MAX};
  hipError_t he = hipMemcpyAsync(d.err, init, sizeof(init), hipMemcpyHostToDevice, s);
  if (he == hipSuccess && d.n_ele > 0)
  {
    fcg::TsiElementArgs a;
    a.n_ele = d.n_ele;
    a.ele_nodes = d.ele_nodes;
    a.node_x = d.node_x;
    a.dof_col_s = d.dof_col_s;
    a.dof_col_t = d.dof_col_t;
    a.v_col = d_v_col;
    a.T_col = d_T_col;
    a.inc_of = d.inc_of;
    a.tables = d.tables;
    a.scratch = d.scratch;
    a.err = d.err;
    a.m = d.m;
    a.T0 = d.T0;
    a.conduct = d.conduct;
    a.kts_fac = -timefac * timefac_d;  // linear_coupled_tang (4C_thermo_ele_impl.cpp:1189)
    a.want = parts;
    const int grid = fcg::grid_for(d.n_ele, 256 * 32);
    if (d.npe == 8)
      hipLaunchKernelGGL(fcg::tsi_element_kernel<8>, dim3(grid), dim3(64), 0, s, a);
    else
      hipLaunchKernelGGL(fcg::tsi_element_kernel<27>, dim3(grid), dim3(64), 0, s, a);
    he = hipGetLastError();
  }
  if (he == hipSuccess && d.n_rownodes > 0)
  {
    fcg::TsiAssembleArgs a;
    a.n_rownodes = d.n_rownodes;
    a.inc_ptr = d.inc_ptr;
    a.rn_srow = d.rn_srow;
    a.rn_trow = d.rn_trow;
    a.pos_st = d.pos_st;
    a.pos_ts = d.pos_ts;
    a.pos_tt = d.pos_tt;
    a.scratch = d.scratch;
    a.rowptr_st = d.rowptr_st;
    a.rowptr_ts = d.rowptr_ts;
    a.rowptr_tt = d.rowptr_tt;
    a.Kst = d_Kst;
    a.Kts = d_Kts;
    a.Ktt = d_Ktt;
    a.fs = d_fs_row;
    a.fT = d_fT_row;
    a.want = parts;
    a.overwrite = mode == FCG_OVERWRITE;
    const int grid = fcg::grid_for(d.n_rownodes, 256 * 32);
    if (d.npe == 8)
      hipLaunchKernelGGL(fcg::tsi_assemble_kernel<8>, dim3(grid), dim3(64), 0, s, a);
    else
      hipLaunchKernelGGL(fcg::tsi_assemble_kernel<27>, dim3(grid), dim3(64), 0, s, a);
    he = hipGetLastError();
  }
  int32_t errv[2] = {0, INT32_MAX};
  if (he == hipSuccess) he = hipMemcpyAsync(errv, d.err, sizeof(errv), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  if (errv[0] != 0)
  {
    int32_t gid = -1;
    if (errv[1] >= 0 && errv[1] < d.n_ele)
      (void)hipMemcpy(&gid, d.ele_gid + errv[1], sizeof(int32_t), hipMemcpyDeviceToHost);
    if (bad_ele_gid) *bad_ele_gid = gid;
    ctx->last_error = errv[0] == FCG_ERR_NODAL_DETJ
                          ? "non-positive jacobian determinant in element " + std::to_string(gid)
                          : "singular 3x3 matrix in element " + std::to_string(gid);
    return errv[0];
  }
  return FCG_OK;
}

int fcg_tsi_evaluate_fused(fcg_ctx* sctx, fcg_tsi_ctx* ctx, int mode, const double* d_u_col,
    const double* d_v_col, const double* d_T_col, double timefac, double timefac_d,
    double* d_fs_row, double* d_Kss, double* d_Kst, double* d_fT_row, double* d_Ktt,
    double* d_Kts, void* stream_ptr, int32_t* bad_ele_gid)
{
  if (!ctx) return FCG_ERR_ARG;
  if (!sctx)
  {
    ctx->last_error = "no structural context";
    return FCG_ERR_ARG;
  }
  fcg::TsiDevice& d = ctx->d;
  const fcg::DeviceMesh& m = sctx->mesh;
  auto rel_eq = [](double a, double b) { return std::fabs(a - b) <= 1e-14 * std::fabs(b); };
  if (m.path != FCG_PATH_STRUCTURED || m.kinem != 0 || m.material != FCG_MAT_STVK || m.npe != 8 ||
      !d.fusable || sctx->device != ctx->device || m.n_node != d.n_node || m.n_ele != d.n_ele ||
      m.n_rows != d.n_rows_s || m.n_cols != d.n_cols_s || m.nnz != 9 * d.nnz_tt ||
      !rel_eq(m.lambda, d.lambda) || !rel_eq(m.mu, d.mu))
  {
    ctx->last_error =
        "fused TSI needs a structured hex8 StVK context with linear kinematics, the TSI material's "
        "E and nu, and node-consistent thermo numbering (thermo LID = structural LID / 3)";
    return FCG_ERR_ARG;
  }
  if ((mode != FCG_ACCUMULATE && mode != FCG_OVERWRITE) ||
      (d.n_ele > 0 && (!d_u_col || !d_v_col || !d_T_col)) ||
      (d.n_rows_s > 0 && (!d_fs_row || !d_Kss || !d_Kst || !d_fT_row || !d_Ktt || !d_Kts)))
  {
    ctx->last_error = "invalid fused TSI evaluate arguments";
    return FCG_ERR_ARG;
  }
  (void)hipSetDevice(ctx->device);
  // the fused pass re-initialises the structural context's flags: a queued (async) evaluate's
  // failure is reported first, as fcg_evaluate_host does, instead of being overwritten
  if (sctx->pending)
  {
    const int rc = fcg_check_error(sctx, bad_ele_gid);
    if (rc != FCG_OK) return rc;
  }
  hipStream_t s = stream_ptr ? static_cast<hipStream_t>(stream_ptr) : ctx->stream;
  hipError_t he = hipSuccess;
  if (d.fused_with != static_cast<const void*>(sctx))
  {
    fcg::FusedCheckArgs c;
    c.n_node = d.n_node;
    c.n_ele8 = d.n_ele * 8;
    c.n_rows_s = d.n_rows_s;
    c.s_dof_col = m.node_dof_col;
    c.t_dof_col_s = d.dof_col_s;
    c.s_ele = m.ele_nodes;
    c.t_ele = d.ele_nodes;
    c.s_x = m.node_x;
    c.t_x = d.node_x;
    c.rp_ss = m.rowptr;
    c.col_ss = m.col_lid;
    c.rp_tt = d.rowptr_tt;
    c.col_tt = d.col_tt;
    c.flag = d.err;
    int32_t flag = 0;
    he = hipMemcpyAsync(d.err, &flag, sizeof(flag), hipMemcpyHostToDevice, s);
    if (he == hipSuccess)
    {
      const int64_t work = std::max(std::max(d.n_node, d.n_ele * 8), d.n_rows_s);
      hipLaunchKernelGGL(fcg::tsi_fused_check_kernel, dim3(fcg::grid_for((work + 255) / 256, 4096)),
          dim3(256), 0, s, c);
      he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemcpyAsync(&flag, d.err, sizeof(flag), hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    if (he != hipSuccess)
    {
      ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
      return fcg_device_error();
    }
    if (flag)
    {
      ctx->last_error = "structural context and TSI context do not share the mesh and node graph";
      return FCG_ERR_ARG;
    }
    d.fused_with = sctx;
  }
  const int32_t init[2] = {0, INT32_MAX};
  sctx->mesh.err_clean = false;  // the fused sweep reports through the structural context's flags
  he = hipMemcpyAsync(m.err, init, sizeof(init), hipMemcpyHostToDevice, s);
  if (he == hipSuccess)
  {
    fcg::SweepTsi t;
    t.v_col = d_v_col;
    t.T_col = d_T_col;
    t.Ngp = d.tables + 8 * 8 * 3;
    t.Kst = d_Kst;
    t.Kts = d_Kts;
    t.Ktt = d_Ktt;
    t.fT = d_fT_row;
    t.m = d.m;
    t.T0 = d.T0;
    t.conduct = d.conduct;
    t.kts = -timefac * timefac_d;  // linear_coupled_tang (4C_thermo_ele_impl.cpp:1189)
    // the structural sweep + a thermal-only pass (default), or the one fused pass
    static const bool split = [] {
      const char* e = std::getenv("FCG_TSI_SPLIT");
      return !(e && e[0] == '0');
    }();
    t.split = split;
    he = fcg::launch_sweep_h8_tsi(m, d_u_col, mode == FCG_OVERWRITE, d_Kss, d_fs_row, t, s);
  }
  int32_t errv[2] = {0, INT32_MAX};
  if (he == hipSuccess) he = hipMemcpyAsync(errv, m.err, sizeof(errv), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  if (errv[0] != 0)
  {
    int32_t gid = -1;
    if (errv[1] >= 0 && errv[1] < m.n_ele)
      (void)hipMemcpy(&gid, m.ele_gid + errv[1], sizeof(int32_t), hipMemcpyDeviceToHost);
    if (bad_ele_gid) *bad_ele_gid = gid;
    ctx->last_error = errv[0] == FCG_ERR_NODAL_DETJ
                          ? "non-positive jacobian determinant in element " + std::to_string(gid)
                          : "singular 3x3 matrix in element " + std::to_string(gid);
    return errv[0];
  }
  return FCG_OK;
}

}  // extern "C"
