// integration_4c.cpp -- the INTEGRATION.md binding (lines "Filling fcg_desc from a 4C
// discretization") compiled and run as written.  TEST INFRASTRUCTURE.
//
// The 4C side is played by minimal stand-ins with the method names the snippet calls
// (Discretization::element_col_map / node_col_map / l_col_element / l_col_node / dof_row_map /
// dof_col_map / dof, Epetra_Map::NumMyElements / LID, Epetra_CrsMatrix::ExtractCrsDataPointers /
// ColMap, Vector::get_values, FOUR_C_THROW), filled from the GridGenerator restatement
// (fcg_box_mesh_*) -- what a 4C rank holds after fill_complete() and the first stiff->complete().
// The results of fcg_evaluate, of the C++ facade (fourc_gpu.hpp: Discretization::evaluate with
// a ParameterList "action") and of its zero()-fused variant are compared with the CPU oracle
// (liborc) on the same rank.
//
// usage: integration_4c [nx ny nz] [nranks] [--expect-no-device]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "fourc_gpu.h"
#include "fourc_gpu.hpp"
#include "fourc_oracle.h"

// FOUR_C_THROW stand-in: the format string and its arguments, space separated
template <class... A>
static std::string FourC_fmt(const A&... a)
{
  std::ostringstream os;
  ((os << ' ' << a), ...);
  return os.str();
}
#define FOUR_C_THROW(fmt, ...) throw std::runtime_error(std::string(fmt) + FourC_fmt(__VA_ARGS__))

// ------------------------------------------------------------------ 4C stand-ins
struct Epetra_Map {
  std::vector<int> gids;
  std::unordered_map<int, int> lid;
  explicit Epetra_Map(std::vector<int> g = {}) : gids(std::move(g))
  {
    for (size_t i = 0; i < gids.size(); ++i) lid[gids[i]] = int(i);
  }
  int NumMyElements() const { return int(gids.size()); }
  int LID(int gid) const
  {
    auto it = lid.find(gid);
    return it == lid.end() ? -1 : it->second;
  }
};
struct Node {
  int gid;
  double xyz[3];
  int id() const { return gid; }
  const double* x() const { return xyz; }
};
struct Element {
  int gid;
  std::vector<int> nodes;
  int id() const { return gid; }
  int num_node() const { return int(nodes.size()); }
  const int* node_ids() const { return nodes.data(); }
};
struct Discretization {
  Epetra_Map elecol, nodecol, dofrow, dofcol;
  std::vector<Element> eles;
  std::vector<Node> nodes;
  const Epetra_Map* element_col_map() const { return &elecol; }
  const Epetra_Map* node_col_map() const { return &nodecol; }
  const Epetra_Map* dof_row_map() const { return &dofrow; }
  const Epetra_Map* dof_col_map() const { return &dofcol; }
  const Element* l_col_element(int e) const { return &eles[e]; }
  const Node* l_col_node(int n) const { return &nodes[n]; }
  int dof(const Node* n, int j) const { return 3 * n->id() + j; }  // DofSet, first node gid 0
};
struct Epetra_CrsMatrix {
  std::vector<int> rowptr, cols;
  std::vector<double> vals;
  Epetra_Map colmap;
  int ExtractCrsDataPointers(int*& rp, int*& ci, double*& v)
  {
    rp = rowptr.data();
    ci = cols.data();
    v = vals.data();
    return 0;
  }
  const Epetra_Map& ColMap() const { return colmap; }
};
struct SparseMatrix {
  std::shared_ptr<Epetra_CrsMatrix> m = std::make_shared<Epetra_CrsMatrix>();
  Epetra_CrsMatrix* epetra_matrix() { return m.get(); }
};
struct Vector {
  std::vector<double> v;
  double* get_values() { return v.data(); }
};
struct StVK {
  double youngs_ = 210.0, poisson_ratio_ = 0.3;
};

// ------------------------------------------------------------------ the rank's state from the box
static void build_rank(const fcg_box& box, int rank, int nranks, Discretization& dis,
    SparseMatrix& stiff, fcg_box_mesh** keep)
{
  if (fcg_box_mesh_create(&box, rank, nranks, keep) != FCG_OK) throw std::runtime_error("box mesh");
  fcg_desc d;
  fcg_box_mesh_desc(*keep, FCG_LINEAR, 1.0, 0.0, 0, &d);
  const int32_t *row_gid, *col_gid, *owner;
  const int64_t* node_gid;
  fcg_box_mesh_maps(*keep, &row_gid, &col_gid, &node_gid, &owner);
  std::vector<int> ng(d.n_node), eg(d.n_ele);
  for (int64_t n = 0; n < d.n_node; ++n)
  {
    ng[n] = int(node_gid[n]);
    dis.nodes.push_back({ng[n], {d.node_x[3 * n], d.node_x[3 * n + 1], d.node_x[3 * n + 2]}});
  }
  const int npe = d.celltype == FCG_HEX8 ? 8 : 27;
  for (int64_t e = 0; e < d.n_ele; ++e)
  {
    eg[e] = d.ele_gid[e];
    Element el{d.ele_gid[e], {}};
    for (int a = 0; a < npe; ++a) el.nodes.push_back(ng[d.ele_nodes[npe * e + a]]);
    dis.eles.push_back(el);
  }
  dis.elecol = Epetra_Map(eg);
  dis.nodecol = Epetra_Map(ng);
  dis.dofrow = Epetra_Map(std::vector<int>(row_gid, row_gid + d.n_rows));
  dis.dofcol = Epetra_Map(std::vector<int>(col_gid, col_gid + d.n_cols));
  auto& M = *stiff.epetra_matrix();
  M.rowptr.assign(d.rowptr, d.rowptr + d.n_rows + 1);
  M.cols.assign(d.col_lid, d.col_lid + d.rowptr[d.n_rows]);
  M.vals.assign(d.rowptr[d.n_rows], 0.0);  // Structure::reset: stiff zeroed
  M.colmap = dis.dofcol;                   // FillComplete's column map = the DOF column map here
}

static double rel(const std::vector<double>& a, const std::vector<double>& b)
{
  double num = 0, den = 0;
  for (size_t i = 0; i < a.size(); ++i)
  {
    num += (a[i] - b[i]) * (a[i] - b[i]);
    den += b[i] * b[i];
  }
  return std::sqrt(num / (den > 0 ? den : 1.0));
}

int main(int argc, char** argv)
{
  int iv[3] = {6, 5, 4}, nranks = 2;
  bool expect_no_device = false;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i)
  {
    if (!std::strcmp(argv[i], "--expect-no-device"))
      expect_no_device = true;
    else
      pos.push_back(argv[i]);
  }
  if (pos.size() >= 3)
    for (int k = 0; k < 3; ++k) iv[k] = std::atoi(pos[k].c_str());
  if (pos.size() >= 4) nranks = std::atoi(pos[3].c_str());
  fcg_box box{};
  box.celltype = FCG_HEX8;
  for (int k = 0; k < 3; ++k)
  {
    box.interval[k] = iv[k];
    box.lower[k] = 0.0;
    box.upper[k] = 1.0;
  }
  box.jitter = 0.1;
  box.jitter_seed = 20251015;
  const int local_rank = 0;
  StVK stvk;
  const StVK* params_stvk = &stvk;
  int failures = 0;
  for (int rank = 0; rank < nranks; ++rank)
  {
    Discretization dis;
    SparseMatrix stiff_obj;
    SparseMatrix* stiff = &stiff_obj;
    fcg_box_mesh* bm = nullptr;
    build_rank(box, rank, nranks, dis, stiff_obj, &bm);

    // ============ INTEGRATION.md, "Filling fcg_desc from a 4C discretization" ============
    // once after fill_complete() and the first stiff->complete() (graph is final)
    fcg_desc d{};
    d.abi_version = FCG_ABI_VERSION;
    d.celltype = FCG_HEX8;                       // Solid::shape()
    d.kinematics = FCG_LINEAR;                   // Inpar::Solid::KinemType
    d.youngs = params_stvk->youngs_;  d.poisson = params_stvk->poisson_ratio_;
    d.device = local_rank;
    const auto& colele = *dis.element_col_map();  const auto& colnode = *dis.node_col_map();
    std::vector<int32_t> ele_nodes, ele_gid, node_dof_col, node_dof_row, node_dof_kcol;
    std::vector<double> x;
    for (int e = 0; e < colele.NumMyElements(); ++e) {
      auto* ele = dis.l_col_element(e);
      ele_gid.push_back(ele->id());
      for (int a = 0; a < ele->num_node(); ++a) ele_nodes.push_back(colnode.LID(ele->node_ids()[a]));
    }
    const Epetra_Map& rowdofs = *dis.dof_row_map();
    const Epetra_Map& coldofs = *dis.dof_col_map();
    const Epetra_Map& kcol = stiff->epetra_matrix()->ColMap();
    for (int n = 0; n < colnode.NumMyElements(); ++n) {
      auto* node = dis.l_col_node(n);
      const int dof0 = dis.dof(node, 0);         // DofSet: 3*(gid - min gid), consecutive per node
      node_dof_col.push_back(coldofs.LID(dof0));
      node_dof_row.push_back(rowdofs.LID(dof0)); // -1 when not owned
      node_dof_kcol.push_back(kcol.LID(dof0));
      for (int k = 0; k < 3; ++k) x.push_back(node->x()[k]);
    }
    int nrows; int* rowptr32; int* cols; double* vals;          // Epetra_CrsMatrix after FillComplete
    stiff->epetra_matrix()->ExtractCrsDataPointers(rowptr32, cols, vals);
    std::vector<int64_t> rowptr(rowptr32, rowptr32 + rowdofs.NumMyElements() + 1);
    d.n_ele = ele_gid.size(); d.n_node = node_dof_col.size();
    d.n_rows = rowdofs.NumMyElements(); d.n_cols = coldofs.NumMyElements();
    d.ele_nodes = ele_nodes.data(); d.ele_gid = ele_gid.data(); d.node_x = x.data();
    d.node_dof_col = node_dof_col.data(); d.node_dof_row = node_dof_row.data();
    d.node_dof_kcol = node_dof_kcol.data(); d.rowptr = rowptr.data(); d.col_lid = cols;
    fcg_ctx* ctx = nullptr;
    if (fcg_create(&d, &ctx) != FCG_OK) {
      if (expect_no_device) { std::printf("rank %d: fcg_create without a device: %s (expected)\n", rank, fcg_last_error(nullptr)); fcg_box_mesh_destroy(bm); continue; }
      FOUR_C_THROW("{}", fcg_last_error(nullptr));
    }
    if (expect_no_device) { std::printf("rank %d: a device answered although none was expected\n", rank); return 2; }
    // the displacement state, imported into the column map (set_state) and the zeroed fint
    Vector dis_col_obj, fint_obj;
    Vector* dis_col = &dis_col_obj; Vector* fint = &fint_obj;
    dis_col->v.resize(d.n_cols);
    for (int n = 0; n < colnode.NumMyElements(); ++n)
      for (int k = 0; k < 3; ++k)
        dis_col->v[node_dof_col[n] + k] = 1e-3 * std::sin(3.0 * x[3 * n + k] + 2.0 * x[3 * n + (k + 1) % 3]);
    fint->v.assign(d.n_rows, 0.0);
    nrows = int(d.n_rows);

    // in Structure::evaluate_internal, instead of discret().evaluate(p, stiff, null, fint, null, null):
    int32_t bad = -1;
    int rc = fcg_evaluate(ctx, FCG_CALC_NLNSTIFF, dis_col->get_values(), fint->get_values(), vals, &bad);
    if (rc != FCG_OK) FOUR_C_THROW("element {}: {}", bad, fcg_last_error(ctx));
    // =====================================================================================

    // the oracle on the same rank (reference MPI semantics: column elements, owned rows)
    std::vector<int64_t> en64(ele_nodes.begin(), ele_nodes.end()), ngid(d.n_node);
    std::vector<int32_t> own(d.n_node);
    for (int64_t n = 0; n < d.n_node; ++n)
    {
      ngid[n] = dis.nodes[n].gid;
      own[n] = node_dof_row[n] >= 0 ? 0 : -1;
    }
    int max_gid = 0;
    for (int g : coldofs.gids) max_gid = std::max(max_gid, g);
    std::vector<int32_t> rl(max_gid + 1, -1), cl(max_gid + 1, -1);
    for (int i = 0; i < rowdofs.NumMyElements(); ++i) rl[rowdofs.gids[i]] = i;
    for (int i = 0; i < coldofs.NumMyElements(); ++i) cl[coldofs.gids[i]] = i;
    std::vector<double> Kr(rowptr[nrows], 0.0), fr(nrows, 0.0);
    orc_csr A{nrows, rowptr.data(), cols, Kr.data(), rl.data(), cl.data(), max_gid};
    int64_t bad_ele = -1;
    if (orc_discretization_evaluate(FCG_HEX8, FCG_LINEAR, d.youngs, d.poisson, d.n_ele, en64.data(),
            d.n_node, x.data(), ngid.data(), own.data(), 0, 1, dis_col->v.data(), &A, fr.data(),
            &bad_ele) != 0)
      FOUR_C_THROW("oracle failed");
    std::vector<double> K(vals, vals + rowptr[nrows]);
    const double ek = rel(K, Kr), ef = rel(fint->v, fr);
    std::printf("rank %d/%d: %lld elements, %d rows: fcg_evaluate |dK|/|K| %.2e |df|/|f| %.2e\n", rank,
        nranks, (long long)d.n_ele, nrows, ek, ef);
    failures += !(ek <= 1e-12 && ef <= 1e-10);

    // single rank: the tangent's linear solve through the native AMG object instead of Belos +
    // MueLu ("The linear solve on the device"), clamped x = 0 face
    if (nranks == 1)
    {
      const int64_t nnz = rowptr[nrows];
      std::vector<int32_t> dbc;
      std::vector<double> xb(size_t(nrows), 0.0), b(size_t(nrows), 0.0);
      for (int n = 0; n < colnode.NumMyElements(); ++n)
      {
        const int r0 = node_dof_row[n];
        if (r0 < 0) continue;
        for (int k = 0; k < 3; ++k) xb[size_t(r0 + k)] = x[3 * n + k];
        if (x[3 * n] == 0.0)
          for (int k = 0; k < 3; ++k) dbc.push_back(r0 + k);
        b[size_t(r0 + 2)] = -1e-3 * (1.0 + x[3 * n]);  // a distributed downward load
      }
      std::vector<double> xnode(xb.size());  // coordinates of block row b's node: rows 3b..3b+2
      for (int i = 0; i < nrows; ++i) xnode[size_t(i)] = xb[size_t(i)];
      void *dK = nullptr, *db = nullptr, *dx = nullptr, *drows = nullptr;
      fcg_device_alloc(0, nnz * 8, &dK);
      fcg_device_alloc(0, int64_t(nrows) * 8, &db);
      fcg_device_alloc(0, int64_t(nrows) * 8, &dx);
      fcg_device_alloc(0, int64_t(dbc.size()) * 4, &drows);
      fcg_memcpy_h2d(dK, vals, nnz * 8);
      fcg_memcpy_h2d(db, b.data(), int64_t(nrows) * 8);
      fcg_memcpy_h2d(drows, dbc.data(), int64_t(dbc.size()) * 4);
      rc = fcg_dirichlet_apply(ctx, int64_t(dbc.size()), static_cast<int32_t*>(drows),
          static_cast<double*>(dK), static_cast<double*>(db), nullptr, nullptr);
      if (rc != FCG_OK) FOUR_C_THROW("{}", fcg_last_error(ctx));
      fcg_amg* amg = nullptr;
      rc = fcg_amg_create(ctx, rowptr.data(), cols, xnode.data(), int64_t(dbc.size()), dbc.data(),
          nullptr, &amg);
      if (rc != FCG_OK) FOUR_C_THROW("{}", fcg_last_error(ctx));
      int iters = 0;
      double relres = 0.0;
      rc = fcg_amg_solve(amg, static_cast<double*>(dK), static_cast<double*>(db),
          static_cast<double*>(dx), 1e-8, 500, &iters, &relres, nullptr);
      if (rc != FCG_OK) FOUR_C_THROW("{}", fcg_amg_last_error(amg));
      std::vector<double> Kd(static_cast<size_t>(nnz)), bd(static_cast<size_t>(nrows)), xs(static_cast<size_t>(nrows));
      fcg_memcpy_d2h(Kd.data(), dK, nnz * 8);
      fcg_memcpy_d2h(bd.data(), db, int64_t(nrows) * 8);
      fcg_memcpy_d2h(xs.data(), dx, int64_t(nrows) * 8);
      double rr = 0.0, bb = 0.0;
      for (int i = 0; i < nrows; ++i)
      {
        double t = bd[size_t(i)];
        for (int64_t j = rowptr[i]; j < rowptr[i + 1]; ++j) t -= Kd[size_t(j)] * xs[size_t(cols[j])];
        rr += t * t;
        bb += bd[size_t(i)] * bd[size_t(i)];
      }
      const double truerel = std::sqrt(rr / bb);
      std::printf("  fcg_amg: %d levels, %d FCG iterations, reported |r|/|b| %.2e, recomputed %.2e\n",
          fcg_amg_levels(amg), iters, relres, truerel);
      failures += !(relres <= 1e-8 && truerel <= 2e-8 && fcg_amg_levels(amg) >= 2);
      fcg_amg_destroy(amg);
      for (void* pbuf : {dK, db, dx, drows}) fcg_device_free(pbuf);
    }

    // the C++ facade: Discretization::evaluate(params, stiff, null, fint, null, null) (+=) and
    // its zero()-fused variant on garbage-filled storage
    fcg_destroy(ctx);
    fourc_gpu::Discretization gdis(d);
    fourc_gpu::ParameterList p;
    p.set("action", "calc_struct_nlnstiff");
    std::vector<double> K2(K.size(), 0.0), f2(nrows, 0.0);
    fourc_gpu::SparseMatrixView Kv{K2.data(), int64_t(K2.size())};
    fourc_gpu::VectorView fv{f2.data(), nrows};
    gdis.set_state("displacement", fourc_gpu::VectorView{dis_col->v.data(), int64_t(d.n_cols)});
    gdis.evaluate(p, &Kv, nullptr, &fv, nullptr, nullptr);
    const double ek2 = rel(K2, Kr), ef2 = rel(f2, fr);
    std::fill(K2.begin(), K2.end(), 13.0);
    std::fill(f2.begin(), f2.end(), -7.0);
    gdis.evaluate_zeroed(p, &Kv, &fv);
    const double ek3 = rel(K2, Kr), ef3 = rel(f2, fr);
    std::printf("  facade evaluate %.2e %.2e, evaluate_zeroed %.2e %.2e\n", ek2, ef2, ek3, ef3);
    failures += !(ek2 <= 1e-12 && ef2 <= 1e-10 && ek3 <= 1e-12 && ef3 <= 1e-10);
    // FOUR_C_THROW's contract: unsupported requests throw
    bool threw = false;
    try
    {
      fourc_gpu::VectorView extra{f2.data(), nrows};
      gdis.evaluate(p, &Kv, nullptr, &fv, &extra, nullptr);
    }
    catch (const fourc_gpu::Exception& e)
    {
      threw = e.code() == FCG_ERR_ARG;
    }
    failures += !threw;
    fcg_box_mesh_destroy(bm);
  }
  std::printf(failures ? "FAIL (%d)\n" : "PASS\n", failures);
  return failures ? 1 : 0;
}
