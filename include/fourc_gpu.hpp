/*
 * fourc_gpu.hpp -- header-only C++17 facade over the C ABI (fourc_gpu.h) with the operator shape
 * of 4C's Core::FE::Discretization on this path, so that a C++ host calls it like the reference:
 *
 *   reference (4C_fem_discretization_evaluate.cpp:31-61, 4C_fem_discretization.cpp:503-548)
 *     discret.set_state(0, "displacement", disn);
 *     discret.evaluate(params, stiff, nullptr, fint, nullptr, nullptr);   // params "action"
 *   here
 *     fourc_gpu::Discretization dis(desc);                                // fcg_create
 *     dis.set_state("displacement", fourc_gpu::VectorView{u_col, n_cols});
 *     dis.evaluate(params, &K, nullptr, &fint, nullptr, nullptr);         // fcg_evaluate_host
 *
 * Errors follow FOUR_C_THROW: a non-zero status becomes fourc_gpu::Exception (code, element GID).
 * Semantics of the reference: `+=` into the caller's (zeroed) storage, owned rows only; with
 * evaluate_zeroed() the caller's SparseMatrix::zero() is fused (values only written).  Views with
 * device == true address HBM-resident storage and use fcg_evaluate_device.
 */
#ifndef FOURC_GPU_HPP
#define FOURC_GPU_HPP

#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>

#include "fourc_gpu.h"

namespace fourc_gpu {

class Exception : public std::runtime_error {
 public:
  Exception(int code, const std::string& what, int32_t element_gid = -1)
      : std::runtime_error(what), code_(code), element_gid_(element_gid)
  {
  }
  int code() const { return code_; }
  int32_t element_gid() const { return element_gid_; }

 private:
  int code_;
  int32_t element_gid_;
};

/* The entries Discretization::evaluate reads on this path: "action" =
 * "calc_struct_nlnstiff" | "calc_struct_internalforce" (the names Structure::evaluate_internal
 * sets, 4C_structure_new_model_evaluator_structure.cpp:2018-2021; enum ActionType,
 * 4C_legacy_enum_definitions_element_actions.hpp:19-75). */
class ParameterList {
 public:
  void set(const std::string& key, const std::string& value) { s_[key] = value; }
  bool is_parameter(const std::string& key) const { return s_.count(key) != 0; }
  const std::string& get(const std::string& key) const
  {
    auto it = s_.find(key);
    if (it == s_.end()) throw Exception(FCG_ERR_ARG, "parameter '" + key + "' not set");
    return it->second;
  }

 private:
  std::map<std::string, std::string> s_;
};

/* Epetra-shaped storage: the values of a filled Epetra_CrsMatrix in its CSR order
 * (ExtractCrsDataPointers) and the values of an Epetra_Vector. */
struct SparseMatrixView {
  double* values = nullptr;
  int64_t nnz = 0;
  bool device = false;
};
struct VectorView {
  double* values = nullptr;
  int64_t length = 0;
  bool device = false;
};

inline int action_of(const ParameterList& p)
{
  const std::string& a = p.get("action");
  if (a == "calc_struct_nlnstiff") return FCG_CALC_NLNSTIFF;
  if (a == "calc_struct_internalforce") return FCG_CALC_INTERNALFORCE;
  throw Exception(FCG_ERR_ARG, "action '" + a + "' is not on this path");
}

class Discretization {
 public:
  explicit Discretization(const fcg_desc& desc)
  {
    const int rc = fcg_create(&desc, &ctx_);
    if (rc != FCG_OK) throw Exception(rc, std::string("fcg_create: ") + fcg_last_error(nullptr));
    fcg_info info;
    fcg_get_info(ctx_, &info);
    n_rows_ = info.n_rows;
    n_cols_ = info.n_cols;
    nnz_ = info.nnz;
  }
  ~Discretization()
  {
    if (ctx_) fcg_destroy(ctx_);
  }
  Discretization(const Discretization&) = delete;
  Discretization& operator=(const Discretization&) = delete;
  Discretization(Discretization&& o) noexcept
      : ctx_(std::exchange(o.ctx_, nullptr)), state_(o.state_), n_rows_(o.n_rows_),
        n_cols_(o.n_cols_), nnz_(o.nnz_)
  {
  }

  /* Discretization::set_state(0, "displacement", vec): the DOF column vector (already imported
   * into the column map, or see fcg_halo_import for the device import). */
  void set_state(const std::string& name, const VectorView& col)
  {
    if (name != "displacement") throw Exception(FCG_ERR_ARG, "state '" + name + "' is not used");
    if (col.length != n_cols_) throw Exception(FCG_ERR_ARG, "state length != dof column map size");
    state_ = col;
  }

  /* Discretization::evaluate(params, systemmatrix1, systemmatrix2, systemvector1,
   * systemvector2, systemvector3): K += and f_int += on the owned rows.  This path fills no mass
   * matrix and no second / third vector: passing them throws, like an element that does not
   * implement the request. */
  void evaluate(const ParameterList& params, SparseMatrixView* systemmatrix1,
      SparseMatrixView* systemmatrix2, VectorView* systemvector1, VectorView* systemvector2,
      VectorView* systemvector3)
  {
    run(params, systemmatrix1, systemmatrix2, systemvector1, systemvector2, systemvector3,
        FCG_ACCUMULATE);
  }
  /* The same with SparseMatrix::zero() / fint->put_scalar(0) of the caller fused (4C zeroes both
   * right before the evaluate, Structure::reset, 4C_structure_new_model_evaluator_structure.cpp:
   * 136-159): the storage is only written. */
  void evaluate_zeroed(const ParameterList& params, SparseMatrixView* systemmatrix1,
      VectorView* systemvector1)
  {
    run(params, systemmatrix1, nullptr, systemvector1, nullptr, nullptr, FCG_OVERWRITE);
  }

  fcg_ctx* handle() const { return ctx_; }
  int64_t num_rows() const { return n_rows_; }
  int64_t num_cols() const { return n_cols_; }
  int64_t nnz() const { return nnz_; }

 private:
  void run(const ParameterList& params, SparseMatrixView* K, SparseMatrixView* M, VectorView* f,
      VectorView* v2, VectorView* v3, int mode)
  {
    const int action = action_of(params);
    if (M || v2 || v3)
      throw Exception(FCG_ERR_ARG, "only systemmatrix1 and systemvector1 are filled on this path");
    if (!state_.values && n_cols_) throw Exception(FCG_ERR_ARG, "set_state(\"displacement\") first");
    if (!f || f->length != n_rows_) throw Exception(FCG_ERR_ARG, "systemvector1 != dof row map size");
    if (action == FCG_CALC_NLNSTIFF && (!K || K->nnz != nnz_))
      throw Exception(FCG_ERR_ARG, "systemmatrix1 does not hold the graph's values");
    double* kv = (action == FCG_CALC_NLNSTIFF && K) ? K->values : nullptr;
    const bool dev = state_.device || f->device || (kv && K->device);
    if (dev && !(state_.device && f->device && (!kv || K->device)))
      throw Exception(FCG_ERR_ARG, "state, matrix and vector must all be host or all device");
    int32_t bad = -1;
    const int rc = dev ? fcg_evaluate_device(ctx_, action, mode, state_.values, f->values, kv,
                             nullptr, &bad)
                       : fcg_evaluate_host(ctx_, action, mode, state_.values, f->values, kv, &bad);
    if (rc != FCG_OK) throw Exception(rc, fcg_last_error(ctx_), bad);
  }

  fcg_ctx* ctx_ = nullptr;
  VectorView state_;
  int64_t n_rows_ = 0, n_cols_ = 0, nnz_ = 0;
};

}  // namespace fourc_gpu

#endif /* FOURC_GPU_HPP */
