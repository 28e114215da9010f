"""ctypes binding of libfourc_gpu (include/fourc_gpu.h) for tests, bench and Python hosts.

This is glue, not the product: every evaluation goes through the C ABI into the HIP kernels of
4c_amd/csrc.  There is no CPU fallback -- if the shared library is missing the import fails loudly.
Device buffers are torch tensors on `cuda:N` (PyTorch supplies device memory and streams only).
"""

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libfourc_gpu.so")
# diagnostics / A-B timing only: FCG_LIB=<name> loads lib/libfourc_gpu_<name>.so instead
# (diag = the phase-stamp build, make -C 4c_amd diag)
if os.environ.get("FCG_LIB"):
    LIB_PATH = os.path.join(PKG_DIR, "lib", "libfourc_gpu_%s.so" % os.environ["FCG_LIB"])

HEX8, HEX27 = 0, 1
LINEAR, TOTLAG = 0, 1
CALC_NLNSTIFF, CALC_INTERNALFORCE = 0, 1
ACCUMULATE, OVERWRITE = 0, 1
PATH_AUTO, PATH_GENERAL, PATH_STRUCTURED, PATH_COLORED, PATH_GATHER = 0, 1, 2, 3, 4
MAT_STVK, MAT_ELASTHYPER_COUPNEOHOOKE = 0, 1
TSI_STRUCT_FORCE, TSI_STIFFTEMP, TSI_THERMO_FINTCOND, TSI_COUPLTANG = 1, 2, 4, 8
TSI_ALL = 15
ABI_VERSION = 2

FCG_OK, FCG_ERR_NODAL_DETJ, FCG_ERR_SINGULAR, FCG_ERR_ARG, FCG_ERR_DEVICE = 0, 1, 2, 3, 4
STATUS = {0: "FCG_OK", 1: "FCG_ERR_NODAL_DETJ", 2: "FCG_ERR_SINGULAR", 3: "FCG_ERR_ARG",
          4: "FCG_ERR_DEVICE"}

_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_dp = ctypes.POINTER(ctypes.c_double)


class FcgDesc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("celltype", ctypes.c_int32),
                ("kinematics", ctypes.c_int32), ("device", ctypes.c_int32),
                ("youngs", ctypes.c_double), ("poisson", ctypes.c_double),
                ("n_ele", ctypes.c_int64), ("n_node", ctypes.c_int64), ("n_rows", ctypes.c_int64),
                ("n_cols", ctypes.c_int64), ("ele_nodes", _i32p), ("ele_gid", _i32p),
                ("node_x", _dp), ("node_dof_col", _i32p), ("node_dof_row", _i32p),
                ("node_dof_kcol", _i32p), ("rowptr", _i64p), ("col_lid", _i32p),
                ("ele_ijk", _i32p), ("path", ctypes.c_int32), ("material", ctypes.c_int32)]


class FcgBox(ctypes.Structure):
    _fields_ = [("celltype", ctypes.c_int32), ("interval", ctypes.c_int32 * 3),
                ("lower", ctypes.c_double * 3), ("upper", ctypes.c_double * 3),
                ("rotation", ctypes.c_double * 3), ("first_node_gid", ctypes.c_int64),
                ("jitter", ctypes.c_double), ("jitter_seed", ctypes.c_uint64)]


class FcgInfo(ctypes.Structure):
    _fields_ = [("n_ele", ctypes.c_int64), ("n_node", ctypes.c_int64), ("n_rows", ctypes.c_int64),
                ("n_cols", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("n_incidences", ctypes.c_int64), ("scratch_bytes", ctypes.c_int64),
                ("device_bytes", ctypes.c_int64), ("path", ctypes.c_int32),
                ("h27_slabs", ctypes.c_int32)]


class FcgImportPlan(ctypes.Structure):
    _fields_ = [("nranks", ctypes.c_int32), ("rank", ctypes.c_int32),
                ("n_rows", ctypes.c_int64), ("n_cols", ctypes.c_int64),
                ("n_same", ctypes.c_int64), ("n_permute", ctypes.c_int64),
                ("permute_from", _i32p), ("permute_to", _i32p),
                ("send_counts", _i64p), ("send_row", _i32p),
                ("recv_counts", _i64p), ("recv_col", _i32p)]


class FcgSharedPlan(ctypes.Structure):
    _fields_ = [("nranks", ctypes.c_int32), ("rank", ctypes.c_int32),
                ("n_global", ctypes.c_int64), ("n_local", ctypes.c_int64),
                ("n_owned", ctypes.c_int64), ("row", _i32p), ("pos", _i64p)]


# fcg_alltoallv_fn: (send_buf, send_counts, recv_buf, recv_counts, item_bytes, user) -> int
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _i64p, ctypes.c_void_p, _i64p,
                                ctypes.c_int64, ctypes.c_void_p)
FCG_OP_SUM, FCG_OP_MAX = 0, 1
BOX_GHOSTED, BOX_STRICT = 0, 1
# fcg_transport (distributed solve): import (user, d_x_row, d_x_col, stream), all-reduce (user,
# d_vals, n, stream), both -> int
IMPORT_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_void_p)
# (user, d_send, send_counts[nranks], d_recv, recv_counts[nranks], stream): MPI_Alltoallv of doubles
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p,
                               ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p)


class FcgTransport(ctypes.Structure):
    _fields_ = [("import_fn", IMPORT_FN), ("allreduce_fn", ALLREDUCE_FN), ("user", ctypes.c_void_p),
                ("rank", ctypes.c_int32), ("nranks", ctypes.c_int32), ("exchange_fn", EXCHANGE_FN)]


class FcgRcclPair(ctypes.Structure):
    _fields_ = [("comm", ctypes.c_void_p), ("halo", ctypes.c_void_p)]


class FcgTsiDesc(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("celltype", ctypes.c_int32),
                ("device", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("youngs", ctypes.c_double), ("poisson", ctypes.c_double),
                ("thexpans", ctypes.c_double), ("inittemp", ctypes.c_double),
                ("conduct", ctypes.c_double),
                ("n_ele", ctypes.c_int64), ("n_node", ctypes.c_int64),
                ("n_rows_s", ctypes.c_int64), ("n_cols_s", ctypes.c_int64),
                ("n_rows_t", ctypes.c_int64), ("n_cols_t", ctypes.c_int64),
                ("ele_nodes", _i32p), ("ele_gid", _i32p), ("node_x", _dp),
                ("node_dof_col_s", _i32p), ("node_dof_row_s", _i32p),
                ("node_dof_col_t", _i32p), ("node_dof_row_t", _i32p),
                ("rowptr_st", _i64p), ("col_st", _i32p),
                ("rowptr_ts", _i64p), ("col_ts", _i32p),
                ("rowptr_tt", _i64p), ("col_tt", _i32p)]


# every symbol declared in include/fourc_gpu.h
class FcgAmgOptions(ctypes.Structure):
    """fcg_amg_options (include/fourc_gpu.h)."""
    _fields_ = [("nu", ctypes.c_int32), ("max_levels", ctypes.c_int32),
                ("coarse_max", ctypes.c_int64), ("coarse_max_iter", ctypes.c_int32),
                ("coarse_rtol", ctypes.c_double), ("omega", ctypes.c_double),
                ("ratio", ctypes.c_double), ("boost", ctypes.c_double)]


EXPORTS = ["fcg_create", "fcg_destroy", "fcg_last_error", "fcg_evaluate", "fcg_evaluate_device",
           "fcg_device_alloc", "fcg_device_free", "fcg_memcpy_h2d", "fcg_memcpy_d2h",
           "fcg_memset_device", "fcg_set_timing", "fcg_get_timing", "fcg_get_info",
           "fcg_get_diagnostics", "fcg_get_create_phases", "fcg_measure_peaks", "fcg_measure_hbm", "fcg_spmv", "fcg_dirichlet_apply",
           "fcg_pcg_solve", "fcg_spmv_f32", "fcg_tangent_apply", "fcg_box_stencil_apply", "fcg_box_transfer", "fcg_block_jacobi_setup", "fcg_block_jacobi_apply", "fcg_chebyshev_step", "fcg_node_transfer",
           "fcg_neumann_surface", "fcg_neumann_volume",
           "fcg_graph_build_device", "fcg_get_graph",
           "fcg_tsi_create", "fcg_tsi_destroy", "fcg_tsi_last_error", "fcg_tsi_evaluate_device",
           "fcg_tsi_evaluate_fused",
           "fcg_box_mesh_create", "fcg_box_mesh_destroy", "fcg_box_mesh_desc", "fcg_box_mesh_maps",
           "fcg_box_mesh_counts", "fcg_box_mesh_create_ex", "fcg_box_mesh_owned_rows",
           "fcg_comm_unique_id", "fcg_comm_create", "fcg_comm_destroy", "fcg_comm_size", "fcg_comm_rank", "fcg_comm_allreduce",
           "fcg_comm_alltoallv", "fcg_import_plan_build", "fcg_plan_free", "fcg_halo_create",
           "fcg_halo_destroy", "fcg_halo_import", "fcg_halo_pack", "fcg_halo_unpack",
           "fcg_shared_plan_build", "fcg_shared_create", "fcg_shared_destroy", "fcg_shared_reduce",
           "fcg_shared_pack", "fcg_shared_unpack", "fcg_norm2", "fcg_set_async", "fcg_check_error",
           "fcg_evaluate_host",
           "fcg_amg_aggregate", "fcg_amg_tentative", "fcg_bsr_symbolic", "fcg_bsr_transpose_pattern",
           "fcg_bsr_spmv", "fcg_bsr_spgemm", "fcg_bsr_product_plan", "fcg_bsr_spgemm_planned", "fcg_bsr_transpose_values", "fcg_bsr_from_node_csr",
           "fcg_bsr_block_jacobi_setup", "fcg_bsr_block_jacobi_apply", "fcg_amg_smooth_prolongator",
           "fcg_bsr_to_dense", "fcg_amg_default_options", "fcg_amg_create", "fcg_amg_solve",
           "fcg_amg_levels", "fcg_amg_level_info", "fcg_amg_setup_ms", "fcg_amg_stats", "fcg_amg_last_error",
           "fcg_amg_destroy", "fcg_amg_setup", "fcg_amg_iterate", "fcg_amg_apply",
           "fcg_amg_coupled_levels", "fcg_amg_coupled_stats", "fcg_comm_exchange_device",
           "fcg_transport_rccl", "fcg_dfcg_solve"]

_lib = None
FUNCT_FN = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_int, _dp, ctypes.c_double, ctypes.c_void_p)


class FcgError(RuntimeError):
    def __init__(self, code, msg, bad_ele_gid=-1):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code
        self.bad_ele_gid = bad_ele_gid


def lib():
    """Load libfourc_gpu.so (built by `make -C 4c_amd`); raise if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make -C 4c_amd` (no CPU fallback exists)")
    # One HIP runtime per process: when torch supplies the device buffers, its libamdhip64 must be
    # the one the library binds to, so torch is loaded first (same soname -> shared).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    L.fcg_create.argtypes = [ctypes.POINTER(FcgDesc), ctypes.POINTER(vp)]
    L.fcg_destroy.argtypes = [vp]
    L.fcg_last_error.argtypes = [vp]
    L.fcg_last_error.restype = ctypes.c_char_p
    L.fcg_evaluate.argtypes = [vp, ctypes.c_int, _dp, _dp, _dp, _i32p]
    L.fcg_evaluate_device.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, _i32p]
    L.fcg_device_alloc.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.POINTER(vp)]
    L.fcg_device_free.argtypes = [vp]
    L.fcg_memcpy_h2d.argtypes = [vp, vp, ctypes.c_int64]
    L.fcg_memcpy_d2h.argtypes = [vp, vp, ctypes.c_int64]
    L.fcg_memset_device.argtypes = [vp, ctypes.c_int, ctypes.c_int64]
    L.fcg_set_timing.argtypes = [vp, ctypes.c_int]
    L.fcg_get_timing.argtypes = [vp, _dp, _dp]
    L.fcg_get_info.argtypes = [vp, ctypes.POINTER(FcgInfo)]
    L.fcg_get_diagnostics.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    if hasattr(L, "fcg_get_create_phases"):  # absent from older A/B builds (FCG_LIB)
        L.fcg_get_create_phases.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    L.fcg_spmv.argtypes = [vp, vp, vp, vp, vp]
    L.fcg_measure_peaks.argtypes = [ctypes.c_int, _dp, _dp, _dp]
    L.fcg_measure_hbm.argtypes = [ctypes.c_int, _dp, _dp]
    L.fcg_dirichlet_apply.argtypes = [vp, ctypes.c_int64, vp, vp, vp, vp, vp]
    L.fcg_pcg_solve.argtypes = [vp, vp, vp, vp, ctypes.c_double, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_int), _dp, vp]
    L.fcg_spmv_f32.argtypes = [vp, vp, vp, vp, vp]
    L.fcg_tangent_apply.argtypes = [vp, vp, vp, vp, vp]
    L.fcg_box_stencil_apply.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp, vp]
    L.fcg_box_transfer.argtypes = [ctypes.c_int] * 8 + [vp, vp, vp, vp, vp, ctypes.c_int, vp]
    L.fcg_block_jacobi_setup.argtypes = [vp, vp, vp, vp]
    L.fcg_block_jacobi_apply.argtypes = [vp, vp, vp, vp, ctypes.c_double, ctypes.c_int, vp]
    L.fcg_chebyshev_step.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_double, ctypes.c_double, ctypes.c_int, vp]
    L.fcg_node_transfer.argtypes = [ctypes.c_int, ctypes.c_int64, vp, vp, vp, vp, vp, vp,
                                    ctypes.c_int, vp]
    neu = [ctypes.c_int, ctypes.c_int64, _i32p, _dp, _i32p, _i32p, _dp, _i32p, FUNCT_FN,
           ctypes.c_void_p, ctypes.c_double, _dp]
    L.fcg_neumann_surface.argtypes = neu
    L.fcg_neumann_volume.argtypes = neu
    L.fcg_box_mesh_create.argtypes = [ctypes.POINTER(FcgBox), ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(vp)]
    L.fcg_box_mesh_destroy.argtypes = [vp]
    L.fcg_box_mesh_desc.argtypes = [vp, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_int, ctypes.POINTER(FcgDesc)]
    L.fcg_box_mesh_maps.argtypes = [vp, ctypes.POINTER(_i32p), ctypes.POINTER(_i32p),
                                    ctypes.POINTER(_i64p), ctypes.POINTER(_i32p)]
    L.fcg_box_mesh_counts.argtypes = [vp, _i64p, _i64p]
    L.fcg_box_mesh_create_ex.argtypes = [ctypes.POINTER(FcgBox), ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(vp)]
    L.fcg_box_mesh_owned_rows.argtypes = [vp, _i64p]
    L.fcg_comm_unique_id.argtypes = [vp]
    L.fcg_comm_create.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L.fcg_comm_destroy.argtypes = [vp]
    L.fcg_comm_size.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.fcg_comm_rank.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.fcg_comm_allreduce.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int, vp]
    L.fcg_comm_alltoallv.argtypes = [vp, _i64p, vp, _i64p, ctypes.c_int64, vp]
    L.fcg_import_plan_build.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, _i32p,
                                        ctypes.c_int64, _i32p, _i32p, ALLTOALLV_FN, vp,
                                        ctypes.POINTER(FcgImportPlan), ctypes.POINTER(vp)]
    L.fcg_plan_free.argtypes = [vp]
    L.fcg_plan_free.restype = None
    L.fcg_halo_create.argtypes = [ctypes.POINTER(FcgImportPlan), ctypes.c_int, ctypes.POINTER(vp)]
    L.fcg_halo_destroy.argtypes = [vp]
    L.fcg_halo_import.argtypes = [vp, vp, vp, vp, vp]
    L.fcg_halo_pack.argtypes = [vp, vp, vp, vp, vp]
    L.fcg_halo_unpack.argtypes = [vp, vp, vp, vp]
    L.fcg_shared_plan_build.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, _i32p,
                                        ctypes.c_int64, _i32p, _i32p, ALLTOALLV_FN, vp,
                                        ctypes.POINTER(FcgSharedPlan), ctypes.POINTER(vp)]
    L.fcg_shared_create.argtypes = [ctypes.POINTER(FcgSharedPlan), ctypes.c_int, ctypes.POINTER(vp)]
    L.fcg_shared_destroy.argtypes = [vp]
    L.fcg_shared_reduce.argtypes = [vp, vp, vp, vp]
    L.fcg_shared_pack.argtypes = [vp, vp, vp, vp]
    L.fcg_shared_unpack.argtypes = [vp, vp, vp, vp]
    L.fcg_norm2.argtypes = [vp, vp, ctypes.c_int64, vp, _dp]
    L.fcg_set_async.argtypes = [vp, ctypes.c_int]
    L.fcg_check_error.argtypes = [vp, _i32p]
    L.fcg_evaluate_host.argtypes = [vp, ctypes.c_int, ctypes.c_int, _dp, _dp, _dp, _i32p]
    L.fcg_graph_build_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, vp,
                                         ctypes.c_int64, vp, vp, ctypes.c_int64, vp, vp,
                                         ctypes.c_int64, _i64p, vp]
    L.fcg_get_graph.argtypes = [vp, _i64p, _i32p, ctypes.c_int64, _i64p]
    L.fcg_tsi_create.argtypes = [ctypes.POINTER(FcgTsiDesc), ctypes.POINTER(vp)]
    L.fcg_tsi_destroy.argtypes = [vp]
    L.fcg_tsi_last_error.argtypes = [vp]
    L.fcg_tsi_last_error.restype = ctypes.c_char_p
    L.fcg_tsi_evaluate_device.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_double,
                                          ctypes.c_double, vp, vp, vp, vp, vp, vp, _i32p]
    L.fcg_tsi_evaluate_fused.argtypes = [vp, vp, ctypes.c_int, vp, vp, vp, ctypes.c_double,
                                         ctypes.c_double, vp, vp, vp, vp, vp, vp, vp, _i32p]
    i64, c_int, c_dbl = ctypes.c_int64, ctypes.c_int, ctypes.c_double
    L.fcg_amg_aggregate.argtypes = [i64, vp, vp, vp, vp]
    L.fcg_amg_aggregate.restype = i64
    L.fcg_amg_tentative.argtypes = [i64, c_int, vp, vp, i64, vp, vp, vp]
    L.fcg_bsr_symbolic.argtypes = [i64, vp, vp, vp, vp, i64, vp, vp]
    L.fcg_bsr_symbolic.restype = i64
    L.fcg_bsr_transpose_pattern.argtypes = [i64, i64, vp, vp, vp, vp, vp]
    L.fcg_bsr_spmv.argtypes = [c_int, c_int, c_int, i64, vp, vp, vp, vp, vp, c_dbl, c_int, vp]
    L.fcg_bsr_spgemm.argtypes = [c_int, c_int, c_int, c_int, i64, vp, vp, vp, vp, vp, vp, vp, vp,
                                 vp, vp]
    L.fcg_bsr_product_plan.argtypes = [i64, vp, vp, vp, vp, vp, vp, i64, vp, vp, vp]
    L.fcg_bsr_product_plan.restype = i64
    L.fcg_bsr_spgemm_planned.argtypes = [c_int, c_int, c_int, c_int, i64, vp, vp, vp, vp, vp, vp, vp, vp]
    L.fcg_bsr_transpose_values.argtypes = [c_int, c_int, c_int, i64, vp, vp, vp, vp]
    L.fcg_bsr_from_node_csr.argtypes = [c_int, i64, vp, vp, vp, vp, vp]
    L.fcg_bsr_block_jacobi_setup.argtypes = [c_int, c_int, i64, vp, vp, vp, vp, vp, vp]
    L.fcg_bsr_block_jacobi_apply.argtypes = [c_int, c_int, i64, vp, vp, vp, c_dbl, c_int, vp]
    L.fcg_amg_smooth_prolongator.argtypes = [c_int, c_int, i64, vp, vp, vp, vp, vp, vp, c_dbl, vp,
                                             vp]
    L.fcg_bsr_to_dense.argtypes = [c_int, c_int, i64, vp, vp, vp, vp, vp]
    L.fcg_amg_default_options.argtypes = [ctypes.POINTER(FcgAmgOptions)]
    L.fcg_amg_default_options.restype = None
    L.fcg_amg_create.argtypes = [vp, vp, vp, vp, i64, vp, ctypes.POINTER(FcgAmgOptions),
                                 ctypes.POINTER(vp)]
    L.fcg_amg_solve.argtypes = [vp, vp, vp, vp, c_dbl, c_int, ctypes.POINTER(c_int), _dp, vp]
    L.fcg_amg_setup.argtypes = [vp, vp, vp]
    L.fcg_amg_iterate.argtypes = [vp, vp, vp, vp, c_dbl, c_int, ctypes.POINTER(c_int), _dp, vp]
    L.fcg_amg_levels.argtypes = [vp]
    L.fcg_amg_level_info.argtypes = [vp, c_int, _i64p, _i64p, _dp]
    L.fcg_amg_setup_ms.argtypes = [vp]
    L.fcg_amg_setup_ms.restype = c_dbl
    L.fcg_amg_stats.argtypes = [vp, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]
    L.fcg_amg_last_error.argtypes = [vp]
    L.fcg_amg_last_error.restype = ctypes.c_char_p
    L.fcg_amg_destroy.argtypes = [vp]
    L.fcg_amg_apply.argtypes = [vp, vp, vp, vp, vp]
    L.fcg_amg_coupled_levels.argtypes = [vp]
    if hasattr(L, "fcg_amg_coupled_stats"):  # absent from older A/B builds (FCG_LIB)
        L.fcg_amg_coupled_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_int64), c_int]
    L.fcg_transport_rccl.argtypes = [ctypes.POINTER(FcgRcclPair), ctypes.POINTER(FcgTransport)]
    L.fcg_dfcg_solve.argtypes = [vp, vp, ctypes.POINTER(FcgTransport), vp, vp, vp, c_dbl, c_int, vp,
                                 ctypes.POINTER(c_int), _dp]
    _lib = L
    return L


def _torch_stream(stream, device=None):
    """The HIP stream of a library call on torch tensors: the given torch stream, else torch's
    current stream of `device` (the context's device, not whichever device is current) -- never
    the context's own stream, which is not ordered with the torch work that produced or consumes
    the buffers."""
    import torch
    if stream is None:
        stream = torch.cuda.current_stream(device)
    return ctypes.c_void_p(stream.cuda_stream)


def _np_ptr(a, t):
    return a.ctypes.data_as(t)


def lattice_ijk(ele_nodes):
    """Element lattice positions (ex, ey, ez) of a hex8 mesh whose elements stack like a
    GridGenerator box: neighbours share whole faces in 4C node order (+x: nodes 1 2 6 5 of the
    element are 0 3 7 4 of the neighbour; +y: 3 2 6 7 -> 0 1 5 4; +z: 4 5 6 7 -> 0 1 2 3).
    Returns an int32 [n_ele][3] array (minimum 0), or None if the mesh is not such a lattice --
    the fcg_desc.ele_ijk hint, which fcg_create verifies again."""
    en = np.asarray(ele_nodes, dtype=np.int64).reshape(-1, 8)
    n = len(en)
    if n == 0:
        return None
    dirs = (((1, 2, 6, 5), (0, 3, 7, 4), (1, 0, 0)), ((3, 2, 6, 7), (0, 1, 5, 4), (0, 1, 0)),
            ((4, 5, 6, 7), (0, 1, 2, 3), (0, 0, 1)))
    maps = []
    for hi, lo, _ in dirs:
        mhi = {tuple(r): e for e, r in enumerate(en[:, list(hi)].tolist())}
        mlo = {tuple(r): e for e, r in enumerate(en[:, list(lo)].tolist())}
        maps.append((mhi, mlo))
    ijk = np.full((n, 3), np.iinfo(np.int64).min, dtype=np.int64)
    ijk[0] = 0
    stack = [0]
    while stack:
        e = stack.pop()
        for (hi, lo, off), (mhi, mlo) in zip(dirs, maps):
            for nb, sgn in ((mlo.get(tuple(en[e, list(hi)].tolist())), 1),
                            (mhi.get(tuple(en[e, list(lo)].tolist())), -1)):
                if nb is None:
                    continue
                want = ijk[e] + sgn * np.asarray(off)
                if ijk[nb, 0] == np.iinfo(np.int64).min:
                    ijk[nb] = want
                    stack.append(nb)
                elif not np.array_equal(ijk[nb], want):
                    return None
    if (ijk[:, 0] == np.iinfo(np.int64).min).any():
        return None
    ijk -= ijk.min(axis=0)
    if len(np.unique(ijk, axis=0)) != n or ijk.max() >= 2 ** 31:
        return None
    return np.ascontiguousarray(ijk, dtype=np.int32)


class Discretization:
    """Arrays of one rank's discretization as 4C holds them after FillComplete (the fcg_desc
    contents), for meshes that are not GridGenerator boxes -- e.g. the reference's input files."""

    def __init__(self, celltype, ele_nodes, node_x, node_dof_col, node_dof_row, rowptr, col_lid,
                 n_cols=None, ele_gid=None):
        self.celltype = celltype
        self.npe = 8 if celltype == HEX8 else 27
        self.ele_nodes = np.ascontiguousarray(ele_nodes, dtype=np.int32).reshape(-1, self.npe)
        self.node_x = np.ascontiguousarray(node_x, dtype=np.float64).reshape(-1, 3)
        self.node_dof_col = np.ascontiguousarray(node_dof_col, dtype=np.int32)
        self.node_dof_row = np.ascontiguousarray(node_dof_row, dtype=np.int32)
        self.rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        self.col_lid = np.ascontiguousarray(col_lid, dtype=np.int32)
        self.ele_gid = (np.ascontiguousarray(ele_gid, dtype=np.int32) if ele_gid is not None
                        else np.arange(len(self.ele_nodes), dtype=np.int32))
        self.n_ele, self.n_node = len(self.ele_nodes), len(self.node_x)
        self.n_rows = len(self.rowptr) - 1
        self.n_cols = int(n_cols) if n_cols is not None else self.n_rows
        self.nnz = int(self.rowptr[-1])
        self.ele_ijk = None  # optional structured-lattice hint (lattice_ijk)

    @staticmethod
    def from_elements(celltype, ele_nodes, node_x, lattice=False):
        """Single-rank discretization: DOF LID = 3 * node + d, CSR graph of the element couplings.
        lattice=True attaches the structured-lattice hint (hex8 meshes stacked like a box)."""
        en = np.asarray(ele_nodes, dtype=np.int64)
        n_node = len(node_x)
        nbr = [set() for _ in range(n_node)]
        for el in en:
            for a in el:
                nbr[a].update(int(b) for b in el)
        rows, cols = [0], []
        for a in range(n_node):
            c = sorted(nbr[a])
            cd = [3 * b + d for b in c for d in range(3)]
            for _ in range(3):
                cols.extend(cd)
                rows.append(len(cols))
        dof = 3 * np.arange(n_node, dtype=np.int32)
        dis = Discretization(celltype, en, node_x, dof, dof, np.array(rows), np.array(cols))
        if lattice and celltype == HEX8:
            dis.ele_ijk = lattice_ijk(en)
        return dis

    def desc(self, kinematics, youngs, poisson, device=0, path=PATH_AUTO, material=MAT_STVK):
        d = FcgDesc()
        d.abi_version = ABI_VERSION
        d.celltype = self.celltype
        d.kinematics = kinematics
        d.device = device
        d.youngs = youngs
        d.poisson = poisson
        d.n_ele, d.n_node, d.n_rows, d.n_cols = self.n_ele, self.n_node, self.n_rows, self.n_cols
        d.ele_nodes = _np_ptr(self.ele_nodes, _i32p)
        d.ele_gid = _np_ptr(self.ele_gid, _i32p)
        d.node_x = _np_ptr(self.node_x, _dp)
        d.node_dof_col = _np_ptr(self.node_dof_col, _i32p)
        d.node_dof_row = _np_ptr(self.node_dof_row, _i32p)
        d.node_dof_kcol = None
        d.rowptr = _np_ptr(self.rowptr, _i64p)
        d.col_lid = _np_ptr(self.col_lid, _i32p)
        d.ele_ijk = (_np_ptr(self.ele_ijk, _i32p)
                     if self.ele_ijk is not None and path != PATH_GENERAL else None)
        d.path = path
        d.material = material
        return d

    @staticmethod
    def renumbered(box, seed=0):
        """A single-rank box mesh as an input-file mesh would arrive: random node and element
        numbering (DOF LID = 3 * node), no lattice hint; same geometry, graph and element
        orientation.  Vectorised, for benchmark-sized meshes."""
        assert box.n_rows == box.n_cols and np.array_equal(box.node_dof_col, 3 * np.arange(box.n_node))
        rng = np.random.default_rng(seed)
        nn = box.n_node
        perm = rng.permutation(nn)                 # new number of old node
        inv = np.argsort(perm)                     # old node of new number
        en = perm[box.ele_nodes][rng.permutation(box.n_ele)]
        X = np.empty_like(box.node_x)
        X[perm] = box.node_x
        rp = box.rowptr
        cnt = (rp[1::3][:nn] - rp[0::3][:nn]) // 3  # neighbour nodes of each old node
        cnt_new = cnt[inv]
        start = np.concatenate([[0], np.cumsum(cnt_new)])
        owner = np.repeat(np.arange(nn), cnt_new)
        k = np.arange(start[-1]) - start[owner]
        nb = perm[box.col_lid[rp[3 * inv[owner]] + 3 * k] // 3]
        nb = nb[np.lexsort((nb, owner))]
        rowlen = np.repeat(3 * cnt_new, 3)
        rowptr = np.concatenate([[0], np.cumsum(rowlen)]).astype(np.int64)
        row = np.repeat(np.arange(3 * nn), rowlen)
        off = np.arange(rowptr[-1]) - rowptr[row]
        col = (3 * nb[start[row // 3] + off // 3] + off % 3).astype(np.int32)
        dof = 3 * np.arange(nn, dtype=np.int32)
        dis = Discretization(box.celltype, en, X, dof, dof, rowptr, col)
        dis.node_perm = perm  # new number of every box node (DOF 3 * perm[old] + d)
        return dis


def _neumann(entry, celltype, conn, node_x, node_dof_row, onoff, val, funct, fn, time, fext):
    """fcg_neumann_surface / fcg_neumann_volume into the numpy vector `fext` (+=)."""
    conn = np.ascontiguousarray(conn, dtype=np.int32)
    node_x = np.ascontiguousarray(node_x, dtype=np.float64)
    node_dof_row = np.ascontiguousarray(node_dof_row, dtype=np.int32)
    oo = np.ascontiguousarray(onoff, dtype=np.int32)
    vv = np.ascontiguousarray(val, dtype=np.float64)
    ff = np.ascontiguousarray(funct if funct is not None else [0, 0, 0], dtype=np.int32)
    err = []

    def cb(fid, x, t, _user):
        try:
            return float(fn(fid, (x[0], x[1], x[2]), t))
        except Exception as e:  # surfaced after the call
            err.append(e)
            return 0.0

    cfn = FUNCT_FN(cb) if fn is not None else FUNCT_FN()
    n = conn.shape[0]
    rc = getattr(lib(), entry)(celltype, n, _np_ptr(conn, _i32p), _np_ptr(node_x, _dp),
                               _np_ptr(node_dof_row, _i32p), _np_ptr(oo, _i32p), _np_ptr(vv, _dp),
                               _np_ptr(ff, _i32p), cfn, None, float(time), _np_ptr(fext, _dp))
    if err:
        raise err[0]
    if rc != 0:
        raise FcgError(rc, entry + " failed")


def neumann_surface(celltype, face_nodes, node_x, node_dof_row, onoff, val, fext, funct=None,
                    fn=None, time=1.0):
    _neumann("fcg_neumann_surface", celltype, face_nodes, node_x, node_dof_row, onoff, val, funct,
             fn, time, fext)


def neumann_volume(celltype, ele_nodes, node_x, node_dof_row, onoff, val, fext, funct=None,
                   fn=None, time=1.0):
    _neumann("fcg_neumann_volume", celltype, ele_nodes, node_x, node_dof_row, onoff, val, funct,
             fn, time, fext)


def _tensor_ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class _NativeBoxMesh:
    """Owner of an fcg_box_mesh: destroyed when the last numpy view of its arrays goes."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        if self.h:
            try:
                lib().fcg_box_mesh_destroy(self.h)
            except Exception:  # noqa: BLE001 - interpreter shutdown: the process frees it anyway
                pass
            self.h = None


class BoxMesh:
    """One rank of a GridGenerator box (the fcg_box_mesh_* builder), as numpy views."""

    def __init__(self, celltype, interval, lower=(0.0, 0.0, 0.0), upper=(1.0, 1.0, 1.0),
                 rotation=(0.0, 0.0, 0.0), first_node_gid=0, jitter=0.0, seed=20251015,
                 rank=0, nranks=1, strict=False):
        """strict=True: FCG_BOX_STRICT (row elements only, extended rows for the non-owned
        nodes they touch after the n_owned_rows owned rows)."""
        L = lib()
        box = FcgBox()
        box.celltype = celltype
        for d in range(3):
            box.interval[d] = int(interval[d])
            box.lower[d] = float(lower[d])
            box.upper[d] = float(upper[d])
            box.rotation[d] = float(rotation[d])
        box.first_node_gid = int(first_node_gid)
        box.jitter = float(jitter)
        box.jitter_seed = int(seed)
        self.box = box
        self.celltype = celltype
        self.npe = 8 if celltype == HEX8 else 27
        self.rank, self.nranks = rank, nranks
        self.strict = bool(strict)
        h = ctypes.c_void_p()
        rc = L.fcg_box_mesh_create_ex(ctypes.byref(box), rank, nranks,
                                      BOX_STRICT if strict else BOX_GHOSTED, ctypes.byref(h))
        if rc != 0:
            raise FcgError(rc, "fcg_box_mesh_create failed")
        self._h = h
        d = FcgDesc()
        L.fcg_box_mesh_desc(h, LINEAR, 1.0, 0.0, 0, ctypes.byref(d))
        self.n_ele, self.n_node = d.n_ele, d.n_node
        self.n_rows, self.n_cols = d.n_rows, d.n_cols

        # zero-copy views of the builder's arrays; the native mesh is released when the last
        # view is (a 1M-hex27 box holds 18.5 GB of column indices: no second copy)
        keeper = _NativeBoxMesh(h)
        ctype_of = {np.int32: ctypes.c_int32, np.int64: ctypes.c_int64, np.float64: ctypes.c_double}

        def view(p, n, dt):
            if n == 0:
                return np.zeros(0, dtype=dt)
            buf = (ctype_of[dt] * n).from_address(ctypes.cast(p, ctypes.c_void_p).value)
            buf._keep = keeper
            return np.frombuffer(buf, dtype=dt)

        self.ele_nodes = view(d.ele_nodes, d.n_ele * self.npe, np.int32).reshape(-1, self.npe)
        self.ele_gid = view(d.ele_gid, d.n_ele, np.int32)
        self.ele_ijk = view(d.ele_ijk, d.n_ele * 3, np.int32).reshape(-1, 3)
        self.node_x = view(d.node_x, d.n_node * 3, np.float64).reshape(-1, 3)
        self.node_dof_col = view(d.node_dof_col, d.n_node, np.int32)
        self.node_dof_row = view(d.node_dof_row, d.n_node, np.int32)
        self.rowptr = view(d.rowptr, d.n_rows + 1, np.int64)
        self.nnz = int(self.rowptr[-1]) if d.n_rows else 0
        self.col_lid = view(d.col_lid, self.nnz, np.int32)
        rg, cg, ng, no = _i32p(), _i32p(), _i64p(), _i32p()
        L.fcg_box_mesh_maps(h, ctypes.byref(rg), ctypes.byref(cg), ctypes.byref(ng), ctypes.byref(no))
        self.row_gid = view(rg, d.n_rows, np.int32)
        self.col_gid = view(cg, d.n_cols, np.int32)
        self.node_gid = view(ng, d.n_node, np.int64)
        self.node_owner = view(no, d.n_node, np.int32)
        ng_, nr_ = ctypes.c_int64(), ctypes.c_int64()
        L.fcg_box_mesh_counts(h, ctypes.byref(ng_), ctypes.byref(nr_))
        self.n_ele_global, self.n_ele_row = ng_.value, nr_.value
        no_ = ctypes.c_int64()
        L.fcg_box_mesh_owned_rows(h, ctypes.byref(no_))
        self.n_owned_rows = no_.value
        self._h = None  # owned by the views' keeper

    def desc(self, kinematics, youngs, poisson, device=0, path=PATH_AUTO, material=MAT_STVK):
        d = FcgDesc()
        d.abi_version = ABI_VERSION
        d.celltype = self.celltype
        d.kinematics = kinematics
        d.device = device
        d.youngs = youngs
        d.poisson = poisson
        d.n_ele, d.n_node, d.n_rows, d.n_cols = self.n_ele, self.n_node, self.n_rows, self.n_cols
        d.ele_nodes = _np_ptr(self.ele_nodes, _i32p)
        d.ele_gid = _np_ptr(self.ele_gid, _i32p)
        d.node_x = _np_ptr(self.node_x, _dp)
        d.node_dof_col = _np_ptr(self.node_dof_col, _i32p)
        d.node_dof_row = _np_ptr(self.node_dof_row, _i32p)
        d.node_dof_kcol = None
        d.rowptr = _np_ptr(self.rowptr, _i64p)
        d.col_lid = _np_ptr(self.col_lid, _i32p)
        d.ele_ijk = _np_ptr(self.ele_ijk, _i32p) if path != PATH_GENERAL else None
        d.path = path
        d.material = material
        return d

    def node_displacement(self, amplitude):
        """Synthetic state u(X) = A (sin2piX cospiY, sinpiY cos2piZ, sin2piZ cospiX)."""
        X = self.node_x
        u = np.empty_like(X)
        u[:, 0] = np.sin(2 * np.pi * X[:, 0]) * np.cos(np.pi * X[:, 1])
        u[:, 1] = np.sin(np.pi * X[:, 1]) * np.cos(2 * np.pi * X[:, 2])
        u[:, 2] = np.sin(2 * np.pi * X[:, 2]) * np.cos(np.pi * X[:, 0])
        return amplitude * u

    def u_col(self, amplitude):
        u = np.zeros(self.n_cols)
        un = self.node_displacement(amplitude)
        for d in range(3):
            u[self.node_dof_col + d] = un[:, d]
        return u


class Evaluator:
    """Device context (fcg_ctx): the MI355X replacement of Discretization::evaluate for SOLID
    hex8/hex27 + StVK.  Keeps 4C's error behaviour: a non-zero status raises FcgError."""

    def __init__(self, desc_or_mesh, kinematics=LINEAR, youngs=210.0, poisson=0.3, device=0,
                 path=PATH_AUTO, material=MAT_STVK):
        L = lib()
        if isinstance(desc_or_mesh, (BoxMesh, Discretization)):
            self._mesh = desc_or_mesh
            desc = desc_or_mesh.desc(kinematics, youngs, poisson, device, path, material)
        else:
            self._mesh = None
            desc = desc_or_mesh
        self.device = desc.device
        self.kinematics = int(desc.kinematics)
        h = ctypes.c_void_p()
        rc = L.fcg_create(ctypes.byref(desc), ctypes.byref(h))
        if rc != 0:
            raise FcgError(rc, L.fcg_last_error(None).decode())
        self._h = h
        info = FcgInfo()
        L.fcg_get_info(h, ctypes.byref(info))
        self.info = info

    def graph(self):
        """fcg_get_graph: (rowptr int64, col_lid int32) host copies of the context's CSR graph --
        the device-built one when the descriptor came without rowptr / col_lid."""
        L = lib()
        nnz = ctypes.c_int64(0)
        rc = L.fcg_get_graph(self._h, None, None, 0, ctypes.byref(nnz))
        if rc != 0:
            self._raise(rc, -1)
        rowptr = np.empty(self.info.n_rows + 1, dtype=np.int64)
        col = np.empty(max(nnz.value, 1), dtype=np.int32)
        rc = L.fcg_get_graph(self._h, _np_ptr(rowptr, _i64p), _np_ptr(col, _i32p), nnz.value,
                             ctypes.byref(nnz))
        if rc != 0:
            self._raise(rc, -1)
        return rowptr, col[:nnz.value]

    def close(self):
        if getattr(self, "_h", None):
            lib().fcg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _raise(self, rc, bad):
        raise FcgError(rc, lib().fcg_last_error(self._h).decode(), bad)

    def evaluate(self, action, u_col, fint_row, K_vals=None):
        """Host-pointer path (blocking, `+=` semantics like SparseMatrix::assemble)."""
        bad = ctypes.c_int32(-1)
        rc = lib().fcg_evaluate(self._h, action, _np_ptr(u_col, _dp), _np_ptr(fint_row, _dp),
                                _np_ptr(K_vals, _dp) if K_vals is not None else None,
                                ctypes.byref(bad))
        if rc != 0:
            self._raise(rc, bad.value)

    def evaluate_host(self, action, mode, u_col, fint_row, K_vals=None):
        """fcg_evaluate_host: host (numpy) buffers; mode OVERWRITE fuses the caller's zero()."""
        bad = ctypes.c_int32(-1)
        rc = lib().fcg_evaluate_host(self._h, action, mode, _np_ptr(u_col, _dp),
                                     _np_ptr(fint_row, _dp),
                                     _np_ptr(K_vals, _dp) if K_vals is not None else None,
                                     ctypes.byref(bad))
        if rc != 0:
            self._raise(rc, bad.value)

    def set_async(self, enable):
        """fcg_set_async: evaluate_device returns once queued; check_error reports failures."""
        rc = lib().fcg_set_async(self._h, 1 if enable else 0)
        if rc != 0:
            self._raise(rc, -1)

    def check_error(self):
        bad = ctypes.c_int32(-1)
        rc = lib().fcg_check_error(self._h, ctypes.byref(bad))
        if rc != 0:
            self._raise(rc, bad.value)

    def evaluate_device(self, action, mode, u_col, fint_row, K_vals=None, stream=None):
        """Device-resident path; tensors are float64 torch tensors on this device."""
        bad = ctypes.c_int32(-1)
        s = _torch_stream(stream, self.device)
        rc = lib().fcg_evaluate_device(self._h, action, mode, _tensor_ptr(u_col),
                                       _tensor_ptr(fint_row), _tensor_ptr(K_vals), s,
                                       ctypes.byref(bad))
        if rc != 0:
            self._raise(rc, bad.value)

    def _stream(self, stream):
        return _torch_stream(stream, self.device)

    def spmv(self, K_vals, x_col, y_row, stream=None):
        rc = lib().fcg_spmv(self._h, _tensor_ptr(K_vals), _tensor_ptr(x_col), _tensor_ptr(y_row),
                            self._stream(stream))
        if rc != 0:
            self._raise(rc, -1)

    def spmv_f32(self, K32, x_col, y_row, stream=None):
        """y = K x with an FP32 copy of the matrix values (asynchronous)."""
        rc = lib().fcg_spmv_f32(self._h, _tensor_ptr(K32), _tensor_ptr(x_col), _tensor_ptr(y_row),
                                self._stream(stream))
        if rc != 0:
            self._raise(rc, -1)

    def tangent_apply(self, u_col, x_col, y_row, stream=None):
        """y = K(u) x without a matrix (fcg_tangent_apply; hex27 StVK): the tangent the evaluate
        assembles at u, before Dirichlet rows, applied element by element (asynchronous).  u_col
        may be None for linear kinematics."""
        rc = lib().fcg_tangent_apply(self._h, _tensor_ptr(u_col), _tensor_ptr(x_col),
                                     _tensor_ptr(y_row), self._stream(stream))
        if rc != 0:
            self._raise(rc, -1)

    def dirichlet_apply(self, rows, K_vals=None, rhs=None, freact=None, stream=None):
        """rows: int32 device tensor of DBC row LIDs."""
        rc = lib().fcg_dirichlet_apply(self._h, int(rows.numel()), _tensor_ptr(rows),
                                       _tensor_ptr(K_vals), _tensor_ptr(rhs), _tensor_ptr(freact),
                                       self._stream(stream))
        if rc != 0:
            self._raise(rc, -1)

    def pcg_solve(self, K_vals, b, x, rtol=1e-12, max_iter=10000, stream=None):
        """K x = b (block-Jacobi PCG from x = 0); returns (iterations, relative residual)."""
        it, rr = ctypes.c_int(0), ctypes.c_double(0.0)
        rc = lib().fcg_pcg_solve(self._h, _tensor_ptr(K_vals), _tensor_ptr(b), _tensor_ptr(x),
                                 float(rtol), int(max_iter), ctypes.byref(it), ctypes.byref(rr),
                                 self._stream(stream))
        if rc != 0:
            self._raise(rc, -1)
        return it.value, rr.value

    def set_timing(self, enable):
        lib().fcg_set_timing(self._h, 1 if enable else 0)

    def diagnostics(self):
        """Per-phase cycle counters of the fused kernel (FCG_STAMPS=1 at creation), or None."""
        buf = (ctypes.c_uint64 * 16)()
        n = lib().fcg_get_diagnostics(self._h, buf, 16)
        return list(buf) if n > 0 else None

    CREATE_PHASES = ("checks", "graph_device", "node_rows", "lattice_plans", "incidences",
                     "incidence_positions", "device_plans", "total")

    def create_phases(self):
        """fcg_create's phase wall times (s) by name (fcg_get_create_phases)."""
        buf = (ctypes.c_double * 8)()
        lib().fcg_get_create_phases(self._h, buf, 8)
        return dict(zip(self.CREATE_PHASES, list(buf)))

    def timing(self):
        a, b = ctypes.c_double(), ctypes.c_double()
        lib().fcg_get_timing(self._h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value


class TsiGraph:
    """The thermo field of a rank for TSI: one temperature DOF per node of the cloned thermo
    discretization (same nodes, elements and owners as the structure; thermo DOF GIDs follow the
    structural ones, 4C_fem_dofset.cpp:628-632) and the Epetra graphs of k_ST, k_TS and k_TT.
    Derived from the structural node graph of `mesh` (BoxMesh or Discretization), whose DOF
    column LIDs are 3 per node in node order."""

    def __init__(self, mesh):
        nn = mesh.n_node
        self.node_dof_col_t = np.ascontiguousarray(mesh.node_dof_col // 3, dtype=np.int32)
        self.node_dof_row_t = np.ascontiguousarray(
            np.where(mesh.node_dof_row >= 0, mesh.node_dof_row // 3, -1), dtype=np.int32)
        self.n_rows_t = int(mesh.n_rows) // 3
        self.n_cols_t = int(mesh.n_cols) // 3
        assert len(self.node_dof_col_t) == nn
        rp = np.asarray(mesh.rowptr, dtype=np.int64)
        cl = np.asarray(mesh.col_lid)
        starts = rp[0:-1:3]                     # first structural row of every owned node
        nnb = (rp[1::3] - rp[0:-1:3]) // 3      # neighbour nodes of the row
        tot = int(nnb.sum())
        self.rowptr_tt = np.concatenate([[0], np.cumsum(nnb)]).astype(np.int64)
        off = np.arange(tot, dtype=np.int64) - np.repeat(self.rowptr_tt[:-1], nnb)
        self.col_tt = np.ascontiguousarray(cl[np.repeat(starts, nnb) + 3 * off] // 3, dtype=np.int32)
        # k_ST: 3 rows per node with the node's thermo columns
        n3 = np.repeat(nnb, 3)
        self.rowptr_st = np.concatenate([[0], np.cumsum(n3)]).astype(np.int64)
        src = np.repeat(np.repeat(self.rowptr_tt[:-1], 3), n3)
        off3 = np.arange(int(n3.sum()), dtype=np.int64) - np.repeat(self.rowptr_st[:-1], n3)
        self.col_st = np.ascontiguousarray(self.col_tt[src + off3], dtype=np.int32)
        # k_TS: one row per node with the node's structural columns (= its structural row)
        self.rowptr_ts = np.concatenate([[0], np.cumsum(3 * nnb)]).astype(np.int64)
        off_ts = np.arange(3 * tot, dtype=np.int64) - np.repeat(self.rowptr_ts[:-1], 3 * nnb)
        self.col_ts = np.ascontiguousarray(cl[np.repeat(starts, 3 * nnb) + off_ts], dtype=np.int32)
        self.nnz_st, self.nnz_ts, self.nnz_tt = len(self.col_st), len(self.col_ts), len(self.col_tt)


class TsiEvaluator:
    """Device context (fcg_tsi_ctx) for the temperature-dependent TSI blocks of one rank."""

    def __init__(self, mesh, youngs, poisson, thexpans, inittemp, conduct, device=0, graph=None):
        L = lib()
        self.mesh = mesh
        self.graph = g = graph or TsiGraph(mesh)
        d = FcgTsiDesc()
        d.abi_version = ABI_VERSION
        d.celltype = mesh.celltype
        d.device = device
        d.youngs, d.poisson, d.thexpans = youngs, poisson, thexpans
        d.inittemp, d.conduct = inittemp, conduct
        d.n_ele, d.n_node = mesh.n_ele, mesh.n_node
        d.n_rows_s, d.n_cols_s = mesh.n_rows, mesh.n_cols
        d.n_rows_t, d.n_cols_t = g.n_rows_t, g.n_cols_t
        d.ele_nodes = _np_ptr(mesh.ele_nodes, _i32p)
        d.ele_gid = _np_ptr(mesh.ele_gid, _i32p)
        d.node_x = _np_ptr(mesh.node_x, _dp)
        d.node_dof_col_s = _np_ptr(mesh.node_dof_col, _i32p)
        d.node_dof_row_s = _np_ptr(mesh.node_dof_row, _i32p)
        d.node_dof_col_t = _np_ptr(g.node_dof_col_t, _i32p)
        d.node_dof_row_t = _np_ptr(g.node_dof_row_t, _i32p)
        d.rowptr_st, d.col_st = _np_ptr(g.rowptr_st, _i64p), _np_ptr(g.col_st, _i32p)
        d.rowptr_ts, d.col_ts = _np_ptr(g.rowptr_ts, _i64p), _np_ptr(g.col_ts, _i32p)
        d.rowptr_tt, d.col_tt = _np_ptr(g.rowptr_tt, _i64p), _np_ptr(g.col_tt, _i32p)
        self.device = device
        h = ctypes.c_void_p()
        rc = L.fcg_tsi_create(ctypes.byref(d), ctypes.byref(h))
        if rc != 0:
            raise FcgError(rc, L.fcg_tsi_last_error(None).decode())
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().fcg_tsi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def evaluate_device(self, parts, mode, v_col, T_col, timefac=1.0, timefac_d=1.0, fs=None,
                        Kst=None, fT=None, Ktt=None, Kts=None, stream=None):
        """Tensors: float64 on this device (v_col / T_col in the structural / thermo column maps)."""
        bad = ctypes.c_int32(-1)
        s = _torch_stream(stream, self.device)
        rc = lib().fcg_tsi_evaluate_device(self._h, parts, mode, _tensor_ptr(v_col),
                                           _tensor_ptr(T_col), float(timefac), float(timefac_d),
                                           _tensor_ptr(fs), _tensor_ptr(Kst), _tensor_ptr(fT),
                                           _tensor_ptr(Ktt), _tensor_ptr(Kts), s, ctypes.byref(bad))
        if rc != 0:
            raise FcgError(rc, lib().fcg_tsi_last_error(self._h).decode(), bad.value)

    def evaluate_fused(self, struct_ev, mode, u_col, v_col, T_col, timefac=1.0, timefac_d=1.0,
                       fs=None, Kss=None, Kst=None, fT=None, Ktt=None, Kts=None, stream=None):
        """fcg_tsi_evaluate_fused: the whole monolithic tangent (K_SS, k_ST, k_TS, k_TT) and both
        residuals in one sweep; `struct_ev` is the structured linear StVK Evaluator of the mesh."""
        bad = ctypes.c_int32(-1)
        s = _torch_stream(stream, self.device)
        rc = lib().fcg_tsi_evaluate_fused(struct_ev._h, self._h, mode, _tensor_ptr(u_col),
                                          _tensor_ptr(v_col), _tensor_ptr(T_col), float(timefac),
                                          float(timefac_d), _tensor_ptr(fs), _tensor_ptr(Kss),
                                          _tensor_ptr(Kst), _tensor_ptr(fT), _tensor_ptr(Ktt),
                                          _tensor_ptr(Kts), s, ctypes.byref(bad))
        if rc != 0:
            raise FcgError(rc, lib().fcg_tsi_last_error(self._h).decode(), bad.value)


def graph_build_device(celltype, ele_nodes, node_dof_col, node_dof_row, n_rows, device=0,
                       stream=None):
    """fcg_graph_build_device on torch tensors (int32, on `device`): returns (rowptr int64,
    col_lid int32) device tensors -- the FillComplete graph of the rank's owned rows."""
    import torch
    dev = torch.device("cuda", device)
    rowptr = torch.empty(int(n_rows) + 1, dtype=torch.int64, device=dev)
    nnz = ctypes.c_int64(0)
    s = _torch_stream(stream, device)
    args = (device, celltype, int(ele_nodes.numel() // (8 if celltype == HEX8 else 27)),
            _tensor_ptr(ele_nodes), int(node_dof_col.numel()), _tensor_ptr(node_dof_col),
            _tensor_ptr(node_dof_row), int(n_rows), _tensor_ptr(rowptr))
    rc = lib().fcg_graph_build_device(*args, None, 0, ctypes.byref(nnz), s)
    if rc != 0:
        raise FcgError(rc, "fcg_graph_build_device (sizing) failed")
    col = torch.empty(max(1, nnz.value), dtype=torch.int32, device=dev)
    rc = lib().fcg_graph_build_device(*args, _tensor_ptr(col), nnz.value, ctypes.byref(nnz), s)
    if rc != 0:
        raise FcgError(rc, "fcg_graph_build_device failed")
    return rowptr, col[:nnz.value]


def measure_peaks(device=0):
    """fcg_measure_peaks: (STREAM-triad GB/s, FP64 VALU TFLOP/s, FP64 MFMA TFLOP/s) on `device`."""
    a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    rc = lib().fcg_measure_peaks(int(device), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    if rc != 0:
        raise FcgError(rc, "fcg_measure_peaks failed")
    return a.value, b.value, c.value


def measure_hbm(device=0):
    """fcg_measure_hbm: (16-byte copy GB/s, write-only fill GB/s) on `device`."""
    a, b = ctypes.c_double(), ctypes.c_double()
    rc = lib().fcg_measure_hbm(int(device), ctypes.byref(a), ctypes.byref(b))
    if rc != 0:
        raise FcgError(rc, "fcg_measure_hbm failed")
    return a.value, b.value
