// fcg_internal.hpp -- context layout and kernel launch interface shared by the HIP translation
// units of libfourc_gpu.  Not part of the public ABI (include/fourc_gpu.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "fourc_gpu.h"

namespace fcg {

// Per-incidence scratch record written by the element kernel and consumed by the row-assembly
// kernel: the element's block-row of node a (3 rows x 3*npe columns, b-major) then f_a (3).
// One owned incidence's block row (3 x 3 npe) and its 3 residual entries.  hex27: padded to
// FCG_REC27 = 256 doubles so that records start on 128-byte lines: no line is shared by two
// records, which the overlapped schedule needs (a row node on another XCD reads its records
// while a neighbouring record's element may not have run yet; a shared line could then sit stale
// in that XCD's L2).  Unpadded (246) measured the same (profiles/r06/r06_h27_record_store_ab.txt).
#ifndef FCG_REC27
#define FCG_REC27 256
#endif
constexpr int64_t record_doubles(int npe) { return npe == 27 ? int64_t(FCG_REC27) : 9 * int64_t(npe) + 3; }

struct DeviceMesh {
  int celltype = 0, kinem = 0, npe = 8;
  int64_t n_ele = 0, n_node = 0, n_rows = 0, n_cols = 0, nnz = 0;
  int64_t n_rownodes = 0, n_inc = 0;
  double lambda = 0, mu = 0, cdiag = 0;  // StVK: C_00 = cdiag, C_01 = lambda, C_33 = mu
  int material = FCG_MAT_STVK;
  double nh_c = 0, nh_beta = 0;          // ElastHyper/CoupNeoHooke constants

  int32_t* ele_nodes = nullptr;     // [n_ele][npe]
  int32_t* ele_gid = nullptr;       // [n_ele]
  double* node_x = nullptr;         // [n_node][3]
  int32_t* node_dof_col = nullptr;  // [n_node]
  int32_t* inc_of = nullptr;        // [n_ele][npe] incidence id or -1
  int64_t* inc_ptr = nullptr;       // [n_rownodes+1]
  int32_t* rownode_row0 = nullptr;  // [n_rownodes]
  uint16_t* inc_pos = nullptr;      // [n_inc][npe] column position of node b in the row
  int64_t* rowptr = nullptr;        // [n_rows+1]
  double* scratch = nullptr;        // [n_inc][record_doubles(npe)]
  int32_t* err = nullptr;           // [3]: code, min failing element index; [2] the solver flag
  // (Dirichlet / block-Jacobi / PCG kernels write only err[2], so a failed element's flags from an
  // async evaluate survive them until fcg_check_error reads them)
  // evaluate's error-flag protocol: err holds {0, INT32_MAX} between calls while err_clean is set
  // (no per-call re-initialisation); whatever else writes err clears err_clean.  The flags come
  // back through the pinned err_host (a DMA, not a staged pageable copy).
  int32_t* err_host = nullptr;      // [2], pinned host memory
  bool err_clean = false;
  int32_t max_rowlen = 0;

  // colour-ordered direct assembly (hex27 on a verified lattice, FCG_PATH_COLORED)
  int32_t* col_ele = nullptr;       // [n_ele] elements sorted by colour (lattice parity), then index
  int64_t color_ptr[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // col_ele range of colour c
  uint8_t* ele_ft = nullptr;        // [n_ele] first-touch bits (see fcg_kernels.hip)
  int32_t* inc_row0 = nullptr;      // [n_inc] row LID of the incidence's node
  // hex27 StVK on a verified lattice: the matrix-core element kernel in pencil order (fcg_hex27.hip)
  bool h27_pencil = false;
  int64_t* pen_ptr = nullptr;       // [n_pencils+1] pencil ranges in col_ele (pencil order)
  int64_t pen_color[5] = {0, 0, 0, 0, 0};  // pencil range of colour c
  uint32_t* ele_nb = nullptr;       // [n_ele] lattice neighbours present | ey & 1 << 27 | ez & 1 << 28

  // node-row gather plan (hex8, FCG_PATH_GATHER): a row node's incidences in records of <= 8
  // records: one per node with <= 8 elements [0, n_rec_single), then those of the other nodes
  int64_t n_rec = 0, n_rec_single = 0, n_multi = 0;
  int64_t* multi_ptr = nullptr;     // [n_multi+1] record range of each node with > 8 elements
  int32_t* rec_row0 = nullptr;      // [n_rec] first row LID of the record's node
  int32_t* rec_meta = nullptr;      // [n_rec] slots | first record << 4 | last record << 5 | row length << 8
  int64_t* rec_base = nullptr;      // [n_rec] CSR offset of the node's first row
  int32_t* rec_ele = nullptr;       // [n_rec][8] element of each slot, -1 = empty
  uint8_t* rec_a = nullptr;         // [n_rec][8] local node of the row node in the slot's element
  uint32_t* rec_tmap = nullptr;     // [n_rec][32] per column triple: slot s's element node in nibble s (8 = none)
  // hex27 StVK general path (fcg_hex27.hip): per-element symmetric records in `scratch`
  bool h27s = false;
  bool h27_increc = false;  // hex27 element kernel writes incidence block rows (assemble27_kernel)
  int32_t* inc_ele = nullptr;       // [n_inc] element of each incidence
  uint8_t* inc_a = nullptr;         // [n_inc] local node of the row node in that element
  int32_t* asm_order = nullptr;     // [n_rownodes] row nodes in Morton order of their coordinates
  int32_t* ele_orig = nullptr;      // [n_ele] column element index of each storage slot (Morton order)
  double* ele_x = nullptr;          // [n_ele][8][3] element node coordinates (storage slot order)
  double* ele_gp = nullptr;         // [n_ele][8][10] Gauss-point factors (gather_precompute)
  int32_t gp_bad_code = 0, gp_bad_ele = 0;  // a Jacobian failure found by gather_precompute
  int32_t* ele_dof = nullptr;       // [n_ele][8] column LID of each element node's first DOF
  double* gather_dummy = nullptr;   // [4] store target of a row without columns
  double* apply_ye = nullptr;       // [n_inc][3] fcg_tangent_apply's node parts (allocated on first use)
  int32_t* apply_dof = nullptr;     // [n_ele][27] column LID of each element node's first DOF (idem)
  // hex27 slab schedule (FCG_H27_SLAB): the elements run in slabs of h27_slab consecutive
  // elements; after slab s the row nodes whose last incident element lies in slab s are assembled,
  // so an incidence record lives only from its slab to its row's slab, in a ring of h27_ring
  // records (instead of one record per incidence)
  int64_t h27_nslab = 0, h27_slab = 0, h27_ring = 0;
  int h27_el_grid = 512;             // element workgroups per slab launch (the resident ones)
  std::vector<int64_t> h27_asm_ptr;  // [h27_nslab + 1] range of h27_rows assembled after slab s
  int32_t* h27_rows = nullptr;       // [n_rownodes] row nodes by completing slab, then Morton order
  int32_t* h27_rslot0 = nullptr;     // [n_rownodes] ring slot of the row node's first record
  int32_t* h27_slot = nullptr;       // [n_ele][27] ring slot of incidence (e, a), -1 = not owned
  // hex27 overlapped schedule (FCG_H27_OVERLAP=1 with the full scratch; measured slower than the
  // element launch + row-assembly launch): one queue of element chunks (ovl_chunk
  // consecutive elements) and row items (runs of row nodes whose incident elements all lie in
  // completed bands of ovl_band_chunks chunks)
  bool h27_ovl = false;
  int64_t ovl_items = 0, ovl_chunk = 0, ovl_nchunks = 0, ovl_nbands = 0;
  int ovl_band_chunks = 1;
  int32_t* ovl_queue = nullptr;     // [ovl_items] chunk c >= 0 | ~row item
  int32_t* ovl_ritem = nullptr;     // [row items][4] rows [j0, j1) of ovl_rows, bands [lo, hi]
  int32_t* ovl_rows = nullptr;      // [n_rownodes] by completing band, then Morton order
  int64_t* ovl_rmeta = nullptr;     // [n_rownodes][4] of ovl_rows[j]: CSR offset, first row,
                                    // first incidence, row length | incidences << 16
  unsigned* ovl_sync = nullptr;     // [1 + ovl_nbands] claim counter, completed chunks per band

  // structured (row-block sweep) plan, hex8 only
  int path = FCG_PATH_GENERAL;
  int32_t tiles_x = 0, tiles_y = 0, tiles_z = 0, seg_planes = 0;
  int32_t I0 = 0, J0 = 0, K0 = 0, NI = 0, NJ = 0, NK = 0;  // owned-node lattice box
  int32_t EX0 = 0, EY0 = 0, EZ0 = 0, EX = 0, EY = 0, EZ = 0;  // column-element lattice box
  bool sweep_defer = false;         // rows not in lattice order: sweep MODE 3 (fcg_sweep.hip)
  int32_t* elem_at = nullptr;       // [EZ][EY][EX] column element or -1
  double* lat_x = nullptr;          // [EZ+1][EY+1][EX+1][3] node coordinates on the lattice
  int32_t* lat_dof = nullptr;       // [EZ+1][EY+1][EX+1] column LID of the node's first DOF or -1
  uint32_t* plane_rec = nullptr;    // [tiles_y][tiles_x][NK][PLANE_REC_WORDS] row bookkeeping
  double* tables = nullptr;         // dN at GPs [192], dN at nodes [192], weights [8]
  unsigned long long* stamps = nullptr;  // diagnostic phase timers (FCG_STAMPS=1), else NULL

  // operator / solver support (fcg_solver.hip)
  int32_t* col_lid = nullptr;       // [nnz] CSR column LIDs (matrix column map)
  int64_t* diag_pos = nullptr;      // [n_rows] position of the diagonal entry in K values, -1 = none
  bool square_local = false;        // matrix column map == row map (single rank)
  bool owned_cols_first = false;    // column LID of every owned DOF == its row LID (ghosts after)
  double* pcg_work = nullptr;       // PCG vectors and partial sums (allocated on first solve)
  int64_t pcg_n = 0;
};

// One record per (tile, node plane): row0[16] | rowlen[16] | rbase[16] (int64) | npos[16][27]
// (uint16, column position of lattice neighbour t inside the node's rows, 0xFFFF = absent).
constexpr int PLANE_REC_WORDS = 288;

// Launches the structured hex8 row-block sweep (element evaluation + assembly, fcg_sweep.hip).
hipError_t launch_sweep_h8(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream);

// Fused TSI blocks of the structured sweep (fcg_tsi_evaluate_fused): linear kinematics, StVK,
// node-consistent thermo numbering (thermo LID = structural LID / 3, see fcg_tsi.hip).
struct SweepTsi {
  const double* v_col = nullptr;
  const double* T_col = nullptr;
  const double* Ngp = nullptr;  // shape values at the hex8 Gauss points [8][8]
  double* Kst = nullptr;
  double* Kts = nullptr;
  double* Ktt = nullptr;
  double* fT = nullptr;
  double m = 0, T0 = 0, conduct = 0, kts = 0;  // kts = -timefac timefac_d
  bool split = true;  // structural sweep + thermal-only pass (FCG_TSI_SPLIT=0: one fused pass)
};
hipError_t launch_sweep_h8_tsi(const DeviceMesh& m, const double* d_u_col, bool overwrite,
    double* d_K, double* d_fint, const SweepTsi& t, hipStream_t stream);

struct Timing {
  bool enabled = false;
  bool pending = false;  // events recorded, durations not read yet (async evaluate)
  int path = 0;
  bool fused = false;  // ev[1] marks no element/assembly boundary (hex27 slab schedule)
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  double ms_element = 0.0, ms_assemble = 0.0;
};

// Host <-> device copies of the host-buffer entry points through pinned staging chunks: the DMA
// of one chunk overlaps the host-side copy of the previous one (threads > 0), or one pageable
// hipMemcpy (threads == 0).
struct HostStaging {
  double* pin[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipStream_t stream = nullptr;
  int64_t chunk = 0;  // doubles per chunk
  int threads = 8;
};
hipError_t staged_copy(HostStaging& st, int device, void* dst, const void* src, int64_t bytes,
    bool to_device);
void staging_free(HostStaging& st);

void upload_constant_tables(int celltype);  // GP / nodal derivative tables -> __constant__
hipError_t launch_element(const DeviceMesh& m, const double* d_u_col, bool want_k,
    hipStream_t stream);
// Colour-ordered direct assembly (FCG_PATH_COLORED): eight element launches, one per colour,
// each adding (or, first in colour order, writing) its blocks straight into the CSR rows.
hipError_t launch_element_colored(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream);
hipError_t launch_assemble(const DeviceMesh& m, bool want_k, bool overwrite, double* d_K,
    double* d_fint, hipStream_t stream);
// hex27 StVK on any mesh (fcg_hex27.hip): element kernel writing one symmetric record per
// element (blocks a <= b + f_e), then one wavefront per owned row node in Morton order.
void upload_h27_tables();
constexpr int64_t kH27RecDoubles = 378 * 9 + 81 + 1;  // even: 16-byte aligned records
hipError_t launch_h27_element(const DeviceMesh& m, const double* d_u_col, bool want_k,
    hipStream_t stream, int64_t e_begin = 0, int64_t e_end = -1);
// hex27 slab schedule: the row assembly of the row nodes completed by slab s
hipError_t launch_assemble27_slab(const DeviceMesh& m, int64_t s, bool want_k, bool overwrite,
    double* d_K, double* d_fint, hipStream_t stream);
hipError_t launch_h27_assemble(const DeviceMesh& m, bool want_k, bool overwrite, double* d_K,
    double* d_fint, hipStream_t stream);
// hex27 overlapped schedule: element chunks and row items of one queue in one launch
hipError_t launch_h27_overlap(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream);
// hex27 StVK on a verified lattice: the same element kernel adding its blocks straight into the
// CSR rows, four colour launches of pencils (runs of elements along x, one workgroup each)
hipError_t launch_h27_pencil(const DeviceMesh& m, const double* d_u_col, bool want_k,
    bool overwrite, double* d_K, double* d_fint, hipStream_t stream);
// Matrix-free tangent action y_row = K(u) x_col of hex27 StVK (fcg_tangent_apply): the element
// kernel writes each owned incidence's 3 values to m.apply_ye, a row-node pass sums them.
hipError_t launch_h27_apply(const DeviceMesh& m, const double* d_u_col, const double* d_x_col,
    double* d_y_row, hipStream_t stream);
hipError_t launch_h27_apply_plan(const DeviceMesh& m, hipStream_t stream);  // fills m.apply_dof
// Node-row gather (FCG_PATH_GATHER, hex8 StVK on any mesh): one wavefront per owned row node
// (fcg_gather.hip).
hipError_t gather_precompute(DeviceMesh& m, int64_t n_ele, hipStream_t stream);
hipError_t launch_gather_h8(const DeviceMesh& m, const double* d_u_col, bool want_k, bool overwrite,
    double* d_K, double* d_fint, hipStream_t stream);

}  // namespace fcg

struct fcg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  fcg::DeviceMesh mesh;
  fcg::Timing timing;
  std::string last_error;
  int64_t device_bytes = 0;
  // device buffers of the host-pointer entry points
  double* h_u = nullptr;
  double* h_f = nullptr;
  double* h_k = nullptr;
  fcg::HostStaging staging;
  // deferred error check (fcg_set_async)
  bool async = false;
  bool pending = false;
  hipStream_t pending_stream = nullptr;
  double create_phase_s[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // fcg_get_create_phases
};

// fcg_dfcg_solve's AMG preconditioner (fcg_amg_solver.hip; not part of the C ABI): numeric setup
// and one application, with the coarse levels coupled across the ranks of the transport when the
// handle is rank-local (fcg_amgs::Coupled), else the handle's own V-cycle
extern "C" {
int fcg_amg_precond_setup(fcg_amg* h, const double* d_K, const fcg_transport* tr, void* stream);
int fcg_amg_precond_apply(fcg_amg* h, const double* d_K, const fcg_transport* tr, const double* d_r,
    double* d_z, void* stream);
}
