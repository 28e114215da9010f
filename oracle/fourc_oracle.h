/*
 * fourc_oracle.h -- CPU restatement of 4C's solid element evaluation + global assembly path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity oracle and the CPU baseline
 * (`cpu_baseline.kind = "port"` in bench.py).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product path (4c_amd/) never links or calls it.
 *
 * It restates, function by function, the reference files listed in SURVEY.md §8(c); every
 * function cites the file:line it follows (paths relative to the 4C source tree).
 *
 * Parity pinning: the restatement is checked against the reference's own known answers
 * (tests/test_oracle_known_answers.py): GridGenerator unit test (node counts, last gid, rotated
 * coordinates at 1e-14), StVenantKirchhoff unit test (stress, energy), and the end-to-end
 * RESULT DESCRIPTION displacements of solid_ele_hex8_Standard_linear.dat,
 * solid_ele_hex27_Standard_linear.dat (1e-12) and sohex27_patchtest_nl_cost_drt.dat (1e-9).
 * The reference itself cannot be compiled here (Trilinos/MPI absent, C++20 <format> missing;
 * SURVEY.md §8c), so no oracle/_ref build exists.
 */
#ifndef FOURC_ORACLE_H
#define FOURC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_HEX8 = 0, ORC_HEX27 = 1 };
enum { ORC_LINEAR = 0, ORC_TOTLAG = 1 };
enum { ORC_OK = 0, ORC_ERR_NODAL_DETJ = 1, ORC_ERR_SINGULAR = 2, ORC_ERR_ARG = 3 };
/* MAT_Struct_StVenantKirchhoff / MAT_ElastHyper with one ELAST_CoupNeoHooke summand */
enum { ORC_MAT_STVK = 0, ORC_MAT_NEOHOOKE = 1 };

int orc_num_nodes(int celltype);
int orc_num_gp(int celltype);

/* Gauss rule of the stiffness matrix: 4C_fem_general_utils_integration.cpp:74-106 (hex_8point)
 * and :130-245 (hex_27point, truncated constants). xi: [ngp][3], w: [ngp]. */
void orc_gauss_points(int celltype, double* xi, double* w);

/* Shape functions / first derivatives: 4C_fem_general_utils_fem_shapefunctions.hpp:53-72,
 * 190-229 (values) and :386-426, 683-788 (derivs).  dN is column-major 3 x n: dN[3*node+d]. */
void orc_shape(int celltype, const double* xi, double* N);
void orc_shape_deriv1(int celltype, const double* xi, double* dN);

/* Parameter-space node coordinates (4C_fem_general_utils_local_connectivity_matrices.hpp:291). */
void orc_node_param_coords(int celltype, double* xi /* [n][3] */);

/* StVK: 4C_mat_stvenantkirchhoff.cpp:115-145 (fill_cmat), :169-177 (evaluate),
 * strain_energy :184-194.  cmat column-major 6x6. */
void orc_stvk_cmat(double E, double nu, double* cmat);
void orc_stvk_evaluate(double E, double nu, const double* glstrain, double* stress, double* cmat);
double orc_stvk_strain_energy(double E, double nu, const double* glstrain);

/* ElastHyper + CoupNeoHooke (YOUNG E, NUE nu): PK2 stress and cmat (column-major 6x6) at the
 * Green-Lagrange strain (strain-like Voigt), 4C_mat_elasthyper_service.cpp:19-215. */
void orc_elasthyper_coupneohooke(double E, double nu, const double* glstrain, double* stress,
    double* cmat);

/* SolidEleCalc<celltype, Formulation>::evaluate_nonlinear_force_stiffness_mass
 * (4C_solid_3D_ele_calc.cpp:110-240) for DisplacementBased(LinearKinematics)Formulation + StVK.
 * X, u: [n][3] reference coordinates and displacements (node-major as lm).
 * Ke: (3n x 3n) column-major, summed into (+=) when non-NULL.  fe: 3n, += when non-NULL.
 * Returns ORC_OK, ORC_ERR_NODAL_DETJ (calc_lib.hpp:475-496) or ORC_ERR_SINGULAR
 * (invert3x3 det == 0, 4C_linalg_fixedsizematrix.hpp:1394). */
int orc_solid_evaluate(int celltype, int kinem, double E, double nu, const double* X,
    const double* u, double* Ke, double* fe);
/* The same with the material chosen by ORC_MAT_* (E, nu are the summand's YOUNG, NUE). */
int orc_solid_evaluate_mat(int celltype, int kinem, int material, double E, double nu,
    const double* X, const double* u, double* Ke, double* fe);

/* GridGenerator restatement (4C_io_gridgenerator.cpp). */
void orc_hex_element_nodeids(int celltype, int64_t eleid, const int32_t* interval,
    int64_t node_offset, int64_t* nodeids);                                 /* :329-392 */
void orc_lattice_node_coords(int64_t gid, const int32_t* interval, int64_t node_offset,
    const double* lo, const double* hi, const double* rot_deg, double* x);  /* :254-323 */
int orc_box_section(const int32_t* interval, int nproc, int rank, int32_t* range6); /* :87-153 */

/* Global CSR in the Epetra "filled" state: rows = row-map LIDs, col_lid sorted per row. */
typedef struct orc_csr {
  int64_t n_rows;
  const int64_t* rowptr;
  const int32_t* col_lid;
  double* vals;
  const int32_t* row_lid_of_gid; /* dense gid -> row lid (-1 if not a row here) */
  const int32_t* col_lid_of_gid; /* dense gid -> col lid */
  int64_t max_gid;
} orc_csr;

/* SparseMatrix::assemble, filled path (4C_linalg_sparsematrix.cpp:426-576). */
int orc_sparse_assemble(orc_csr* A, int myrank, int nnode, const int* lmstride, int ndof,
    const double* Aele, const int* lmrow, const int* lmrowowner, const int* lmcol);

/* The same for lrowdim x lcoldim element matrices (TSI coupling blocks); numnode / lmstride
 * describe the column nodes. */
int orc_sparse_assemble_rect(orc_csr* A, int myrank, int numnode, const int* lmstride, int lrowdim,
    int lcoldim, const double* Aele, const int* lmrow, const int* lmrowowner, const int* lmcol);

/* LinAlg::assemble(Vector&, ...) (4C_linalg_utils_sparse_algebra_assemble.cpp:72-92). */
int orc_vector_assemble(double* V, const int32_t* lid_of_gid, int64_t max_gid, int ndof,
    const double* Vele, const int* lm, const int* lmowner, int myrank);

/* Discretization::evaluate(struct_calc_nlnstiff / struct_calc_internalforce) over a whole
 * mesh (4C_fem_discretization_evaluate.cpp:65-103), with `nworkers` "ranks" run as OpenMP
 * threads: worker w loops over its column elements (those touching a node it owns) and
 * assembles only rows it owns -- the reference's MPI semantics.
 *   ele_nodes: [n_ele][npe] indices into the node arrays (4C node order)
 *   node_gid:  [n_nodes] node GIDs;  node_owner: [n_nodes] owning worker
 *   dof gid = 3*(node_gid - min_node_gid) + d  (4C_fem_dofset.cpp:343-351)
 *   u: displacement indexed by the col map (col_lid_of_gid)
 *   K carries the maps; K->vals == NULL means internal force only; fint by row lid, +=.
 * Returns 0 or the first element error (its element index written to *bad_ele). */
int orc_discretization_evaluate(int celltype, int kinem, double E, double nu, int64_t n_ele,
    const int64_t* ele_nodes, int64_t n_nodes, const double* node_x, const int64_t* node_gid,
    const int32_t* node_owner, int64_t min_node_gid, int nworkers, const double* u, orc_csr* K,
    double* fint, int64_t* bad_ele);
int orc_discretization_evaluate_mat(int celltype, int kinem, int material, double E, double nu,
    int64_t n_ele, const int64_t* ele_nodes, int64_t n_nodes, const double* node_x,
    const int64_t* node_gid, const int32_t* node_owner, int64_t min_node_gid, int nworkers,
    const double* u, orc_csr* K, double* fint, int64_t* bad_ele);

/* ---------------------------------------------------------------------------------------
 * Thermo-structure interaction, geometrically linear (BASELINE config 5).  Pinned against the
 * RESULT DESCRIPTION of tsi_heatflux_monolithic.dat and tsi_heatflux_flexoutsurf_monolithic.dat
 * (tests/test_oracle_known_answers.py).
 * ------------------------------------------------------------------------------------- */
/* stress-temperature modulus m = -(2 mu + 3 lambda) alpha_T (4C_mat_thermostvenantkirchhoff.cpp:331-369) */
double orc_thermo_stvk_st_modulus(double E, double nu, double alpha);

/* SOLIDSCATRA + ThermoStVenantKirchhoff, KINEM linear:
 *   Ke, fe  struct_calc_nlnstiff with the "temperature" state (4C_solid_scatra_3D_ele_calc.cpp:272-403;
 *           S = C E + m (T_gp - T0) (1,1,1,0,0,0), 4C_mat_thermostvenantkirchhoff.cpp:141-174)
 *   Kst     struct_calc_stifftemp (4C_solid_scatra_3D_ele_calc.cpp:405-490): (3n x n)
 * T: [n] nodal temperatures.  Matrices column-major, all outputs +=, NULL = skip. */
int orc_tsi_solid_evaluate(int celltype, double E, double nu, double alpha, double T0,
    const double* X, const double* u, const double* T, double* Ke, double* fe, double* Kst);

/* Thermo::TemperImpl, geometrically linear TSI (4C_thermo_ele_impl.cpp):
 *   Ktt, fT  calc_thermo_fintcond: linear_thermo_contribution (:802-891) + linear_disp_contribution
 *            (:899-1043) with Fourier conductivity `conduct` and stress-temperature modulus m
 *   Kts      calc_thermo_coupltang: linear_coupled_tang (:1046-1194), (n x 3n)
 * v: [n][3] nodal velocities; timefac, timefac_d per :1094-1132 (statics: 1, 1/dt). */
int orc_tsi_thermo_evaluate(int celltype, double conduct, double m, const double* X,
    const double* T, const double* v, double timefac, double timefac_d, double* Ktt,
    double* fT, double* Kts);

/* All four TSI blocks and both residuals of a mesh, assembled rank by rank (owned rows) like
 * orc_discretization_evaluate.  u, v: structural column vectors (Kss's column map); T: thermo
 * column vector (Ktt's column map). */
int orc_tsi_discretization_evaluate(int celltype, double E, double nu, double alpha, double T0,
    double conduct, double timefac, double timefac_d, int64_t n_ele, const int64_t* ele_nodes,
    const double* node_x, const int64_t* node_gid, const int32_t* node_owner, int64_t min_node_gid,
    int nworkers, const double* u, const double* v, const double* T, orc_csr* Kss, orc_csr* Kst,
    orc_csr* Kts, orc_csr* Ktt, double* fs, double* ft, int64_t* bad_ele);

#ifdef __cplusplus
}
#endif
#endif
