"""Pin the CPU oracle against the reference's own known answers (no GPU needed).

Known answers used (all from /root/reference, copied as data into tests/golden/ by
tests/golden/make_fixtures.py or quoted below with their file:line):
  * unittests/io/4C_gridgenerator_test.cpp:67-130  (node counts, last gid, coordinates 1e-14)
  * unittests/mat/4C_stvenantkirchhoff_test.cpp:42-130 (stress 1e-4, energy 908.6538)
  * tests/input_files/solid_ele_hex8_Standard_linear.dat  RESULT DESCRIPTION (1e-12)
  * tests/input_files/solid_ele_hex27_Standard_linear.dat RESULT DESCRIPTION (1e-12)
  * tests/input_files/sohex27_patchtest_nl_cost_drt.dat   RESULT DESCRIPTION (1e-9)
  * tests/input_files/solid_ele_hex8_Standard_eas_none_volume_neumann.dat, solid_ele_hex27_Standard_volume_neumann.dat
    RESULT DESCRIPTION (ElastHyper/CoupNeoHooke, large deformation, 1e-12)
  * tests/input_files/tsi_heatflux_monolithic.dat         RESULT DESCRIPTION (1e-9 disp, 1e-6 temp)
  * tests/input_files/tsi_heatflux_flexoutsurf_monolithic.dat RESULT DESCRIPTION (1e-8)
The result-test comparison is absolute (4C_utils_result_test.cpp:98).
"""

import json
import os

import numpy as np
import pytest

import oracle_lib as orc
from fe_driver import Problem
from tsi_driver import TsiProblem

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixture(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


# --------------------------------------------------------------------------- grid generator
GG_LO = (-1.0, -2.0, -3.0)
GG_HI = (2.5, 3.5, 4.5)
GG_IV = (5, 10, 15)
GG_OFF = 17


def _gridgen_node_set(celltype):
    n = GG_IV[0] * GG_IV[1] * GG_IV[2]
    nodes = set()
    for e in range(n):
        nodes.update(int(g) for g in orc.hex_nodeids(celltype, e, GG_IV, GG_OFF))
    return n, sorted(nodes)


@pytest.mark.parametrize("celltype,nnodes", [(orc.HEX8, 1056), (orc.HEX27, 7161)])
def test_gridgenerator_counts_and_last_node(celltype, nnodes):
    nele, nodes = _gridgen_node_set(celltype)
    assert nele == 750
    assert len(nodes) == nnodes
    assert nodes[-1] == 7177
    x = orc.node_coords(nodes[-1], GG_IV, GG_OFF, GG_LO, GG_HI)
    np.testing.assert_allclose(x, [2.5, 3.5, 4.5], atol=1e-14, rtol=0)


def test_gridgenerator_rotated():
    _, nodes = _gridgen_node_set(orc.HEX8)
    x = orc.node_coords(nodes[-1], GG_IV, GG_OFF, GG_LO, GG_HI, rot=(30.0, 10.0, 7.0))
    np.testing.assert_allclose(x, [2.6565639116964181, 4.8044393443812901, 2.8980306453470042],
                               atol=1e-14, rtol=0)


def test_box_partition_2x2x2():
    # 8 ranks on a cube -> 2x2x2 sub-boxes (4C_io_gridgenerator.cpp:87-153)
    seen = set()
    for r in range(8):
        rng = orc.box_section((200, 200, 200), 8, r)
        assert all(rng[2 * d + 1] - rng[2 * d] == 100 for d in range(3))
        seen.add(tuple(rng))
    assert len(seen) == 8
    assert list(orc.box_section((200, 100, 100), 2, 1)) == [100, 200, 0, 100, 0, 100]


# --------------------------------------------------------------------------- material
def test_stvk_stress_and_energy():
    E, nu = 210.0, 0.3
    gl = np.ones(6)
    s, c = orc.stvk(E, nu, gl)
    normal = (E / ((1.0 + nu) * (1.0 - 2.0 * nu))) * ((1.0 - nu) + nu + nu)
    shear = (E / ((1.0 + nu) * (1.0 - 2.0 * nu))) * ((1.0 - 2.0 * nu) / 2.0)
    np.testing.assert_allclose(s, [normal] * 3 + [shear] * 3, atol=1e-4)
    assert abs(orc.stvk_energy(E, nu, gl) - 908.6538) < 1e-4
    assert np.allclose(c, c.T)


# --------------------------------------------------------------------------- element level
def test_gauss_rules_truncated_constants():
    xi, w = orc.gauss_points(orc.HEX27)
    assert xi[0, 0] == -0.7745966692415
    assert w[26] == 0.8888888888889 * 0.8888888888889 * 0.8888888888889
    xi8, w8 = orc.gauss_points(orc.HEX8)
    assert np.allclose(np.abs(xi8), 1.0 / np.sqrt(3.0)) and np.all(w8 == 1.0)


@pytest.mark.parametrize("celltype", [orc.HEX8, orc.HEX27])
def test_shape_partition_of_unity(celltype):
    xi = np.array([0.13, -0.41, 0.77])
    assert abs(orc.shape(celltype, xi).sum() - 1.0) < 1e-14
    assert np.abs(orc.shape_deriv(celltype, xi).sum(axis=0)).max() < 1e-14


@pytest.mark.parametrize("celltype", [orc.HEX8, orc.HEX27])
@pytest.mark.parametrize("kinem", [orc.LINEAR, orc.TOTLAG])
def test_tangent_is_derivative_of_force(celltype, kinem):
    """K_e must be the consistent linearisation of f_e (finite differences)."""
    rng = np.random.default_rng(7)
    n = 8 if celltype == orc.HEX8 else 27
    # reference coordinates: a jittered unit cube in the element's parameter-space node order
    par = orc.node_param_coords(celltype)
    X = 0.5 * (par + 1.0) + 0.05 * rng.standard_normal(par.shape)
    u = 0.02 * rng.standard_normal((n, 3))
    err, K, f = orc.solid_evaluate(celltype, kinem, 210.0, 0.3, X, u)
    assert err == 0
    h = 1e-6
    for j in rng.choice(3 * n, size=6, replace=False):
        up = u.copy().reshape(-1)
        um = u.copy().reshape(-1)
        up[j] += h
        um[j] -= h
        _, _, fp = orc.solid_evaluate(celltype, kinem, 210.0, 0.3, X, up, want_k=False)
        _, _, fm = orc.solid_evaluate(celltype, kinem, 210.0, 0.3, X, um, want_k=False)
        fd = (fp - fm) / (2 * h)
        assert np.abs(fd - K[:, j]).max() <= 1e-6 * np.abs(K).max()
    assert np.abs(K - K.T).max() <= 1e-12 * np.abs(K).max()


def test_negative_nodal_jacobian_is_reported():
    par = np.array([[-1, -1, -1], [1, -1, -1], [1, 1, -1], [-1, 1, -1], [-1, -1, 1], [1, -1, 1],
                    [1, 1, 1], [-1, 1, 1]], dtype=float)
    X = par.copy()
    X[[0, 1]] = X[[1, 0]]  # swap two nodes -> inverted element
    err, _, _ = orc.solid_evaluate(orc.HEX8, orc.LINEAR, 210.0, 0.3, X, np.zeros((8, 3)))
    assert err == 1


# --------------------------------------------------------------------------- end-to-end
@pytest.mark.parametrize("name", ["solid_ele_hex8_Standard_linear.json",
                                  "solid_ele_hex27_Standard_linear.json",
                                  "sohex27_patchtest_nl_cost_drt.json",
                                  "solid_ele_hex8_Standard_eas_none_volume_neumann.json",
                                  "solid_ele_hex27_Standard_volume_neumann.json"])
def test_result_description(name):
    fx = load_fixture(name)
    prob = Problem(fx)
    t_end = float(fx["dynamic"].get("MAXTIME", 1.0))
    nstep = int(fx["dynamic"].get("NUMSTEP", 1))
    dt = float(fx["dynamic"].get("TIMESTEP", 1.0))
    t = min(t_end, nstep * dt)
    # the reference's load steps (statics: each step converged from the previous one)
    u = prob.solve_statics(t=t, nsteps=max(1, int(round(t / dt))))
    for r in fx["results"]:
        got = prob.disp(u, r["node"], r["dof"])
        assert abs(got - r["value"]) <= r["tol"], (r, got)


# --------------------------------------------------------------------------- TSI (config 5)
@pytest.mark.parametrize("name", ["tsi_heatflux_monolithic.json",
                                  "tsi_heatflux_flexoutsurf_monolithic.json"])
def test_tsi_result_description(name):
    """Static monolithic TSI (both fields statics, KINEM linear, ThermoStVenantKirchhoff + Fourier)
    through the oracle's SOLIDSCATRA and thermo element restatements."""
    fx = load_fixture(name)
    prob = TsiProblem(fx)
    d, T = prob.solve()
    for r in fx["results"]:
        got = prob.result(d, T, r)
        assert abs(got - r["value"]) <= r["tol"], (r, got)


@pytest.mark.parametrize("celltype", [orc.HEX8, orc.HEX27])
def test_tsi_tangent_blocks_are_derivatives(celltype):
    """k_ST = d f_S / dT, k_TT = d f_T / dT and k_TS = (1/dt) d f_T / dV by central differences on a
    distorted element (the blocks the GPU kernels reproduce)."""
    rng = np.random.default_rng(5)
    n = 8 if celltype == orc.HEX8 else 27
    X = orc.node_param_coords(celltype) * np.array([1.0, 0.7, 1.3]) + 0.05 * rng.standard_normal((n, 3))
    u = 1e-3 * rng.standard_normal((n, 3))
    T = 300.0 + 20.0 * rng.standard_normal(n)
    v = 1e-2 * rng.standard_normal((n, 3))
    E, nu, alpha, T0, k, dt = 210.0, 0.3, 1.2e-5, 293.0, 52.0, 0.5
    m = orc.st_modulus(E, nu, alpha)
    assert np.isclose(m, -(2 * E / (2 * (1 + nu)) + 3 * E * nu / ((1 + nu) * (1 - 2 * nu))) * alpha)
    _, _, _, Kst = orc.tsi_solid_evaluate(celltype, E, nu, alpha, T0, X, u, T)
    _, Ktt, _, Kts = orc.tsi_thermo_evaluate(celltype, k, m, X, T, v, 1.0, 1.0 / dt)
    h = 1e-3
    for j in range(n):
        e = np.zeros(n)
        e[j] = h
        fp = orc.tsi_solid_evaluate(celltype, E, nu, alpha, T0, X, u, T + e)[2]
        fm = orc.tsi_solid_evaluate(celltype, E, nu, alpha, T0, X, u, T - e)[2]
        np.testing.assert_allclose(Kst[:, j], (fp - fm) / (2 * h), rtol=1e-7, atol=1e-9 * abs(Kst).max())
        gp = orc.tsi_thermo_evaluate(celltype, k, m, X, T + e, v, 1.0, 1.0 / dt)[2]
        gm = orc.tsi_thermo_evaluate(celltype, k, m, X, T - e, v, 1.0, 1.0 / dt)[2]
        np.testing.assert_allclose(Ktt[:, j], (gp - gm) / (2 * h), rtol=1e-7, atol=1e-9 * abs(Ktt).max())
    hv = 1e-4
    for j in range(3 * n):
        e = np.zeros(3 * n)
        e[j] = hv
        gp = orc.tsi_thermo_evaluate(celltype, k, m, X, T, v + e.reshape(n, 3), 1.0, 1.0 / dt)[2]
        gm = orc.tsi_thermo_evaluate(celltype, k, m, X, T, v - e.reshape(n, 3), 1.0, 1.0 / dt)[2]
        # f_T is linear in v: the difference quotient is exact up to the rounding of f_T
        np.testing.assert_allclose(Kts[:, j], (gp - gm) / (2 * hv) / dt, rtol=1e-6,
                                   atol=1e-6 * abs(Kts).max())


# --------------------------------------------------------------------------- ElastHyper
def test_neohooke_cmat_is_stress_derivative():
    """cmat = dS/dE (strain-like Voigt: shear columns derive w.r.t. the engineering shear), S(0)=0,
    and the small-strain limit is StVK's cmat for the same E, nu."""
    E, nu = 10.0, 0.25
    gl = np.array([0.05, -0.02, 0.03, 0.04, -0.01, 0.02])
    S, C = orc.neohooke(E, nu, gl)
    h = 1e-6
    for j in range(6):
        e = np.zeros(6)
        e[j] = h
        Sp, _ = orc.neohooke(E, nu, gl + e)
        Sm, _ = orc.neohooke(E, nu, gl - e)
        np.testing.assert_allclose(C[:, j], (Sp - Sm) / (2 * h), rtol=1e-6, atol=1e-8)
    S0, C0 = orc.neohooke(E, nu, np.zeros(6))
    np.testing.assert_allclose(S0, 0.0, atol=1e-14)
    _, Cst = orc.stvk(E, nu, np.zeros(6))
    np.testing.assert_allclose(C0, Cst, rtol=1e-12, atol=1e-12)


# --------------------------------------------------------------------------- reactions, error, DOMAIN
import known_answers as ka  # noqa: E402


@pytest.mark.parametrize("name", ["patch_test_cube_linear_test_react.json",
                                  "patch_test_cube_h27_linear_test_react.json"])
def test_reaction_forces(name):
    """tests/input_files/patch_test_cube_*_linear_test_react.dat: displacements and the reaction
    forces (the reference's only direct pin on the assembled residual at Dirichlet rows), 1e-13."""
    fx = load_fixture(name)
    prob = Problem(fx)
    u = prob.solve_statics(t=1.0)
    for r in fx["results"]:
        assert abs(prob.disp(u, r["node"], r["dof"]) - r["value"]) <= r["tol"], r
    fr = ka.reactions(prob, u)
    assert ka.check_reactions(fx, prob, fr) == []
    assert len(fx["reactions"]) >= 4


def test_analytical_error_cantilever():
    """error_analytical_beam_cantilever_end_surface_load_with_poissons_effect.dat: the end-load
    cantilever (10 hex8, ten load steps), its RESULT DESCRIPTION (1e-10) and the L2-error CSV
    (CSV_COMPARISON_TOL_R 1e-10, _A 1e-12, list_of_tests.cmake:509)."""
    fx = load_fixture("error_analytical_beam_cantilever_end_surface_load_with_poissons_effect.json")
    prob = Problem(fx)
    u = prob.solve_statics(t=1.0, nsteps=10)
    for r in fx["results"]:
        assert abs(prob.disp(u, r["node"], r["dof"]) - r["value"]) <= r["tol"], r
    got = ka.analytical_error(fx, prob, u)
    ref = dict(zip(fx["csv_reference"]["columns"], fx["csv_reference"]["rows"][0]))
    tol = fx["csv_tolerance"]
    for k, v in zip(("displacement_error_l2_norm", "displacement_integral", "reference_volume"), got):
        assert abs(v - ref[k]) <= tol["atol"] + tol["rtol"] * abs(ref[k]), (k, v, ref[k])


@pytest.mark.parametrize("nranks", [1, 2])
def test_domain_altgeogeneration(nranks):
    """sohex8_disp_altgeogeneration.dat: STRUCTURE DOMAIN 3x3x3 hex8 TotLag on [0,4]^3 built by the
    GridGenerator restatement (fcg_box_mesh_create) at NP 1 and NP 2 (the reference runs NP 2),
    assembled by the oracle rank by rank; NODE 49 (GID 48, the corner (4,4,0) of the 7^3 lattice)
    dispx = 4.0 at 1e-14."""
    from parity_util import oracle_evaluate
    fx = load_fixture("sohex8_disp_altgeogeneration.json")
    meshes = ka.domain_meshes(fx, nranks)
    g48 = [m.node_x[list(m.node_gid).index(48)] for m in meshes if 48 in m.node_gid]
    np.testing.assert_allclose(g48[0], [4.0, 4.0, 0.0], atol=1e-14)
    E, nu = fx["material"]["young"], fx["material"]["nue"]

    def assemble(m, u):
        err, _, K, f = oracle_evaluate(m, orc.TOTLAG, E, nu, u)
        assert err == 0
        return K, f

    u = ka.domain_solve(fx, meshes, assemble)
    assert ka.check_domain_results(fx, u) == []


def test_singular_gauss_point_jacobian_oracle():
    """The hex27 element of tests/test_gpu_parity.py::SINGULAR_HEX27_X4 passes the nodal check
    (calc_lib.hpp:475-496) and hits det J == 0 at the centre Gauss point: invert3x3's throw
    (4C_linalg_fixedsizematrix.hpp:1394), error code 2."""
    from test_gpu_parity import SINGULAR_HEX27_X4
    X = np.array(SINGULAR_HEX27_X4, dtype=float) / 8.0
    for kin in (orc.LINEAR, orc.TOTLAG):
        assert orc.solid_evaluate(orc.HEX27, kin, 210.0, 0.3, X, np.zeros((27, 3)))[0] == 2
