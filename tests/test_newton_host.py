"""Host-side pieces of the Newton path: the library's Neumann loads against the known-answer
driver (tests/fe_driver.py, whose fext reproduces the reference's RESULT values), and the CSR
built for reference input files.  CPU only."""
import json
import os

import numpy as np
import pytest

import fixture_problem as fp

GOLD = os.path.join(os.path.dirname(__file__), "golden")
NAMES = ["solid_ele_hex8_Standard_linear.json", "solid_ele_hex27_Standard_linear.json",
         "sohex27_patchtest_nl_cost_drt.json"]


@pytest.mark.parametrize("name", NAMES)
def test_neumann_matches_known_answer_driver(name):
    fx = json.load(open(os.path.join(GOLD, name)))
    prob = fp.problem(fx)
    t = fp.end_time(fx)
    ref = prob.fext(t)
    got = fp.fext(prob, t)
    assert np.abs(ref).max() > 0
    np.testing.assert_allclose(got, ref, rtol=1e-14, atol=1e-14 * np.abs(ref).max())


@pytest.mark.parametrize("name", NAMES)
def test_fixture_csr_covers_element_couplings(name):
    fx = json.load(open(os.path.join(GOLD, name)))
    prob = fp.problem(fx)
    dis = fp.discretization(prob)
    rows = np.repeat(np.arange(dis.n_rows), np.diff(dis.rowptr))
    pairs = set(zip(rows.tolist(), dis.col_lid.tolist()))
    for el in dis.ele_nodes:
        dofs = [3 * n + d for n in el for d in range(3)]
        for a in dofs:
            for b in dofs:
                assert (a, b) in pairs
    for r in range(dis.n_rows):
        c = dis.col_lid[dis.rowptr[r]:dis.rowptr[r + 1]]
        assert np.all(np.diff(c) > 0)


def test_forcing_term_sequence():
    """newton.ForcingTerm against hand-evaluated Eisenstat-Walker steps (NOX InexactNewton)."""
    import importlib
    import math
    newton = importlib.import_module("4c_amd.newton")
    ft = newton.ForcingTerm("Constant", constant=1e-8)
    assert ft.compute(0, 1.0) == 1e-8 and ft.compute(3, 1e-3, 1e-2, 1e-4) == 1e-8
    t2 = newton.ForcingTerm("Type 2")
    assert t2.compute(0, 1.0) == 0.1                            # initial, unclamped
    # 0.9 (0.5)^1.5 = 0.318; safeguard 0.9 * 0.1^1.5 = 0.028 < 0.1; clamp to max 0.01
    assert t2.compute(1, 0.5, 1.0) == 0.01
    # 0.9 (1e-3)^1.5 = 2.85e-5; safeguard 0.9 * 0.01^1.5 = 9e-4 < 0.1 -> 2.85e-5
    assert math.isclose(t2.compute(2, 1e-3, 1.0), 0.9 * 1e-3 ** 1.5, rel_tol=1e-15)
    assert t2.compute(3, 1e-9, 1.0) == 1e-6                     # clamp to min
    big = newton.ForcingTerm("Type 2", maximum=0.9)
    big.compute(0, 1.0)
    big.eta = 0.8                                               # safeguard 0.9 * 0.8^1.5 = 0.644 > 0.1
    assert math.isclose(big.compute(1, 1e-4, 1.0), 0.9 * 0.8 ** 1.5, rel_tol=1e-15)
    t1 = newton.ForcingTerm("Type 1")
    assert t1.compute(0, 2.0) == 0.1
    # |0.5 - 0.498| / 2 = 1e-3; safeguard 0.1^1.618 = 0.024 < 0.1
    assert math.isclose(t1.compute(1, 0.5, 2.0, 0.498), 1e-3, rel_tol=1e-12)
    with pytest.raises(ValueError):
        newton.ForcingTerm("Type 3")


def test_accept_linear_solve_rescue_rules():
    """newton.accept_linear_solve: NOX's Rescue Bad Newton Solve decision, host logic only."""
    import importlib
    import math
    import warnings
    newton = importlib.import_module("4c_amd.newton")
    mg = importlib.import_module("4c_amd.multigrid")
    rec = {}
    assert newton.accept_linear_solve(lambda: (5, 1e-12), 1e-10, 0, True, rec) == (5, 1e-12)
    assert "lin_rescued" not in rec
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert newton.accept_linear_solve(lambda: (25, 1e-3), 1e-10, 1, True, rec) == (25, 1e-3)
    assert rec["lin_rescued"] and "Rescue Bad Newton Solve" in str(w[0].message)
    with pytest.raises(RuntimeError):
        newton.accept_linear_solve(lambda: (25, 1e-3), 1e-10, 1, False, {})
    with pytest.raises(RuntimeError):
        newton.accept_linear_solve(lambda: (25, math.nan), 1e-10, 1, True, {})

    def mg_fail(relres):
        def f():
            raise mg.MultigridError("stopped", 30 if relres else None, relres)
        return f
    rec = {}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        assert newton.accept_linear_solve(mg_fail(2e-9), 1e-10, 2, True, rec) == (30, 2e-9)
    assert rec["lin_rescued"]
    with pytest.raises(mg.MultigridError):
        newton.accept_linear_solve(mg_fail(None), 1e-10, 2, True, {})  # indefinite: no direction
    with pytest.raises(mg.MultigridError):
        newton.accept_linear_solve(mg_fail(2e-9), 1e-10, 2, False, {})
