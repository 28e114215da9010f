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
