"""BASELINE config 3 at its stated size: 1M hex27 (100^3), StVK TotLag, 24.4M DOFs and
4,625,301,609 stored nonzeros -- more than 2^31 and 2^32, so the CSR offsets of the tangent only
fit the int64 row pointers of the C ABI (fourc_gpu.h `rowptr`; a single-rank Epetra_CrsMatrix
would overflow its int32 offsets here).

* test_config3_rows_past_int32_offsets_against_oracle: one evaluate of the whole mesh on the
  device (K initialised to NaN, so any entry the library misses stays NaN), then the node rows
  whose CSR ranges straddle 2^31 and 2^32, and the first and last node rows, are rebuilt on the
  host from the oracle's element routine (orc_solid_evaluate: 4C_solid_3D_ele_calc.cpp:110-240 with
  calc_lib.hpp:579-605, 851-927) assembled the reference's way (owned rows, += at the row's
  sorted column position, 4C_linalg_sparsematrix.cpp:444-576) and compared at SURVEY §8d's
  tolerances; the whole K is checked finite and symmetric (x.Ky == y.Kx) on the device.
* The config-3 Newton loop at 100^3 itself is test_fullsize.py::test_config3_newton_equilibrium_
  and_symmetry[100].

FCG_CONFIG3_N overrides the size (>= 83 keeps nnz > 2^31)."""

import importlib
import os

import numpy as np
import pytest

import oracle_lib as orc

fcg = importlib.import_module("4c_amd").fcg
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
E, NU = 210.0, 0.3
N = int(os.environ.get("FCG_CONFIG3_N", "100"))


def _straddling_row(rowptr, offset):
    """The row whose CSR range [rowptr[r], rowptr[r+1]) contains `offset`."""
    return int(np.searchsorted(rowptr, offset, side="right") - 1)


@pytest.mark.parametrize("slab", [0, 5000])
def test_config3_rows_past_int32_offsets_against_oracle(monkeypatch, slab):
    """slab 5000: the slab schedule of the incidence records -- the records live in
    a ring of 1.18 GB instead of one 1,968-byte record per incidence (53 GB)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("FCG_H27_SLAB", str(slab))
    dev = torch.device("cuda:0")
    mesh = fcg.BoxMesh(fcg.HEX27, (N, N, N), jitter=0.02, seed=20251015)
    assert mesh.nnz > 2 ** 31
    if N == 100:
        assert mesh.nnz == 4_625_301_609 and mesh.n_rows == 24_361_803
    u = mesh.u_col(5e-2)
    ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
    if slab and N == 100:
        assert ev.info.scratch_bytes < 1.25e9, ev.info.scratch_bytes
    f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = torch.full((mesh.nnz,), float("nan"), dtype=torch.float64, device=dev)
    u_d = torch.from_numpy(u).to(dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u_d, f, K)
    torch.cuda.synchronize()
    assert not bool(torch.isnan(K).any()), "entries of K never written"
    # symmetry of the StVK TotLag tangent over the whole matrix (int64 offsets in the SpMV too)
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(mesh.n_rows, generator=g, dtype=torch.float64).to(dev)
    y = torch.randn(mesh.n_rows, generator=g, dtype=torch.float64).to(dev)
    Kx, Ky = torch.empty_like(x), torch.empty_like(y)
    ev.spmv(K, x, Kx)
    ev.spmv(K, y, Ky)
    a, b = float(torch.dot(x, Ky)), float(torch.dot(y, Kx))
    assert abs(a - b) <= 1e-12 * float(torch.linalg.vector_norm(x) * torch.linalg.vector_norm(Ky))
    del x, y, Kx, Ky

    rp = mesh.rowptr
    rows = {_straddling_row(rp, 2 ** 31), 0, mesh.n_rows - 1}
    if mesh.nnz > 2 ** 32:
        rows.add(_straddling_row(rp, 2 ** 32))
    node_of_row0 = {}
    for r0 in sorted({3 * (r // 3) for r in rows}):
        hit = np.nonzero(mesh.node_dof_row == r0)[0]
        assert len(hit) == 1
        node_of_row0[r0] = int(hit[0])
    straddle = [r for r in rows if rp[r] < 2 ** 31 < rp[r + 1] or rp[r] < 2 ** 32 < rp[r + 1]]
    assert straddle, "no row straddles 2^31"

    en = mesh.ele_nodes
    worst_k = worst_f = 0.0
    for r0, nd in sorted(node_of_row0.items()):
        ref = {d: np.zeros(int(rp[r0 + d + 1] - rp[r0 + d])) for d in range(3)}
        cols = {d: mesh.col_lid[rp[r0 + d]:rp[r0 + d + 1]] for d in range(3)}
        fref = np.zeros(3)
        eles, locs = np.nonzero(en == nd)
        assert 1 <= len(eles) <= 8
        for e, a_loc in zip(eles, locs):
            nodes = en[e]
            dof = mesh.node_dof_col[nodes]
            ue = np.stack([u[dof + k] for k in range(3)], axis=1)
            err, Ke, fe = orc.solid_evaluate(orc.HEX27, orc.TOTLAG, E, NU, mesh.node_x[nodes], ue)
            assert err == 0
            for d in range(3):
                lids = (dof[:, None] + np.arange(3)).ravel()  # element column order (3b + e)
                pos = np.searchsorted(cols[d], lids)
                assert np.array_equal(cols[d][pos], lids)
                np.add.at(ref[d], pos, Ke[3 * a_loc + d])
            fref += fe[3 * a_loc:3 * a_loc + 3]
        got_f = f[r0:r0 + 3].cpu().numpy()
        worst_f = max(worst_f, np.linalg.norm(got_f - fref) / np.linalg.norm(fref))
        for d in range(3):
            got = K[int(rp[r0 + d]):int(rp[r0 + d + 1])].cpu().numpy()
            dk = np.linalg.norm(got - ref[d]) / np.linalg.norm(ref[d])
            assert np.abs(got - ref[d]).max() <= 1e-12 * np.abs(ref[d]).max(), (r0 + d, dk)
            worst_k = max(worst_k, dk)
    assert worst_k <= 1e-12, worst_k
    assert worst_f <= 1e-10, worst_f
    ev.close()
