"""The node-row gather path (FCG_PATH_GATHER, unstructured hex8) on a reference input mesh tiled
and jittered: the 10-element beam of error_analytical_beam_cantilever_end_surface_load_with_
poissons_effect.dat repeated into a block, coincident nodes merged, interior nodes moved, node and
element numbering shuffled (parity_util.tiled_input_mesh).  K and f_int against the oracle on the
same discretization, for both kinematics, plus ACCUMULATE and the internal-force action."""

import importlib

import numpy as np
import pytest

from parity_util import oracle_evaluate_single, rel_err, tiled_input_mesh
from test_oracle_known_answers import load_fixture

fcg = importlib.import_module("4c_amd").fcg
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
E, NU = 210.0, 0.3
FX = "error_analytical_beam_cantilever_end_surface_load_with_poissons_effect.json"


def _run(dis, kinem, u, action=fcg.CALC_NLNSTIFF, mode=fcg.OVERWRITE, path=fcg.PATH_GATHER, K0=None, f0=None):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda:0")
    ev = fcg.Evaluator(dis, kinematics=kinem, youngs=E, poisson=NU, path=path)
    # AUTO: the gather path, or the sweep when fcg_create finds a lattice in the connectivity
    assert ev.info.path == fcg.PATH_GATHER or (path == fcg.PATH_AUTO and ev.info.path == fcg.PATH_STRUCTURED)
    f = torch.from_numpy(f0.copy()).to(dev) if f0 is not None else torch.zeros(dis.n_rows, dtype=torch.float64, device=dev)
    K = None
    if action == fcg.CALC_NLNSTIFF:
        K = (torch.from_numpy(K0.copy()).to(dev) if K0 is not None
             else torch.full((dis.nnz,), float("nan"), dtype=torch.float64, device=dev))
    ev.evaluate_device(action, mode, torch.from_numpy(u).to(dev), f, K)
    torch.cuda.synchronize()
    out = (K.cpu().numpy() if K is not None else None), f.cpu().numpy()
    ev.close()
    return out


@pytest.mark.parametrize("kinem,amp", [(fcg.LINEAR, 1e-3), (fcg.TOTLAG, 5e-2)])
@pytest.mark.parametrize("reps", [(3, 4, 2), (12, 12, 3)])
def test_tiled_reference_mesh_gather_matches_oracle(kinem, amp, reps):
    dis = tiled_input_mesh(load_fixture(FX), reps, jitter=0.15, seed=sum(reps))
    u = np.random.default_rng(5).standard_normal(dis.n_cols) * amp
    err, _, Kr, fr = oracle_evaluate_single(dis, kinem, E, NU, u, nworkers=8)
    assert err == 0
    for path in (fcg.PATH_GATHER, fcg.PATH_AUTO):
        Kg, fg = _run(dis, kinem, u, path=path)
        assert np.all(np.isfinite(Kg))
        assert rel_err(fg, fr) <= 1e-10, rel_err(fg, fr)
        assert rel_err(Kg, Kr) <= 1e-12, rel_err(Kg, Kr)
        assert np.abs(Kg - Kr).max() <= 1e-12 * np.abs(Kr).max()
    _, fi = _run(dis, kinem, u, action=fcg.CALC_INTERNALFORCE)
    assert rel_err(fi, fr) <= 1e-10
    rng = np.random.default_rng(1)
    K0, f0 = rng.standard_normal(dis.nnz), rng.standard_normal(dis.n_rows)
    Ka, fa = _run(dis, kinem, u, mode=fcg.ACCUMULATE, K0=K0, f0=f0)
    np.testing.assert_allclose(Ka, K0 + Kr, rtol=0, atol=1e-11 * np.abs(Kr).max())
    np.testing.assert_allclose(fa, f0 + fr, rtol=0, atol=1e-9 * max(np.abs(fr).max(), 1.0))
