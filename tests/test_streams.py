"""Stream ordering between torch's default stream and a context's own stream (regression test of
the round-1 race: a library call on the context stream ran before the torch work that produced its
input had finished, seen as a sporadically corrupted coarse-level matrix).  The contexts create
blocking streams, which the legacy default stream orders both ways: torch work queued before a
library call on the context stream (stream = NULL) finishes first, and torch work queued after it
starts after it.  A GPU spin in front makes the wrong order observable: without the ordering the
library would read x before the copy behind the spin lands."""

import ctypes
import importlib

import numpy as np
import pytest

fcg = importlib.import_module("4c_amd").fcg
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


@pytest.fixture(scope="module")
def system():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda:0")
    mesh = fcg.BoxMesh(fcg.HEX8, (40, 40, 40), jitter=0.1)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=210.0, poisson=0.3)
    f64 = dict(dtype=torch.float64, device=dev)
    K = torch.empty(mesh.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(mesh.n_cols, **f64),
                       torch.zeros(mesh.n_rows, **f64), K)
    torch.cuda.synchronize()
    yield mesh, ev, K, dev
    ev.close()


def test_library_call_on_context_stream_waits_for_torch(system):
    mesh, ev, K, dev = system
    n = mesh.n_rows
    x_new = torch.from_numpy(np.random.default_rng(1).standard_normal(n)).to(dev)
    ref = torch.empty_like(x_new)
    ev.spmv(K, x_new, ref)  # torch's stream
    torch.cuda.synchronize()
    for _ in range(3):
        x = torch.zeros(n, dtype=torch.float64, device=dev)
        y = torch.full((n,), float("nan"), dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        torch.cuda._sleep(50_000_000)  # ~20 ms spin on torch's default stream
        x.copy_(x_new)                  # lands after the spin
        rc = fcg.lib().fcg_spmv(ev._h, _p(K), _p(x), _p(y), None)  # the context's own stream
        assert rc == 0
        torch.cuda.synchronize()
        assert torch.equal(y, ref)


def test_torch_work_after_a_library_call_waits_for_it(system):
    mesh, ev, K, dev = system
    n = mesh.n_rows
    x = torch.from_numpy(np.random.default_rng(2).standard_normal(n)).to(dev)
    ref = torch.empty_like(x)
    ev.spmv(K, x, ref)
    torch.cuda.synchronize()
    ref_sum = float(ref.sum())
    for _ in range(3):
        y = torch.zeros(n, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        # twenty operator applications queued on the context stream: torch's sum must follow them
        for _ in range(20):
            assert fcg.lib().fcg_spmv(ev._h, _p(K), _p(x), _p(y), None) == 0
        s = y.sum()  # torch's default stream
        assert float(s) == ref_sum
