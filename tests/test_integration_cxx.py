"""The INTEGRATION.md C++ binding, compiled (tests/cxx/integration_4c.cpp, built by
__graft_entry__.build() / `make -C tests/cxx`) and run: on the CPU it must build, link against
libfourc_gpu.so and report fcg_create's device error cleanly; on the GPU every rank of a 2-rank
GridGenerator box evaluates through fcg_evaluate and through the C++ facade
(fourc_gpu::Discretization::evaluate with a ParameterList action) and matches the oracle."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CXX = os.path.join(ROOT, "tests", "cxx")
BIN = os.path.join(CXX, "_build", "integration_4c")


def _binary():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", CXX], check=True)
    return BIN


def test_integration_builds_and_reports_missing_device():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the device run is the gpu test")
    p = subprocess.run([_binary(), "--expect-no-device"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASS" in p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["6", "5", "4", "2"], ["9", "7", "8", "3"], ["5", "5", "5", "1"]])
def test_integration_on_device(args):
    p = subprocess.run([_binary()] + args, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASS" in p.stdout, p.stdout


NATIVE = os.path.join(CXX, "_build", "config3_native")


@pytest.mark.gpu
@pytest.mark.parametrize("n,ranks,dist", [(8, 2, "auto"), (40, 2, "auto"), (32, 4, "auto"), (40, 2, "1"),
                                          (32, 4, "1"), (40, 2, "deep"), (32, 4, "deep")])
def test_config3_native_cxx_host(n, ranks, dist):
    """BASELINE config 3's problem (hex27 StVK TotLag cube, x- clamped, traction -1 on x+) solved by
    a C++ host through the C ABI alone (tests/cxx/config3_native.cpp): Newton with fcg_dfcg_solve
    and each rank's fcg_amg; ranks as threads with a host exchange on one GPU.  1 rank and `ranks`
    ranks converge quadratically to the same displacement by DOF GID (n = 40: config 3 at 40^3)
    within 1.5x the 1-rank FCG iterations.  dist "1": the AMG's level 1 distributed across the
    ranks (FCG_AMG_DIST=1; the host transport's exchange_fn) -- each rank then stores only its own
    level-1 rows and all-reduces only level 2.  dist "deep": every coarser level that still shrinks
    distributed too (FCG_AMG_DIST_MIN=0) -- at least two distributed levels, a replicated level
    smaller than level 2, the same 1.5x iteration bound."""
    if not os.path.exists(NATIVE):
        subprocess.run(["make", "-s", "-C", CXX], check=True)
    env = dict(os.environ)
    if dist == "deep":
        env.update(FCG_AMG_DIST="1", FCG_AMG_DIST_MIN="0")
    elif dist != "auto":
        env["FCG_AMG_DIST"] = dist
    p = subprocess.run([NATIVE, str(n), str(ranks)], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASS" in p.stdout, p.stdout
    stats = [[int(v) for v in line.split(":")[1].split()] for line in p.stdout.splitlines()
             if line.startswith("coupled AMG rank")]
    assert len(stats) == ranks, p.stdout
    print(p.stdout)
    if dist == "deep":
        glob = stats[0][2]
        assert all(st[0] >= 2 and st[0] == stats[0][0] for st in stats), p.stdout
        assert sum(st[1] for st in stats) == glob, p.stdout
        assert all(st[8] * 6 == st[4] for st in stats), p.stdout  # the replicated level all-reduced
    if dist == "1":
        glob = stats[0][2]
        assert all(st[0] == 1 for st in stats), p.stdout
        assert sum(st[1] for st in stats) == glob, p.stdout  # each level-1 row on one rank
        assert all(st[4] < 6 * glob for st in stats), p.stdout  # level 2 all-reduced, not level 1


@pytest.mark.gpu
@pytest.mark.parametrize("n,ranks,at", [(16, 2, 0), (16, 2, 4), (16, 4, 2), (16, 4, 9)])
def test_config3_native_failure_inside_the_amg_build(n, ranks, at):
    """Thread transport (tests/cxx/config3_native.cpp `inject`): rank 1 throws inside the coupled
    AMG build at its at-th collective (FCG_AMG_INJECT_BUILD_FAIL, level 1 distributed); the host
    never releases the other ranks' barriers, so a rank left inside a collective would hang until
    the timeout -- every rank's fcg_dfcg_solve must return an error instead."""
    if not os.path.exists(NATIVE):
        subprocess.run(["make", "-s", "-C", CXX], check=True)
    env = dict(os.environ, FCG_AMG_DIST="1", FCG_AMG_INJECT_BUILD_FAIL=f"1:{at}")
    p = subprocess.run([NATIVE, str(n), str(ranks), "inject"], capture_output=True, text=True,
                       timeout=120, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASS" in p.stdout, p.stdout
