"""bench.py's own rank launcher (tools/rank_launcher.py): `bench.py --gpus N` without an external
launcher starts N rank processes (the `mpirun -np N` of a 4C run), before anything touches the GPU.
CPU only: argument and environment plumbing, stdout routing, exit-code propagation."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import rank_launcher as rl  # noqa: E402


def test_plan_single_gpu_runs_in_process():
    assert rl.plan(["--steps", "3"], {}) == ("run", None)
    assert rl.plan(["--gpus", "1"], {}) == ("run", None)


def test_plan_spawns_without_launcher():
    assert rl.plan(["--gpus", "8", "--steps", "5"], {}) == ("spawn", 8)
    assert rl.plan(["--gpus=2"], {"OMP_NUM_THREADS": "16"}) == ("spawn", 2)


def test_plan_under_launcher_runs_and_checks_world():
    assert rl.plan(["--gpus", "4"], {"WORLD_SIZE": "4", "RANK": "2"}) == ("run", None)
    with pytest.raises(SystemExit) as e:
        rl.plan(["--gpus", "8"], {"WORLD_SIZE": "4"})
    assert "WORLD_SIZE=4" in str(e.value) and "--gpus 8" in str(e.value)
    with pytest.raises(SystemExit):
        rl.plan(["--gpus", "0"], {})


def test_rank_env_sets_and_replaces_rank_variables():
    base = {"PATH": "/bin", "RANK": "7", "MASTER_PORT": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    env = rl.rank_env(base, 3, 8, 29500)
    assert env["RANK"] == "3" and env["LOCAL_RANK"] == "3" and env["WORLD_SIZE"] == "8"
    assert env["LOCAL_WORLD_SIZE"] == "8" and env["GROUP_RANK"] == "0"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29500"
    assert env["PATH"] == "/bin" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert base["RANK"] == "7"


CHILD = textwrap.dedent("""
    import json, os, sys, time
    r = int(os.environ["RANK"])
    fail = os.environ.get("FAIL_RANK")
    if fail is not None and r == int(fail):
        sys.exit(3)
    if fail is not None:
        time.sleep(60)
    print(json.dumps({k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                                 "MASTER_ADDR", "MASTER_PORT")}))
""")


def _run_launcher(tmp_path, n, extra_env=None):
    child = tmp_path / "child.py"
    child.write_text(CHILD)
    drv = tmp_path / "drv.py"
    drv.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {os.path.join(ROOT, 'tools')!r})
        import rank_launcher
        sys.exit(rank_launcher.spawn([sys.executable, {str(child)!r}], {n}, grace_s=5.0))
    """))
    env = {k: v for k, v in os.environ.items() if k not in rl.RANK_VARS}
    env.update(extra_env or {})
    t = time.time()
    p = subprocess.run([sys.executable, str(drv)], capture_output=True, text=True, env=env,
                       timeout=60)
    return p, time.time() - t


def test_spawn_routes_rank0_stdout_and_sets_env(tmp_path):
    p, _ = _run_launcher(tmp_path, 4)
    assert p.returncode == 0, p.stderr
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1  # only rank 0 on stdout (bench.py's one JSON line)
    d = json.loads(lines[0])
    assert d["RANK"] == "0" and d["LOCAL_RANK"] == "0" and d["WORLD_SIZE"] == "4"
    assert d["MASTER_ADDR"] == "127.0.0.1" and int(d["MASTER_PORT"]) > 0
    others = [json.loads(l) for l in p.stderr.splitlines() if l.startswith("{")]
    assert sorted(int(o["RANK"]) for o in others) == [1, 2, 3]
    assert len({o["MASTER_PORT"] for o in others} | {d["MASTER_PORT"]}) == 1


def test_spawn_propagates_a_failing_rank_and_stops_the_others(tmp_path):
    p, wall = _run_launcher(tmp_path, 3, {"FAIL_RANK": "1"})
    assert p.returncode == 3
    assert "rank 1 exited with 3" in p.stderr
    assert wall < 30  # the sleeping ranks were terminated, not waited for


def test_bench_refuses_mismatched_world_before_importing_torch():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0")
    p = subprocess.run([sys.executable, "-X", "importtime", os.path.join(ROOT, "bench.py"),
                        "--gpus", "2"], capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=3" in p.stderr and "--gpus 2" in p.stderr
    assert "| torch" not in p.stderr  # failed before torch was imported


def test_sigterm_to_the_launcher_stops_every_rank(tmp_path):
    """A SIGTERM to the launcher (harness timeout) stops the ranks before it exits: no orphans."""
    import signal
    child = tmp_path / "child.py"
    child.write_text(textwrap.dedent(f"""
        import os, time
        open(os.path.join({str(tmp_path)!r}, "pid%s" % os.environ["RANK"]), "w").write(str(os.getpid()))
        time.sleep(120)
        """))
    launcher = tmp_path / "launch.py"
    launcher.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {os.path.join(ROOT, "tools")!r})
        import rank_launcher as rl
        sys.exit(rl.spawn([sys.executable, {str(child)!r}], 2, grace_s=5.0))
        """))
    p = subprocess.Popen([sys.executable, str(launcher)])
    t0 = time.time()
    while len(list(tmp_path.glob("pid*"))) < 2 and time.time() - t0 < 30:
        time.sleep(0.1)
    pids = [int((tmp_path / f"pid{r}").read_text()) for r in range(2)]
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    for pid in pids:
        t0 = time.time()
        while time.time() - t0 < 10:
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.1)
        else:
            raise AssertionError(f"rank process {pid} outlived the launcher")
