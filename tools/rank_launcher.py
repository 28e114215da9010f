"""One process per GPU for `bench.py --gpus N` without an external launcher.

The driver may run `python bench.py --gpus N` directly or under `torch.distributed.run`.  In the
first case WORLD_SIZE is unset and this module starts the N ranks itself, the way `mpirun -np N`
starts 4C's ranks over the GridGenerator box split (4C_io_gridgenerator.cpp:87-153): N child
processes of the same command with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set.  The parent never touches the GPU (it runs before torch is
imported) and never execs: it waits for the children and exits with the first non-zero exit code
(the other ranks are then terminated, since they would wait forever in a collective).  Rank 0's
stdout is the parent's stdout (bench.py's one JSON line); the other ranks' stdout goes to stderr.

Standard library only, so that bench.py can call it before any import that could initialise HIP.
"""
import argparse
import os
import signal
import socket
import subprocess
import sys
import time

RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
             "MASTER_ADDR", "MASTER_PORT")


class LaunchError(SystemExit):
    pass


def requested_gpus(argv):
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args(argv)
    return a.gpus


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base, rank, world, port):
    """The environment of rank `rank` of a single-node job of `world` ranks."""
    env = {k: v for k, v in base.items() if k not in RANK_VARS}
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    return env


def plan(argv, environ):
    """('run', None): this process is a rank (or the only one); ('spawn', N): start N ranks.
    Raises LaunchError when the environment and --gpus disagree."""
    n = requested_gpus(argv)
    if n < 1:
        raise LaunchError(f"bench.py: --gpus {n}: at least one GPU")
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != n:
            raise LaunchError(f"bench.py: WORLD_SIZE={ws} from the launcher but --gpus {n}; "
                              f"they must agree")
        return "run", None
    return ("spawn", n) if n > 1 else ("run", None)


class _Signalled(Exception):
    def __init__(self, signum):
        super().__init__(signum)
        self.signum = signum


def _raise_signal(signum, _frame):
    raise _Signalled(signum)


def spawn(cmd, n, environ=None, poll_s=0.2, grace_s=20.0):
    """Run `cmd` as ranks 0..n-1; return the job's exit code (0, or the first failure's).
    A SIGTERM / SIGINT to the launcher (a harness timeout, another launcher stopping the job)
    stops every rank first -- children left behind would hold their GPUs, possibly blocked in a
    collective -- and then returns 128 + the signal number."""
    environ = dict(os.environ if environ is None else environ)
    port = free_port()
    procs = []
    old = {}
    try:
        for sig in (signal.SIGTERM, signal.SIGINT):
            old[sig] = signal.signal(sig, _raise_signal)
    except ValueError:  # not the main thread: no handlers, the finally below still stops ranks
        pass
    try:
        for r in range(n):
            out = None if r == 0 else sys.stderr.fileno()
            procs.append(subprocess.Popen(cmd, env=rank_env(environ, r, n, port), stdout=out))
        rc = 0
        live = set(range(n))
        while live:
            for r in sorted(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.discard(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print(f"rank_launcher: rank {r} exited with {c}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    _stop([procs[q] for q in live], grace_s)
            if live:
                time.sleep(poll_s)
        return rc
    except _Signalled as e:
        # a second signal must not interrupt the clean-up either
        for sig in old:
            signal.signal(sig, signal.SIG_IGN)
        print(f"rank_launcher: signal {e.signum}; stopping the ranks", file=sys.stderr, flush=True)
        _stop([p for p in procs if p.poll() is None], grace_s)
        return 128 + e.signum
    finally:
        # no second signal may interrupt the clean-up
        for sig in old:
            signal.signal(sig, signal.SIG_IGN)
        _stop([p for p in procs if p.poll() is None], grace_s)
        for sig, h in old.items():
            signal.signal(sig, h)


def _stop(procs, grace_s):
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t = time.time() + grace_s
    for p in procs:
        try:
            p.wait(max(0.1, t - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def run_or_spawn(argv, script):
    """Called by bench.py at import time, before torch: returns if this process runs the bench,
    else starts the ranks and exits with the job's code."""
    what, n = plan(argv[1:], os.environ)
    if what == "run":
        return
    rc = spawn([sys.executable, script] + list(argv[1:]), n)
    sys.exit(rc)
