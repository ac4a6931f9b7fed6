"""A failing replica must exit non-zero promptly (train/dist.py):
the atexit teardown aborts the process group after an uncaught exception
instead of blocking on collectives a dead peer never completes.  gloo,
world 2, CPU."""
import os
import socket
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import os, sys, time
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    from tf_operator_amd.train import dist as tdist
    info = tdist.init(backend="gloo")
    x = torch.ones(1 << 16)
    for step in range(10_000):
        dist.all_reduce(x)
        x.fill_(1.0)
        if info.rank == 1 and step == 20:
            raise RuntimeError("replica 1 fails mid-step")
    print("finished", flush=True)
""")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(script, world, port):
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TOA_NO_GPU="1")
        procs.append(subprocess.Popen([sys.executable, "-c", script], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    return procs


def test_peer_failure_exits_every_rank_nonzero_quickly():
    procs = _launch(SCRIPT.format(root=ROOT), 2, _port())
    t0 = time.time()
    codes = []
    try:
        for p in procs:
            codes.append(p.wait(timeout=90))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    logs = [p.stdout.read() for p in procs]
    assert all(c != 0 for c in codes), (codes, logs)
    assert "replica 1 fails mid-step" in logs[1]
    assert elapsed < 80, elapsed


def test_clean_run_exits_zero():
    script = SCRIPT.format(root=ROOT).replace("step == 20", "step == -1").replace("range(10_000)", "range(30)")
    procs = _launch(script, 2, _port())
    codes = [p.wait(timeout=90) for p in procs]
    assert codes == [0, 0], [p.stdout.read() for p in procs]


def test_sys_exit_status_survives_a_hung_teardown():
    """sys.exit(3) does not reach sys.excepthook: the status is
    recorded, the teardown takes the failure path, and if even that hangs
    the replica leaves with 3 -- never 0, which would hide the failure from
    the operator.  The hang is forced by a process-group abort that blocks."""
    script = textwrap.dedent("""
        import sys, time
        sys.path.insert(0, {root!r})
        import torch.distributed as dist
        from tf_operator_amd.train import dist as tdist
        tdist.init(backend="gloo")
        tdist.EXIT_TEARDOWN_S = 1.0
        dist.distributed_c10d._abort_process_group = lambda *a, **k: time.sleep(60)
        sys.exit(3)
    """).format(root=ROOT)
    procs = _launch(script, 2, _port())
    t0 = time.time()
    codes = [p.wait(timeout=60) for p in procs]
    assert codes == [3, 3], [p.stdout.read() for p in procs]
    assert time.time() - t0 < 45
