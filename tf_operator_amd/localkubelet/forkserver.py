"""Warm-interpreter fork server for the local kubelet.

Half of BASELINE's headline metric is submit -> first-step latency, and on
one MI355X box about 1.8 s of a 3 s Llama-3-8B job start is the replica's
``import torch`` (``profiles``/BASELINE.md breakdown).  A node that runs
many short or restarting replicas can pay that once: this server imports
torch up front -- WITHOUT touching the GPU (no HIP
call, no HIP kernel library loaded: the HIP runtime must initialise in the
child, after ``HIP_VISIBLE_DEVICES`` is set) -- and forks one child per
container start.  The child takes the container's environment, working
directory and log file, then runs ``python -m module`` / ``python -c code``
/ ``python script.py`` in-process (runpy); nothing is exec'd.

Protocol (JSON lines on stdin / stdout, single-threaded so the fork never
copies a lock held by another thread):

    -> {"id": n, "argv": ["-m", "pkg.mod", ...], "env": {...}, "cwd": d, "log": path}
    <- {"id": n, "pid": pid}            (or {"id": n, "error": "..."})
    <- {"exit": pid, "status": code}    when a child ends (signal N -> -N)

The kubelet falls back to a cold ``subprocess`` start for anything that is
not a Python command line, or when the server is not running.
"""
from __future__ import annotations

import json
import os
import runpy
import select
import signal
import sys
import traceback

# third-party modules only: this package's modules read TOA_* settings at
# import time, and those must come from the container's env, not the server's
PRELOAD = ("torch", "torch.distributed", "torch.nn.functional", "numpy")


def _preload():
    import importlib

    for m in PRELOAD:
        try:
            importlib.import_module(m)
        except Exception as e:  # pragma: no cover - the cold path still works
            print(f"[forkserver] preload {m} failed: {e}", file=sys.stderr, flush=True)


def _run_child(req):
    """In the forked child: become the container process."""
    os.setsid()
    fd = os.open(req["log"], os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644)
    os.dup2(fd, 1)
    os.dup2(fd, 2)
    os.close(fd)
    nul = os.open(os.devnull, os.O_RDONLY)
    os.dup2(nul, 0)
    os.close(nul)
    # fresh stdio objects: never inherit the server's buffers or their locks
    sys.stdin = open(0, "r", closefd=False)
    sys.stdout = open(1, "w", buffering=1, closefd=False)
    sys.stderr = open(2, "w", buffering=1, closefd=False)
    for s in (signal.SIGTERM, signal.SIGINT, signal.SIGCHLD):
        signal.signal(s, signal.SIG_DFL)
    env = req["env"]
    os.environ.clear()
    os.environ.update(env)
    os.chdir(req["cwd"])
    extra = [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p]
    sys.path[:0] = [p for p in extra if p not in sys.path]
    if env.get("OMP_NUM_THREADS", "").isdigit():
        import torch

        torch.set_num_threads(int(env["OMP_NUM_THREADS"]))
    argv = list(req["argv"])
    code = 0
    try:
        if argv and argv[0] == "-m":
            sys.argv = argv[1:]
            sys.path.insert(0, req["cwd"])
            runpy.run_module(argv[1], run_name="__main__", alter_sys=True)
        elif argv and argv[0] == "-c":
            sys.argv = ["-c"] + argv[2:]
            exec(compile(argv[1], "<string>", "exec"), {"__name__": "__main__"})
        else:
            sys.argv = argv
            sys.path.insert(0, os.path.dirname(os.path.abspath(argv[0])))
            runpy.run_path(argv[0], run_name="__main__")
    except SystemExit as e:
        c = e.code
        code = 0 if c is None else (c if isinstance(c, int) else 1)
        if not isinstance(c, (int, type(None))):
            print(c, file=sys.stderr)
    except BaseException:  # noqa: BLE001 - a container's uncaught exception
        traceback.print_exc()
        code = 1
    try:
        sys.stdout.flush()
        sys.stderr.flush()
    finally:
        os._exit(code & 0xFF)


def serve(inp=None, out=None):
    inp = inp or sys.stdin.buffer
    out = out or sys.stdout
    _preload()
    print(json.dumps({"ready": os.getpid()}), file=out, flush=True)
    buf = b""
    fd = inp.fileno()
    while True:
        r, _, _ = select.select([fd], [], [], 0.002)
        if r:
            chunk = os.read(fd, 65536)
            if not chunk:  # the kubelet went away
                break
            buf += chunk
            while b"\n" in buf:
                line, buf = buf.split(b"\n", 1)
                if not line.strip():
                    continue
                req = json.loads(line)
                try:
                    pid = os.fork()
                except OSError as e:
                    print(json.dumps({"id": req.get("id"), "error": str(e)}), file=out, flush=True)
                    continue
                if pid == 0:
                    _run_child(req)  # never returns
                print(json.dumps({"id": req.get("id"), "pid": pid}), file=out, flush=True)
        while True:  # reap
            try:
                pid, status = os.waitpid(-1, os.WNOHANG)
            except ChildProcessError:
                break
            if pid == 0:
                break
            print(json.dumps({"exit": pid, "status": os.waitstatus_to_exitcode(status)}), file=out, flush=True)


if __name__ == "__main__":
    serve()
