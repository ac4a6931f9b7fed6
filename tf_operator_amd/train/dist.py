"""Process-group bootstrap from the operator's env contract.

The operator (C++ core, ``torchenv`` / ``tfconfig`` generators) injects
``MASTER_ADDR``, ``MASTER_PORT``, ``WORLD_SIZE``, ``RANK``, ``LOCAL_RANK``,
``LOCAL_WORLD_SIZE`` (and ``TF_CONFIG`` for TFJob parity) into every replica;
``torchrun`` sets the same variables.  One process per GPU; backend
``nccl`` is RCCL on ROCm (xGMI inside a node), ``gloo`` for CPU plumbing.

Reference parity: SURVEY D7 (pytorch.go:13-68 env contract), P4.
"""
from __future__ import annotations

import atexit
import dataclasses
import datetime
import json
import os
import sys
import threading

import torch
import torch.distributed as dist


@dataclasses.dataclass
class DistInfo:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str | None


def env_rank_world():
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    tf = os.environ.get("TF_CONFIG")
    if tf:  # TF_CONFIG-only replica: chief/master first, then workers
        cfg = json.loads(tf)
        cluster, task = cfg.get("cluster", {}), cfg.get("task", {})
        order = [t for t in ("chief", "master", "worker") if t in cluster]
        rank, world = 0, 0
        for t in order:
            if t == task.get("type"):
                rank = world + int(task.get("index", 0))
            world += len(cluster[t])
        if task.get("type") in order:
            return rank, max(world, 1)
    return 0, 1


_DEVICE_CACHE: dict = {}


def local_device_index() -> int:
    """GPU this replica drives:

    * ``TOA_LOCAL_DEVICE`` when set (the local kubelet names the pod's device
      in its node-visible mode);
    * ``TOA_DEVICE_SOURCE=pod-resources`` (the operator's node-local layout,
      csrc/core/nodelocal.cc): the GPU the kubelet allocated to this pod, by
      PCI address (train/devices.py) -- never LOCAL_RANK, which on a node
      shared with other jobs would pick another job's GPU; raises if the
      kubelet cannot answer;
    * else ``LOCAL_RANK`` (torchrun; 0 under per-pod device pinning)."""
    v = os.environ.get("TOA_LOCAL_DEVICE")
    if v not in (None, ""):
        return int(v)
    if os.environ.get("TOA_DEVICE_SOURCE") == "pod-resources":
        if "idx" not in _DEVICE_CACHE:
            from . import devices

            _DEVICE_CACHE["idx"] = devices.allocated_device_index()
        return _DEVICE_CACHE["idx"]
    return int(os.environ.get("LOCAL_RANK", "0"))


def init(backend=None, timeout_s=1800) -> DistInfo:
    rank, world = env_rank_world()
    local_rank = local_device_index()
    use_cuda = torch.cuda.is_available() and not os.environ.get("TOA_NO_GPU")
    if use_cuda:
        torch.cuda.set_device(local_rank % max(torch.cuda.device_count(), 1))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    # TOA_DIST_BACKEND=gloo: several replicas sharing one GPU (RCCL refuses two
    # ranks on one device), e.g. restart benchmarks on a one-GPU box
    backend = backend or os.environ.get("TOA_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if use_cuda and backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        # a group still alive when the interpreter exits can abort in its
        # destructor ("terminate called without an active exception") and turn
        # a finished replica into a failed one: tear it down at exit --
        # gracefully after a clean run, by abort after an uncaught exception
        # (a graceful destroy can block on collectives a dead peer never
        # completes, and the operator would never see the failure)
        _install_failure_hook()
        atexit.register(_shutdown_quietly)
    return DistInfo(rank, world, local_rank, device, backend if world > 1 else None)


def barrier():
    if dist.is_initialized():
        if torch.cuda.is_available() and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_max(x: float, device) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()


_FAILED = []          # set by the excepthook: the interpreter is exiting on an uncaught exception
_EXIT_STATUS = []     # non-zero sys.exit() statuses (the excepthook does not see SystemExit)
EXIT_TEARDOWN_S = 20.0


def _install_failure_hook():
    prev = sys.excepthook
    if getattr(prev, "_toa_failure_hook", False):
        return

    def hook(tp, val, tb):
        _FAILED.append(tp)
        prev(tp, val, tb)

    hook._toa_failure_hook = True
    sys.excepthook = hook
    # sys.excepthook never sees SystemExit: a replica leaving by sys.exit(n)
    # with n != 0 (examples/dist_mnist.py) records n here, so its teardown
    # takes the failure path and a hung teardown still exits with n, not 0
    prev_exit = sys.exit

    def exit_(status=None):
        code = status if isinstance(status, int) else (0 if status is None else 1)
        if code:
            _EXIT_STATUS.append(code)
        prev_exit(status)

    sys.exit = exit_


def _bounded(fn, timeout: float) -> bool:
    """Run fn on a helper thread; False if it did not return in time."""
    t = threading.Thread(target=fn, name="toa-pg-teardown", daemon=True)
    t.start()
    t.join(timeout)
    return not t.is_alive()


def teardown(failed: bool = False, timeout: float | None = None) -> bool:
    """Bounded teardown of the process group; False if it did not finish in
    time (the caller then leaves with os._exit).  failed=False: graceful
    destroy.  failed=True: abort the group, no waiting on outstanding
    collectives a dead peer never completes."""
    if not dist.is_initialized():
        return True

    def graceful():
        try:
            shutdown()
        except Exception:  # pragma: no cover - a peer already gone
            pass

    def abort():
        try:
            dist.distributed_c10d._abort_process_group()
        except Exception:  # noqa: BLE001 - fall back to the graceful path, still bounded
            graceful()

    if timeout is None:
        timeout = EXIT_TEARDOWN_S if failed else 3 * EXIT_TEARDOWN_S
    return _bounded(abort if failed else graceful, timeout)


def _shutdown_quietly():
    """atexit teardown of the process group.  After a clean run: graceful
    destroy.  After an uncaught exception: abort the group (no waiting on
    outstanding collectives), and if even that does not return within
    EXIT_TEARDOWN_S, leave with status 1 right away, so a failed replica
    always exits non-zero and the operator can restart it."""
    if not dist.is_initialized():
        return
    if _FAILED or _EXIT_STATUS:
        status = _EXIT_STATUS[-1] if _EXIT_STATUS else 1
        if not teardown(failed=True):
            sys.stderr.write(f"[dist] process group teardown did not finish after a failure; exiting {status}\n")
            sys.stderr.flush()
            os._exit(status)
    elif not teardown(failed=False):
        sys.stderr.write("[dist] process group teardown hung after a clean run; exiting 0\n")
        sys.stderr.flush()
        os._exit(0)


def resolve_endpoint(addr: str) -> tuple[str, int]:
    """'svc.ns.svc[.domain]:port' -> (host, port).  On a real cluster DNS
    resolves the service name; under the local kubelet TOA_ENDPOINT_MAP maps
    it to 127.0.0.1:<allocated port>."""
    m = json.loads(os.environ.get("TOA_ENDPOINT_MAP", "{}") or "{}")
    addr = m.get(addr, addr)
    host, _, port = addr.rpartition(":")
    return host, int(port)


def own_port(default: int) -> int:
    """Port this replica should listen on (local kubelet sets PORT)."""
    return int(os.environ.get("PORT", default))
