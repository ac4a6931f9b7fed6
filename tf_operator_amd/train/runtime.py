"""Replica-side runtime shared by the bundled trainers: rendezvous from the
operator's env contract, first-step / throughput reporting back to the
operator (BASELINE metric "submit -> first-step latency"), preemption
handling (SIGTERM -> checkpoint -> exit 143, a retryable code for the
ExitCode / elastic restart policies), and the role of this replica
(chief/worker/ps/evaluator)."""
from __future__ import annotations

import contextlib
import json
import os
import signal
import threading
import time
import urllib.request

from . import dist as tdist

# a lost peer (broken collective) exits with a retryable code (>= 128), so
# ExitCode / elastic policies restart the group instead of failing the job
PEER_LOST_EXIT = 143
_PEER_MARKERS = ("Connection closed by peer", "Connection reset by peer", "Broken pipe", "NCCL", "RCCL",
                 "Socket Timeout", "ProcessGroup", "gloo")


def is_peer_failure(e: BaseException) -> bool:
    try:
        import torch.distributed as d

        if isinstance(e, d.DistError):
            return True
    except Exception:  # pragma: no cover - torch without distributed
        pass
    return isinstance(e, (RuntimeError, ConnectionError)) and any(m in str(e) for m in _PEER_MARKERS)


def process_start_time() -> float | None:
    """Wall-clock start of this process (Linux /proc), None if unknown."""
    try:
        with open("/proc/self/stat") as f:
            ticks = int(f.read().rsplit(")", 1)[1].split()[19])
        # boot time from the clocks, not /proc/stat's whole-second btime (that
        # one is up to 1 s off, which swamped the sub-second start-up phases)
        boot = time.time() - time.clock_gettime(time.CLOCK_BOOTTIME)
        return boot + ticks / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError, IndexError):
        return None


class Runtime:
    def __init__(self, backend=None):
        self.role = os.environ.get("TOA_ROLE") or os.environ.get("TOA_REPLICA_TYPE") or "worker"
        self.job = os.environ.get("TOA_JOB_NAME", "")
        self.namespace = os.environ.get("TOA_JOB_NAMESPACE", "default")
        self.kind = os.environ.get("TOA_JOB_KIND", "TFJob")
        self.report_url = os.environ.get("TOA_REPORT_URL")
        self.ckpt_dir = os.environ.get("TOA_CHECKPOINT_DIR")
        self.preempted = threading.Event()
        self._first_reported = False
        self.t_start = time.time()
        self.phases: dict[str, float] = {}
        self.info = None
        self.backend = backend

    # -------------------------------------------------------------- dist
    def init_dist(self):
        self.info = tdist.init(self.backend)
        return self.info

    @property
    def rank(self):
        return self.info.rank if self.info else 0

    @property
    def world(self):
        return self.info.world if self.info else 1

    @property
    def is_chief(self):
        return self.rank == 0

    @contextlib.contextmanager
    def guard(self):
        """Wrap a training loop: a collective that fails because a peer died
        ends this replica with PEER_LOST_EXIT (no hang in process-group
        teardown) so the operator restarts the whole group."""
        try:
            yield
        except Exception as e:
            if self.info is not None and self.info.world > 1 and is_peer_failure(e):
                self.log(f"lost a peer ({type(e).__name__}: {str(e)[:200]}); exiting {PEER_LOST_EXIT}")
                os._exit(PEER_LOST_EXIT)
            raise
        # normal end: tear the process group down before interpreter exit
        # (a live gloo/RCCL group at exit can abort: "terminate called
        # without an active exception")
        tdist.shutdown()

    # -------------------------------------------------------------- preemption
    def install_preemption_handler(self):
        def _h(signum, frame):
            self.preempted.set()

        try:
            signal.signal(signal.SIGTERM, _h)
        except ValueError:  # not the main thread
            pass

    # -------------------------------------------------------------- reporting
    def report(self, **kw):
        if not self.report_url or not self.is_chief:
            return
        body = {"job": self.job, "namespace": self.namespace, "kind": self.kind,
                "elastic_generation": int(os.environ.get("TOA_ELASTIC_GENERATION", "0") or 0), **kw}
        try:
            req = urllib.request.Request(self.report_url, data=json.dumps(body).encode(),
                                         headers={"Content-Type": "application/json"}, method="POST")
            urllib.request.urlopen(req, timeout=2).read()
        except Exception:
            pass  # reporting is best effort

    def mark(self, phase: str):
        """Record a start-up phase (for the submit -> first-step breakdown)."""
        self.phases[phase] = time.time()

    def first_step_done(self):
        if not self._first_reported:
            self._first_reported = True
            now = time.time()
            t0 = process_start_time() or self.t_start
            marks = {"process_start": t0, "runtime": self.t_start, **self.phases, "first_step": now}
            order = sorted(marks.items(), key=lambda kv: kv[1])
            phases = {f"{a}->{b}": round(tb - ta, 4) for (a, ta), (b, tb) in zip(order, order[1:])}
            if os.environ.get("TOA_LOG_PHASES", "1") == "1" and self.is_chief:
                self.log("start-up phases (s): " + ", ".join(f"{k} {v}" for k, v in phases.items()))
            self.report(first_step_time=now, phases=phases, process_start_time=t0)

    def log(self, *a):
        print(f"[{self.role} rank {self.rank}/{self.world}]", *a, flush=True)
