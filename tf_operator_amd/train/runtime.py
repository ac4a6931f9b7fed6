"""Replica-side runtime shared by the bundled trainers: rendezvous from the
operator's env contract, first-step / throughput reporting back to the
operator (BASELINE metric "submit -> first-step latency"), preemption
handling (SIGTERM -> checkpoint -> exit 143, a retryable code for the
ExitCode / elastic restart policies), and the role of this replica
(chief/worker/ps/evaluator)."""
from __future__ import annotations

import json
import os
import signal
import threading
import time
import urllib.request

from . import dist as tdist


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
        body = {"job": self.job, "namespace": self.namespace, "kind": self.kind, **kw}
        try:
            req = urllib.request.Request(self.report_url, data=json.dumps(body).encode(),
                                         headers={"Content-Type": "application/json"}, method="POST")
            urllib.request.urlopen(req, timeout=2).read()
        except Exception:
            pass  # reporting is best effort

    def first_step_done(self):
        if not self._first_reported:
            self._first_reported = True
            self.report(first_step_time=time.time())

    def log(self, *a):
        print(f"[{self.role} rank {self.rank}/{self.world}]", *a, flush=True)
