"""Fault injection for the local cluster (SURVEY 5 "Failure detection /
elastic recovery / fault injection"; BASELINE config #5).

The reference's only fault injector is the test-server's
``/exit?exitCode=`` endpoint (test/test-server/test_app.py:47-59), reached
through the API-server service proxy.  That stays available
(:mod:`tf_operator_amd.testing.test_server`); this module adds the faults an
elastic MI355X job has to survive:

* :func:`kill_pod` -- SIGKILL (exit 137) or any signal to a pod's process
  group, as the OOM killer or a crashed rank would;
* :func:`preempt_pod` -- delete the pod through the API (what a preempting
  scheduler or a drained node does);
* :func:`set_gpu_capacity` -- shrink / grow the node's allocatable
  ``amd.com/gpu`` (lost devices, a node slice handed to another tenant);
* :class:`ChaosMonkey` -- random faults on an interval, for soak tests.

All functions take a :class:`~tf_operator_amd.testing.cluster.LocalCluster`.
"""
from __future__ import annotations

import os
import random
import signal
import threading
import time


def _pod_procs(cluster, ns, name):
    rec = cluster.kubelet.running.get((ns, name))
    if rec is None:
        return []
    return [p.proc for p in rec["procs"] if p.proc is not None and p.proc.returncode is None]


def kill_pod(cluster, name, ns="default", sig=signal.SIGKILL) -> bool:
    """Send `sig` to every container process group of the pod.  Returns False
    when the pod has no running process."""
    procs = _pod_procs(cluster, ns, name)
    for proc in procs:
        try:
            os.killpg(proc.pid, sig)
        except ProcessLookupError:
            pass
    return bool(procs)


def preempt_pod(cluster, name, ns="default") -> bool:
    """Delete the pod via the API server (SIGTERM, grace period, SIGKILL)."""
    from ..operator.kube import ApiError

    try:
        cluster.run(cluster.kube_kubelet.delete("pods", ns, name))
        return True
    except ApiError:
        return False


def set_gpu_capacity(cluster, gpus: int):
    """Set the node's allocatable GPU count (devices >= gpus disappear)."""
    cluster.run(cluster.kubelet.set_capacity(gpus))


class ChaosMonkey:
    """Every `interval` seconds pick a running pod matching `selector` and
    apply one of `faults` ("kill", "preempt").  Stops after `max_faults`."""

    def __init__(self, cluster, selector: dict, ns="default", interval=5.0, faults=("kill", "preempt"),
                 max_faults=1, seed=0):
        self.cluster, self.selector, self.ns = cluster, selector, ns
        self.interval, self.faults, self.max_faults = interval, faults, max_faults
        self.rng = random.Random(seed)
        self.log: list[tuple[float, str, str]] = []
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.wait(self.interval) and len(self.log) < self.max_faults:
            pods = [p for p in self.cluster.pods(self.ns, self.selector)
                    if (p.get("status") or {}).get("phase") == "Running"
                    and not p["metadata"].get("deletionTimestamp")]
            if not pods:
                continue
            victim = self.rng.choice(pods)["metadata"]["name"]
            fault = self.rng.choice(self.faults)
            ok = kill_pod(self.cluster, victim, self.ns) if fault == "kill" else preempt_pod(self.cluster, victim,
                                                                                           self.ns)
            if ok:
                self.log.append((time.time(), fault, victim))

    def start(self):
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        self._thread.join(timeout=5)
