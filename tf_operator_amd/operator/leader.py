"""Lease-based leader election (coordination.k8s.io/v1 Lease).

Reference: cmd/tf-operator.v1/app/server.go:55-59,168-193 (Endpoints lock
`tf-operator`, lease 15 s, renew deadline 5 s, retry 3 s; OnStoppedLeading
-> log.Fatalf) and the new binary's `--leader-elect` with ID `1ca428e5.`
(cmd/training-operator.v1/main.go:65-67,84).  Same timings; the lock is a
Lease object (Endpoints locks are deprecated upstream).
"""
from __future__ import annotations

import asyncio
import datetime
import logging
import os
import socket
import uuid

from .kube import ApiError, KubeClient

log = logging.getLogger("tf_operator_amd.leader")


def _now_micro():
    return datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def _parse(ts):
    if not ts:
        return None
    for fmt in ("%Y-%m-%dT%H:%M:%S.%fZ", "%Y-%m-%dT%H:%M:%SZ"):
        try:
            return datetime.datetime.strptime(ts, fmt).replace(tzinfo=datetime.timezone.utc)
        except ValueError:
            pass
    return None


class LeaderElector:
    def __init__(self, kube: KubeClient, namespace: str, name: str = "tf-operator", identity: str | None = None,
                 lease_duration=15.0, renew_deadline=5.0, retry_period=3.0, on_started=None, on_stopped=None,
                 on_change=None):
        self.kube = kube
        self.ns = namespace
        self.name = name
        self.identity = identity or f"{socket.gethostname()}_{uuid.uuid4().hex[:8]}"
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.on_started = on_started
        self.on_stopped = on_stopped
        self.on_change = on_change
        self.is_leader = False
        self._observed_holder = None

    async def _try_acquire_or_renew(self) -> bool:
        key = "coordination.k8s.io/leases"
        now = datetime.datetime.now(datetime.timezone.utc)
        try:
            lease = await self.kube.get(key, self.ns, self.name)
        except ApiError as e:
            if e.status != 404:
                raise
            body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                    "metadata": {"name": self.name, "namespace": self.ns},
                    "spec": {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease_duration),
                             "acquireTime": _now_micro(), "renewTime": _now_micro(), "leaseTransitions": 0}}
            try:
                await self.kube.create(key, self.ns, body)
                return True
            except ApiError as e2:
                if e2.status == 409:
                    return False
                raise
        spec = lease.get("spec", {})
        holder = spec.get("holderIdentity")
        if holder != self._observed_holder:
            self._observed_holder = holder
            if self.on_change:
                self.on_change(holder)
        renew = _parse(spec.get("renewTime"))
        dur = float(spec.get("leaseDurationSeconds", self.lease_duration))
        if holder and holder != self.identity and renew and (now - renew).total_seconds() < dur:
            return False
        if holder != self.identity:
            spec["leaseTransitions"] = int(spec.get("leaseTransitions", 0)) + 1
            spec["acquireTime"] = _now_micro()
        spec["holderIdentity"] = self.identity
        spec["renewTime"] = _now_micro()
        spec["leaseDurationSeconds"] = int(self.lease_duration)
        lease["spec"] = spec
        try:
            await self.kube.update(key, self.ns, lease)
            return True
        except ApiError as e:
            if e.status == 409:
                return False
            raise

    async def run(self, stop: asyncio.Event | None = None):
        stop = stop or asyncio.Event()
        # acquire
        while not stop.is_set():
            try:
                if await self._try_acquire_or_renew():
                    break
            except Exception as e:
                log.warning("leader election: %s", e)
            try:
                await asyncio.wait_for(stop.wait(), timeout=self.retry_period)
            except asyncio.TimeoutError:
                pass
        if stop.is_set():
            return
        self.is_leader = True
        log.info("%s became leader of %s/%s", self.identity, self.ns, self.name)
        if self.on_started:
            r = self.on_started()
            if asyncio.iscoroutine(r):
                await r
        # renew
        last_ok = asyncio.get_running_loop().time()
        while not stop.is_set():
            try:
                await asyncio.wait_for(stop.wait(), timeout=self.retry_period)
                break
            except asyncio.TimeoutError:
                pass
            try:
                if await self._try_acquire_or_renew():
                    last_ok = asyncio.get_running_loop().time()
                    continue
            except Exception as e:
                log.warning("lease renew: %s", e)
            if asyncio.get_running_loop().time() - last_ok > self.renew_deadline:
                break
        self.is_leader = False
        log.warning("%s stopped leading", self.identity)
        if self.on_stopped:
            r = self.on_stopped()
            if asyncio.iscoroutine(r):
                await r


def default_namespace():
    return os.environ.get("KUBEFLOW_NAMESPACE") or os.environ.get("MY_POD_NAMESPACE") or "default"
