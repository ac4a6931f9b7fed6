"""A whole single-node "cluster" in one process: fake API server + the
operator (C++ core + asyncio shell) + local kubelet, on a background event
loop.  Used by the E2E test suites (replacing the reference's EKS + Argo
harness) and by the submit->first-step latency benchmark.

    with LocalCluster(gpus=0) as c:
        c.client.create(job)
        c.client.wait_for_job(name, polling_interval=0.2, timeout_seconds=60)
"""
from __future__ import annotations

import asyncio
import json
import os
import shutil
import tempfile
import threading
import time
import urllib.request

from ..fakeapi.server import FakeAPIServer
from ..localkubelet.kubelet import LocalKubelet
from ..operator.controller import ControllerOptions, JobController
from ..operator.kube import KubeClient
from ..operator.metrics import OperatorMetrics


class LocalCluster:
    def __init__(self, gpus=0, kinds=("TFJob", "PyTorchJob", "MXJob", "XGBoostJob"), enable_gang_scheduling=False,
                 threadiness=2, workdir=None, cluster_domain="", nccl_env=None, start_operator=True, qps=0,
                 grace_seconds=2.0, warm_python=None, device_visibility=None):
        self.gpus = gpus
        self.device_visibility = device_visibility
        self.warm_python = warm_python
        self.kinds = kinds
        self.opts = ControllerOptions(threadiness=threadiness, enable_gang_scheduling=enable_gang_scheduling,
                                      cluster_domain=cluster_domain, nccl_env=nccl_env or {})
        self.workdir = workdir or tempfile.mkdtemp(prefix="toa-cluster-")
        self._own_workdir = workdir is None
        self.start_operator = start_operator
        self.qps = qps
        self.grace = grace_seconds
        self.loop = asyncio.new_event_loop()
        self.thread = threading.Thread(target=self._run_loop, daemon=True)
        self.api = None
        self.kubelet = None
        self.controller = None
        self.metrics = OperatorMetrics()
        self.url = None
        self._report_runner = None

    def _run_loop(self):
        asyncio.set_event_loop(self.loop)
        self.loop.run_forever()

    def run(self, coro, timeout=60):
        return asyncio.run_coroutine_threadsafe(coro, self.loop).result(timeout)

    async def _start(self):
        self.api = FakeAPIServer()
        self.url = await self.api.start()
        self.kube_kubelet = KubeClient(self.url, qps=0)
        self.kubelet = LocalKubelet(self.kube_kubelet, self.api, gpus=self.gpus,
                                    workdir=os.path.join(self.workdir, "pods"), grace_seconds=self.grace,
                                    warm_python=self.warm_python, device_visibility=self.device_visibility)
        await self.kubelet.start()
        if self.start_operator:
            await self._start_report_server()
            self.kube_op = KubeClient(self.url, qps=self.qps, burst=max(10, int(self.qps or 10)))
            self.controller = JobController(self.kube_op, self.kinds, self.opts, self.metrics)
            await self.controller.start()

    async def _start_report_server(self):
        from aiohttp import web

        async def report(req):
            if self.controller is not None:
                self.controller.report(await req.json())
            return web.json_response({"ok": True})

        app = web.Application()
        app.router.add_post("/report", report)
        async def metrics(req):
            return web.Response(body=self.metrics.expose(), content_type="text/plain")

        app.router.add_get("/metrics", metrics)
        self._report_runner = web.AppRunner(app, access_log=None)
        await self._report_runner.setup()
        site = web.TCPSite(self._report_runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        self.report_url = f"http://127.0.0.1:{port}/report"
        self.metrics_url = f"http://127.0.0.1:{port}/metrics"
        self.opts.report_url = self.report_url

    async def _stop(self):
        if self.controller:
            await self.controller.stop()
        if self.kubelet:
            await self.kubelet.stop()
        if self._report_runner:
            await self._report_runner.cleanup()
        if self.api:
            await self.api.stop()
        for k in ("kube_op", "kube_kubelet"):
            if hasattr(self, k):
                await getattr(self, k).close()

    def start(self):
        self.thread.start()
        self.run(self._start())
        from ..sdk import TFJobClient

        self.client = TFJobClient(master=self.url)
        return self

    def stop(self):
        try:
            self.run(self._stop(), timeout=60)
        finally:
            self.loop.call_soon_threadsafe(self.loop.stop)
            self.thread.join(timeout=10)
            if self._own_workdir:
                shutil.rmtree(self.workdir, ignore_errors=True)

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()

    # ------------------------------------------------------------------ helpers
    def sdk(self, kind="TFJob"):
        from ..sdk import TFJobClient

        return TFJobClient(master=self.url, job_kind=kind)

    def pods(self, ns="default", labels=None):
        return self.api.list("pods", ns, labels)

    def services(self, ns="default", labels=None):
        return self.api.list("services", ns, labels)

    def events(self, ns="default"):
        return self.api.list("events", ns)

    def proxy(self, ns, service, path, port=2222, timeout=10):
        """GET through the API-server service proxy (E2E fault injection,
        py/kubeflow/tf_operator/util.py:108-139)."""
        url = f"{self.url}/api/v1/namespaces/{ns}/services/{service}:{port}/proxy/{path}"
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.read().decode()

    def wait(self, pred, timeout=30, interval=0.05, what="condition"):
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            v = pred()
            if v:
                return v
            time.sleep(interval)
        raise TimeoutError(f"timed out waiting for {what}")

    def wait_pod_phase(self, name, phase, ns="default", timeout=30):
        def ok():
            p = self.api.get("pods", ns, name)
            return p if p and (p.get("status") or {}).get("phase") == phase else None

        return self.wait(ok, timeout, what=f"pod {name} {phase}")

    def wait_serving(self, ns, service, timeout=30):
        def ok():
            try:
                return self.proxy(ns, service, "", timeout=2) == "hello world"
            except Exception:
                return False

        return self.wait(ok, timeout, interval=0.1, what=f"{service} serving")

    def metrics_text(self):
        return self.metrics.expose().decode()

    def gpu_metrics_text(self, sysfs_root: str | None = None) -> str:
        return self.kubelet.gpu_metrics_text(sysfs_root)


def main(argv=None):
    """Run a single-node cluster in the foreground (the `kind` replacement of
    BASELINE config #1): fake API server + operator + local kubelet.

        python -m tf_operator_amd.testing.cluster --gpus 8 --apply manifests/examples/tfjob-dist-mnist.yaml --wait
    """
    import argparse

    import yaml

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=0)
    ap.add_argument("--gang", action="store_true", help="--enable-gang-scheduling")
    ap.add_argument("--apply", action="append", default=[], help="job YAML to submit (repeatable)")
    ap.add_argument("--wait", action="store_true", help="exit when every applied job finished")
    ap.add_argument("--timeout", type=float, default=3600)
    a = ap.parse_args(argv)
    with LocalCluster(gpus=a.gpus, enable_gang_scheduling=a.gang) as c:
        print(f"API server: {c.url}   metrics: {c.metrics_url}", flush=True)
        names = []
        for path in a.apply:
            for doc in yaml.safe_load_all(open(path)):
                if not doc:
                    continue
                c.sdk(doc["kind"]).create(doc)
                names.append((doc["kind"], doc["metadata"]["name"]))
                print(f"submitted {doc['kind']} {doc['metadata']['name']}", flush=True)
        if a.wait and names:
            rc = 0
            for kind, name in names:
                job = c.sdk(kind).wait_for_job(name, polling_interval=1, timeout_seconds=a.timeout)
                conds = [x["type"] for x in (job.get("status") or {}).get("conditions") or []
                         if x.get("status") == "True"]
                print(f"{kind} {name}: {conds[-1] if conds else 'unknown'}", flush=True)
                rc |= int("Succeeded" not in conds)
            return rc
        try:
            while True:
                time.sleep(3600)
        except KeyboardInterrupt:
            return 0


if __name__ == "__main__":
    raise SystemExit(main())
