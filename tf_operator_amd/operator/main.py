"""`tf-operator-amd` process entry point.

One binary replacing both reference entry points:
cmd/training-operator.v1/main.go (controller-runtime manager: --metrics-bind-address
:8080, --health-probe-bind-address :8081, --leader-elect, --enable-scheme) and
cmd/tf-operator.v1 (legacy: --master, --namespace, --threadiness,
--json-log-format, --enable-gang-scheduling, --gang-scheduler-name,
--monitoring-port, --resyc-period, --qps, --burst, --version; env
KUBEFLOW_NAMESPACE / KUBECONFIG / CUSTOM_CLUSTER_DOMAIN).

HTTP: /metrics (Prometheus), /healthz, /readyz, POST /report (trainer
first-step + throughput reports), /debug/pprof/{heap,tasks} (pprof analog).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import signal
import sys
import time
import tracemalloc

from aiohttp import web

from .. import version
from .controller import ControllerOptions, JobController
from .kube import ApiError, KubeClient
from .leader import LeaderElector, default_namespace
from .metrics import OperatorMetrics

log = logging.getLogger("tf_operator_amd")


class JsonFormatter(logging.Formatter):
    """logrus JSONFormatter + filename hook analog (cmd/tf-operator.v1/main.go:32-37)."""

    def format(self, r):
        d = {"level": r.levelname.lower(), "msg": r.getMessage(), "time": self.formatTime(r, "%Y-%m-%dT%H:%M:%S"),
             "filename": f"{r.filename}:{r.lineno}", "logger": r.name}
        span = getattr(r, "span", None)
        if span is not None:
            d.update(span)
        if r.exc_info:
            d["error"] = self.formatException(r.exc_info)
        return json.dumps(d)


def _duration(s: str) -> float:
    s = s.strip()
    mult = {"ms": 1e-3, "s": 1, "m": 60, "h": 3600}
    for suf in ("ms", "s", "m", "h"):
        if s.endswith(suf):
            return float(s[: -len(suf)]) * mult[suf]
    return float(s)


def _addr(s: str):
    host, _, port = s.rpartition(":")
    return (host or "0.0.0.0"), int(port)


def build_parser():
    p = argparse.ArgumentParser("tf-operator-amd")
    p.add_argument("--metrics-bind-address", default=":8080")
    p.add_argument("--health-probe-bind-address", default=":8081")
    p.add_argument("--leader-elect", action="store_true")
    p.add_argument("--leader-election-id", default="1ca428e5.tf-operator")
    # server.go:56-58: lease 15 s, renew deadline 5 s, retry 3 s
    p.add_argument("--leader-lease-duration", type=float, default=15.0)
    p.add_argument("--leader-renew-deadline", type=float, default=5.0)
    p.add_argument("--leader-retry-period", type=float, default=3.0)
    p.add_argument("--enable-scheme", action="append", default=[],
                   help="TFJob|PyTorchJob|MXJob|XGBoostJob (case-insensitive; repeatable; default all)")
    p.add_argument("--master", default=None, help="API server URL (overrides kubeconfig)")
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--namespace", default=os.environ.get("KUBEFLOW_NAMESPACE") or None,
                   help="watch only this namespace (default: all)")
    p.add_argument("--threadiness", type=int, default=1)
    p.add_argument("--version", action="store_true")
    p.add_argument("--json-log-format", type=lambda v: v.lower() != "false", default=True)
    p.add_argument("--enable-gang-scheduling", action="store_true")
    p.add_argument("--gang-scheduler-name", default="volcano")
    p.add_argument("--monitoring-port", type=int, default=8443,
                   help="legacy /metrics port (options.go:75: default 8443, 0 disables)")
    p.add_argument("--resyc-period", dest="resync_period", default="12h")
    p.add_argument("--qps", type=float, default=5.0)
    p.add_argument("--burst", type=int, default=10)
    p.add_argument("--inject-rocm-env", type=lambda v: v.lower() != "false", default=True)
    p.add_argument("--nccl-env", action="append", default=[], help="K=V injected into trainer replicas")
    p.add_argument("--rccl-defaults", type=lambda v: v.lower() != "false", default=True,
                   help="inject xGMI-oriented RCCL/torch defaults a container does not set itself")
    p.add_argument("--cluster-domain", default=os.environ.get("CUSTOM_CLUSTER_DOMAIN", ""))
    p.add_argument("--report-url", default=os.environ.get("TOA_OPERATOR_REPORT_URL"))
    p.add_argument("--gpu-resource", default="amd.com/gpu", help="extended resource name of a GPU")
    p.add_argument("--gpus-per-node", type=int, default=8,
                   help="GPUs of one node: a job's RCCL ranks up to this many can run in the node-local "
                        "xGMI layout (amd.com/node-local annotation, or automatically when gang-scheduled)")
    p.add_argument("--config", default=None, help="optional YAML file with the same keys as the flags")
    return p


def parse_args(argv=None):
    p = build_parser()
    a = p.parse_args(argv)
    if a.config:
        import yaml

        cfg = yaml.safe_load(open(a.config)) or {}
        for k, v in cfg.items():
            k = k.replace("-", "_")
            if hasattr(a, k) and getattr(a, k) == p.get_default(k):
                setattr(a, k, v)
    return a


SCHEMES = {"tfjob": "TFJob", "pytorchjob": "PyTorchJob", "mxjob": "MXJob", "xgboostjob": "XGBoostJob"}


def enabled_kinds(flags):
    """register_controller.go:52-76: case-insensitive, all when empty."""
    if not flags:
        return list(SCHEMES.values())
    out = []
    for f in flags:
        for part in f.split(","):
            k = SCHEMES.get(part.strip().lower())
            if k is None:
                raise SystemExit(f"unsupported scheme {part!r}; supported: {', '.join(SCHEMES.values())}")
            if k not in out:
                out.append(k)
    return out


class Operator:
    def __init__(self, args, kube: KubeClient | None = None):
        self.args = args
        self.kube = kube or KubeClient.auto(args.master, args.kubeconfig, qps=args.qps, burst=args.burst,
                                            user_agent="tf-operator-amd")
        self.metrics = OperatorMetrics()
        nccl = dict(kv.split("=", 1) for kv in args.nccl_env)
        self.ctrl = JobController(self.kube, enabled_kinds(args.enable_scheme), ControllerOptions(
            namespace=args.namespace, threadiness=args.threadiness,
            enable_gang_scheduling=args.enable_gang_scheduling, gang_scheduler_name=args.gang_scheduler_name,
            inject_rocm_env=args.inject_rocm_env, cluster_domain=args.cluster_domain, nccl_env=nccl,
            rccl_defaults=args.rccl_defaults,
            resync_period=_duration(str(args.resync_period)), report_url=args.report_url,
            gpu_resource=args.gpu_resource, gpus_per_node=args.gpus_per_node), self.metrics)
        self.stop = asyncio.Event()
        self.ready = False
        self.runners = []
        self.ports = {}

    # ---------------------------------------------------------------- http
    async def h_metrics(self, req):
        return web.Response(body=self.metrics.expose(), content_type="text/plain")

    async def h_healthz(self, req):
        return web.Response(text="ok")

    async def h_readyz(self, req):
        return web.Response(text="ok" if self.ready else "not ready", status=200 if self.ready else 503)

    async def h_report(self, req):
        self.ctrl.report(await req.json())
        return web.json_response({"ok": True})

    async def h_heap(self, req):
        if not tracemalloc.is_tracing():
            tracemalloc.start()
            return web.Response(text="tracemalloc started; query again for a snapshot\n")
        top = tracemalloc.take_snapshot().statistics("lineno")[:30]
        return web.Response(text="\n".join(str(s) for s in top) + "\n")

    async def h_tasks(self, req):
        return web.Response(text="\n".join(repr(t) for t in asyncio.all_tasks()) + "\n")

    async def _serve(self, name, bind, routes):
        app = web.Application()
        for method, path, h in routes:
            app.router.add_route(method, path, h)
        runner = web.AppRunner(app, access_log=None)
        await runner.setup()
        host, port = _addr(bind)
        site = web.TCPSite(runner, host, port)
        await site.start()
        self.ports[name] = site._server.sockets[0].getsockname()[1]
        self.runners.append(runner)

    # ---------------------------------------------------------------- lifecycle
    async def _check_crds(self):
        """server.go:232-251 checkCRDExists (warn instead of exiting)."""
        for kind in self.ctrl.kinds:
            plural = kind.lower() + "s"
            try:
                await self.kube.get("apiextensions.k8s.io/customresourcedefinitions", None, f"{plural}.kubeflow.org")
            except ApiError as e:
                log.warning("CRD %s.kubeflow.org not found (%s)", plural, e.status)
            except Exception as e:
                log.warning("CRD check failed: %s", e)

    async def _lead(self):
        self.metrics.is_leader.set(1)
        await self.ctrl.start()
        self.ready = True

    async def _lost(self):
        self.metrics.is_leader.set(0)
        log.error("leader election lost")
        self.stop.set()

    async def run(self):
        m = [("GET", "/metrics", self.h_metrics), ("POST", "/report", self.h_report),
             ("GET", "/debug/pprof/heap", self.h_heap), ("GET", "/debug/pprof/tasks", self.h_tasks)]
        await self._serve("metrics", self.args.metrics_bind_address, m)
        await self._serve("probe", self.args.health_probe_bind_address,
                          [("GET", "/healthz", self.h_healthz), ("GET", "/readyz", self.h_readyz)])
        if self.args.monitoring_port:
            await self._serve("monitoring", f":{self.args.monitoring_port}", m)
        await self._check_crds()
        if self.args.leader_elect:
            el = LeaderElector(self.kube, default_namespace(), self.args.leader_election_id,
                               lease_duration=self.args.leader_lease_duration,
                               renew_deadline=self.args.leader_renew_deadline,
                               retry_period=self.args.leader_retry_period,
                               on_started=self._lead, on_stopped=self._lost)
            self.elector = el
            elect = asyncio.create_task(el.run(self.stop))
        else:
            await self._lead()
            elect = None
        await self.stop.wait()
        await self.ctrl.stop()
        if elect:
            elect.cancel()
        for r in self.runners:
            await r.cleanup()
        await self.kube.close()


def setup_logging(json_format=True, level=logging.INFO):
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(JsonFormatter() if json_format else logging.Formatter(
        "%(asctime)s %(levelname)s %(filename)s:%(lineno)d %(message)s"))
    root = logging.getLogger()
    root.handlers[:] = [h]
    root.setLevel(level)


def main(argv=None):
    args = parse_args(argv)
    if args.version:
        print(version.info())
        return 0
    setup_logging(args.json_log_format)
    log.info(version.info())
    op = Operator(args)

    async def _run():
        loop = asyncio.get_running_loop()
        for s in (signal.SIGINT, signal.SIGTERM):
            try:
                loop.add_signal_handler(s, op.stop.set)
            except NotImplementedError:
                pass
        await op.run()

    asyncio.run(_run())
    return 0


if __name__ == "__main__":
    sys.exit(main())
