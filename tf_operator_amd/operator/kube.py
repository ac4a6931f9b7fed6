"""Asyncio Kubernetes REST + watch client (aiohttp; no `kubernetes` package).

Typed-clientset equivalent of the reference's generated client
(pkg/client/clientset/versioned/typed/tensorflow/v1/tfjob.go:66-193:
Get/List/Watch/Create/Update/UpdateStatus/Delete/DeleteCollection/Patch) for
every resource the operator touches, with the clientset's token-bucket QPS /
burst limiter (clientset.go:62; defaults 5 / 10 from
cmd/tf-operator.v1/app/options/options.go:81-82).  Works against a real
cluster (kubeconfig or in-cluster service account) and the in-process fake
API server.
"""
from __future__ import annotations

import asyncio
import base64
import json
import os
import ssl
import tempfile
import time

import aiohttp

GROUP_VERSIONS = {"kubeflow.org": "v1", "scheduling.volcano.sh": "v1beta1", "coordination.k8s.io": "v1",
                  "apiextensions.k8s.io": "v1"}
CLUSTER_SCOPED = {"namespaces", "nodes", "apiextensions.k8s.io/customresourcedefinitions"}


class ApiError(Exception):
    def __init__(self, status, body):
        self.status = status
        self.body = body
        try:
            self.reason = json.loads(body).get("reason", "")
            self.message = json.loads(body).get("message", body)
        except Exception:
            self.reason, self.message = "", body
        super().__init__(f"{status} {self.reason}: {self.message}")


class TokenBucket:
    def __init__(self, qps, burst):
        self.qps = float(qps)
        self.burst = float(burst)
        self.tokens = float(burst)
        self.t = time.monotonic()
        self._lock = asyncio.Lock()

    async def acquire(self):
        if self.qps <= 0:
            return
        async with self._lock:
            while True:
                now = time.monotonic()
                self.tokens = min(self.burst, self.tokens + (now - self.t) * self.qps)
                self.t = now
                if self.tokens >= 1:
                    self.tokens -= 1
                    return
                await asyncio.sleep((1 - self.tokens) / self.qps)


def resource_path(key: str, ns: str | None = None, name: str | None = None, sub: str | None = None) -> str:
    if "/" in key:
        group, plural = key.split("/", 1)
        base = f"/apis/{group}/{GROUP_VERSIONS.get(group, 'v1')}"
    else:
        plural, base = key, "/api/v1"
    p = base
    if ns is not None and key not in CLUSTER_SCOPED:
        p += f"/namespaces/{ns}"
    p += f"/{plural}"
    if name:
        p += f"/{name}"
    if sub:
        p += f"/{sub}"
    return p


def plural_key(kind_or_plural: str) -> str:
    m = {"tfjob": "tfjobs", "pytorchjob": "pytorchjobs", "mxjob": "mxjobs", "xgboostjob": "xgboostjobs"}
    k = kind_or_plural.lower()
    k = m.get(k, k)
    return "kubeflow.org/" + k


class KubeClient:
    def __init__(self, base_url, token=None, ssl_context=None, qps=5.0, burst=10, user_agent="tf-operator-amd",
                 headers=None):
        self.base = base_url.rstrip("/")
        self.headers = {"User-Agent": user_agent, "Accept": "application/json"}
        if token:
            self.headers["Authorization"] = f"Bearer {token}"
        if headers:
            self.headers.update(headers)
        self.ssl = ssl_context
        self.limiter = TokenBucket(qps, burst)
        self._session = None

    # ---------------------------------------------------------------- config
    @classmethod
    def in_cluster(cls, **kw):
        host, port = os.environ["KUBERNETES_SERVICE_HOST"], os.environ["KUBERNETES_SERVICE_PORT"]
        sa = "/var/run/secrets/kubernetes.io/serviceaccount"
        token = open(os.path.join(sa, "token")).read().strip()
        ctx = ssl.create_default_context(cafile=os.path.join(sa, "ca.crt"))
        return cls(f"https://{host}:{port}", token=token, ssl_context=ctx, **kw)

    @classmethod
    def from_kubeconfig(cls, path=None, context=None, **kw):
        import yaml

        path = path or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
        cfg = yaml.safe_load(open(path))
        ctx_name = context or cfg.get("current-context")
        ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == ctx_name)
        cluster = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in cfg.get("users", []) if u["name"] == ctx.get("user")), {})
        server = cluster["server"]
        sslctx = None
        if server.startswith("https"):
            sslctx = ssl.create_default_context()
            if cluster.get("insecure-skip-tls-verify"):
                sslctx.check_hostname = False
                sslctx.verify_mode = ssl.CERT_NONE
            if cluster.get("certificate-authority-data"):
                sslctx.load_verify_locations(cadata=base64.b64decode(cluster["certificate-authority-data"]).decode())
            elif cluster.get("certificate-authority"):
                sslctx.load_verify_locations(cafile=cluster["certificate-authority"])
            cert, key = user.get("client-certificate"), user.get("client-key")
            if user.get("client-certificate-data"):
                cf = tempfile.NamedTemporaryFile(delete=False, suffix=".crt")
                cf.write(base64.b64decode(user["client-certificate-data"]))
                cf.close()
                kf = tempfile.NamedTemporaryFile(delete=False, suffix=".key")
                kf.write(base64.b64decode(user["client-key-data"]))
                kf.close()
                cert, key = cf.name, kf.name
            if cert:
                sslctx.load_cert_chain(cert, key)
        return cls(server, token=user.get("token"), ssl_context=sslctx, **kw)

    @classmethod
    def auto(cls, master=None, kubeconfig=None, **kw):
        if master:
            return cls(master, **kw)
        if kubeconfig or os.environ.get("KUBECONFIG") or os.path.exists(os.path.expanduser("~/.kube/config")):
            return cls.from_kubeconfig(kubeconfig, **kw)
        return cls.in_cluster(**kw)

    # ---------------------------------------------------------------- http
    async def session(self):
        if self._session is None or self._session.closed:
            self._session = aiohttp.ClientSession(headers=self.headers,
                                                  timeout=aiohttp.ClientTimeout(total=None, sock_connect=10))
        return self._session

    async def close(self):
        if self._session is not None:
            await self._session.close()

    async def request(self, method, path, body=None, params=None, content_type="application/json", timeout=30):
        await self.limiter.acquire()
        s = await self.session()
        data = json.dumps(body) if body is not None else None
        async with s.request(method, self.base + path, data=data, params=params, ssl=self.ssl,
                             headers={"Content-Type": content_type},
                             timeout=aiohttp.ClientTimeout(total=timeout)) as r:
            text = await r.text()
            if r.status >= 400:
                raise ApiError(r.status, text)
            return json.loads(text) if text and r.content_type == "application/json" else text

    # ---------------------------------------------------------------- typed verbs
    async def get(self, key, ns, name):
        return await self.request("GET", resource_path(key, ns, name))

    async def list(self, key, ns=None, label_selector=None, field_selector=None):
        params = {}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        return await self.request("GET", resource_path(key, ns), params=params)

    async def create(self, key, ns, obj):
        return await self.request("POST", resource_path(key, ns), obj)

    async def update(self, key, ns, obj):
        return await self.request("PUT", resource_path(key, ns, obj["metadata"]["name"]), obj)

    async def update_status(self, key, ns, obj):
        return await self.request("PUT", resource_path(key, ns, obj["metadata"]["name"], "status"), obj)

    async def patch(self, key, ns, name, patch, sub=None):
        return await self.request("PATCH", resource_path(key, ns, name, sub), patch,
                                  content_type="application/merge-patch+json")

    async def delete(self, key, ns, name, propagation="Background"):
        return await self.request("DELETE", resource_path(key, ns, name),
                                  {"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": propagation})

    async def delete_collection(self, key, ns, label_selector=None):
        params = {"labelSelector": label_selector} if label_selector else None
        return await self.request("DELETE", resource_path(key, ns), params=params)

    async def watch(self, key, ns=None, label_selector=None, resource_version=None, timeout_seconds=None):
        """Async generator of (event_type, object)."""
        params = {"watch": "true"}
        if label_selector:
            params["labelSelector"] = label_selector
        if resource_version:
            params["resourceVersion"] = str(resource_version)
        if timeout_seconds:
            params["timeoutSeconds"] = str(int(timeout_seconds))
        s = await self.session()
        async with s.get(self.base + resource_path(key, ns), params=params, ssl=self.ssl,
                         timeout=aiohttp.ClientTimeout(total=None, sock_read=None)) as r:
            if r.status >= 400:
                raise ApiError(r.status, await r.text())
            buf = b""
            async for chunk in r.content.iter_any():
                buf += chunk
                while b"\n" in buf:
                    line, buf = buf.split(b"\n", 1)
                    if not line.strip():
                        continue
                    ev = json.loads(line)
                    yield ev.get("type"), ev.get("object")
