"""In-process fake Kubernetes API server (aiohttp).

The subset of kube-apiserver the operator, SDK and local kubelet use, with
the semantics the reference's behaviour depends on:

* CRUD on core ``pods`` / ``services`` / ``events`` / ``namespaces``, the four
  ``kubeflow.org/v1`` job kinds, Volcano ``podgroups``, ``leases`` and
  ``customresourcedefinitions``;
* list + chunked **watch** with monotonically increasing resourceVersion,
  label / field selectors and replay from a resourceVersion;
* the **status subresource** (PUT /status touches only status; PUT / PATCH of
  the object never changes status of kinds that have the subresource);
* optimistic concurrency (409 on stale resourceVersion, 409 AlreadyExists);
* JSON merge-patch;
* **ownerReference cascade** deletion (background GC);
* schema-level admission for the job CRDs (``spec.<x>ReplicaSpecs: Required
  value`` -- py/kubeflow/tf_operator/invalid_tfjob_tests.py:26-44);
* the **service proxy** ``/api/v1/namespaces/{ns}/services/{name}:{port}/proxy/``
  used by the E2E fault injection (test-server ``/exit``), forwarded to the
  local kubelet's port registry;
* pod logs (``/log``, with ``follow``) served from the local kubelet.
"""
from __future__ import annotations

import asyncio
import copy
import json
import time
import uuid

from aiohttp import ClientSession, web

from ..utils.k8s import json_merge_patch, match_fields, match_labels, parse_selector

KUBEFLOW_KINDS = {
    "tfjobs": ("TFJob", "tfReplicaSpecs"),
    "pytorchjobs": ("PyTorchJob", "pytorchReplicaSpecs"),
    "mxjobs": ("MXJob", "mxReplicaSpecs"),
    "xgboostjobs": ("XGBoostJob", "xgbReplicaSpecs"),
}
# resource key -> (kind, namespaced, has status subresource)
RESOURCES = {
    "pods": ("Pod", True, True),
    "services": ("Service", True, False),
    "events": ("Event", True, False),
    "namespaces": ("Namespace", False, False),
    "nodes": ("Node", False, True),
    "configmaps": ("ConfigMap", True, False),
    "scheduling.volcano.sh/podgroups": ("PodGroup", True, True),
    "coordination.k8s.io/leases": ("Lease", True, False),
    "apiextensions.k8s.io/customresourcedefinitions": ("CustomResourceDefinition", False, False),
}
for _plural, (_kind, _f) in KUBEFLOW_KINDS.items():
    RESOURCES["kubeflow.org/" + _plural] = (_kind, True, True)

API_VERSIONS = {
    "pods": "v1", "services": "v1", "events": "v1", "namespaces": "v1", "configmaps": "v1", "nodes": "v1",
    "scheduling.volcano.sh/podgroups": "scheduling.volcano.sh/v1beta1",
    "coordination.k8s.io/leases": "coordination.k8s.io/v1",
    "apiextensions.k8s.io/customresourcedefinitions": "apiextensions.k8s.io/v1",
}
GROUP_VERSIONS = {"kubeflow.org": "v1", "scheduling.volcano.sh": "v1beta1", "coordination.k8s.io": "v1",
                  "apiextensions.k8s.io": "v1"}


def _status(code, reason, message):
    return web.json_response({"kind": "Status", "apiVersion": "v1", "status": "Failure", "reason": reason,
                              "message": message, "code": code}, status=code)


class FakeAPIServer:
    def __init__(self, install_crds=True, history=20000):
        self.objects: dict[str, dict[tuple, dict]] = {r: {} for r in RESOURCES}
        self.rv = 0
        self.events: list[tuple[int, str, str, dict]] = []  # (rv, resource, type, obj)
        self.history = history
        self.watchers: list = []
        self.kubelet = None  # set by LocalKubelet for proxy / logs
        self.app = web.Application()
        self._routes()
        self.runner = None
        self.port = None
        self.requests = 0
        if install_crds:
            for plural, (kind, _) in KUBEFLOW_KINDS.items():
                self._store_put("apiextensions.k8s.io/customresourcedefinitions", {
                    "apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
                    "metadata": {"name": f"{plural}.kubeflow.org"},
                    "spec": {"group": "kubeflow.org", "names": {"kind": kind, "plural": plural},
                             "scope": "Namespaced"}})
            self._store_put("apiextensions.k8s.io/customresourcedefinitions", {
                "apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
                "metadata": {"name": "podgroups.scheduling.volcano.sh"}, "spec": {"group": "scheduling.volcano.sh"}})

    # ------------------------------------------------------------------ routing
    def _routes(self):
        r = self.app.router
        async def healthz(req):
            return web.Response(text="ok")

        async def version(req):
            return web.json_response({"major": "1", "minor": "29", "gitVersion": "tf-operator-amd-fake"})

        r.add_get("/healthz", healthz)
        r.add_get("/version", version)
        core = "/api/v1"
        r.add_route("*", core + "/namespaces/{ns}/services/{svc}/proxy/{path:.*}", self.h_proxy)
        r.add_get(core + "/namespaces/{ns}/pods/{name}/log", self.h_log)
        for res in ("pods", "services", "events", "configmaps"):
            self._add_resource(core, res, res)
        r.add_route("*", core + "/namespaces", self._bind(self.h_collection, "namespaces", None))
        r.add_route("*", core + "/namespaces/{name}", self._bind(self.h_item, "namespaces", None))
        r.add_route("*", core + "/nodes", self._bind(self.h_collection, "nodes", None))
        r.add_route("*", core + "/nodes/{name}", self._bind(self.h_item, "nodes", None))
        r.add_route("*", core + "/nodes/{name}/status", self._bind(self.h_status, "nodes", None))
        for key in RESOURCES:
            if "/" in key:
                group, plural = key.split("/")
                base = f"/apis/{group}/{GROUP_VERSIONS[group]}"
                if RESOURCES[key][1]:
                    self._add_resource(base, plural, key)
                else:
                    r.add_route("*", f"{base}/{plural}", self._bind(self.h_collection, key, None))
                    r.add_route("*", f"{base}/{plural}/{{name}}", self._bind(self.h_item, key, None))

    def _add_resource(self, base, plural, key):
        r = self.app.router
        r.add_route("*", f"{base}/namespaces/{{ns}}/{plural}", self._bind(self.h_collection, key, "ns"))
        r.add_route("*", f"{base}/namespaces/{{ns}}/{plural}/{{name}}", self._bind(self.h_item, key, "ns"))
        r.add_route("*", f"{base}/namespaces/{{ns}}/{plural}/{{name}}/status", self._bind(self.h_status, key, "ns"))
        r.add_get(f"{base}/{plural}", self._bind(self.h_collection, key, None))

    @staticmethod
    def _bind(fn, key, nskey):
        async def h(req):
            ns = req.match_info.get("ns") if nskey else None
            return await fn(req, key, ns)

        return h

    # ------------------------------------------------------------------ storage
    def _next_rv(self):
        self.rv += 1
        return self.rv

    def _store_put(self, key, obj, etype=None):
        md = obj.setdefault("metadata", {})
        ns = md.get("namespace") if RESOURCES[key][1] else None
        k = (ns, md["name"])
        existed = k in self.objects[key]
        md.setdefault("uid", str(uuid.uuid4()))
        md.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
        md["resourceVersion"] = str(self._next_rv())
        obj.setdefault("apiVersion", API_VERSIONS.get(key, "kubeflow.org/v1"))
        obj.setdefault("kind", RESOURCES[key][0])
        self.objects[key][k] = obj
        self._notify(key, etype or ("MODIFIED" if existed else "ADDED"), obj)
        return obj

    def _store_delete(self, key, ns, name):
        obj = self.objects[key].pop((ns, name), None)
        if obj is None:
            return None
        obj = copy.deepcopy(obj)
        obj["metadata"]["resourceVersion"] = str(self._next_rv())
        self._notify(key, "DELETED", obj)
        self._gc(obj["metadata"].get("uid"))
        return obj

    def _gc(self, uid):
        if not uid:
            return
        for key, objs in self.objects.items():
            for (ns, name), o in list(objs.items()):
                if any(ref.get("uid") == uid for ref in o.get("metadata", {}).get("ownerReferences", []) or []):
                    self._store_delete(key, ns, name)

    def _notify(self, key, etype, obj):
        rv = int(obj["metadata"]["resourceVersion"])
        snap = copy.deepcopy(obj)
        self.events.append((rv, key, etype, snap))
        if len(self.events) > self.history:
            del self.events[: len(self.events) - self.history]
        for w in list(self.watchers):
            if w["key"] == key and self._match(w, snap):
                w["queue"].put_nowait((etype, snap))

    @staticmethod
    def _match(w, obj):
        md = obj.get("metadata", {})
        if w["ns"] is not None and md.get("namespace") != w["ns"]:
            return False
        return match_labels(md.get("labels") or {}, w["labels"]) and match_fields(obj, w["fields"])

    # ------------------------------------------------------------------ public helpers (in-process users)
    def get(self, key, ns, name):
        o = self.objects[key].get((ns if RESOURCES[key][1] else None, name))
        return copy.deepcopy(o) if o else None

    def list(self, key, ns=None, labels=None):
        sel = parse_selector(labels) if isinstance(labels, str) else (labels or {})
        out = []
        for (ons, _), o in self.objects[key].items():
            if ns is not None and ons != ns:
                continue
            if match_labels(o.get("metadata", {}).get("labels") or {}, sel):
                out.append(copy.deepcopy(o))
        return out

    def put_status(self, key, ns, name, status):
        o = self.objects[key].get((ns, name))
        if o is None:
            return None
        o = copy.deepcopy(o)
        o["status"] = status
        return self._store_put(key, o)

    def update(self, key, obj):
        return self._store_put(key, copy.deepcopy(obj))

    def delete(self, key, ns, name):
        return self._store_delete(key, ns, name)

    # ------------------------------------------------------------------ handlers
    def _admit(self, key, obj):
        if key.startswith("kubeflow.org/"):
            kind, field = KUBEFLOW_KINDS[key.split("/")[1]]
            spec = obj.get("spec")
            if not isinstance(spec, dict) or not spec.get(field):
                return f'{kind}.kubeflow.org "{obj.get("metadata", {}).get("name", "")}" is invalid: spec.{field}: ' \
                       f"Required value"
            from ..api.validate import job_errors

            errs = job_errors(obj, kind)
            if errs:  # the API server's structural-schema admission of the CRD
                name = obj.get("metadata", {}).get("name", "")
                return f'{kind}.kubeflow.org "{name}" is invalid: ' + (errs[0] if len(errs) == 1 else
                                                                        "[" + ", ".join(errs) + "]")
        if not obj.get("metadata", {}).get("name"):
            gen = obj.get("metadata", {}).get("generateName")
            if gen:
                obj["metadata"]["name"] = gen + uuid.uuid4().hex[:5]
            else:
                return "metadata.name: Required value"
        return None

    def _pod_security(self, obj):
        """PodSecurity admission (the API server's built-in plugin) for
        namespaces labelled pod-security.kubernetes.io/enforce = baseline or
        restricted: host namespaces, privileged containers and hostPath
        volumes are rejected with 403, message in the real server's format."""
        ns = obj.get("metadata", {}).get("namespace", "default")
        nso = self.objects["namespaces"].get((None, ns))
        level = ((nso or {}).get("metadata", {}).get("labels") or {}).get("pod-security.kubernetes.io/enforce")
        if level not in ("baseline", "restricted"):
            return None
        spec = obj.get("spec") or {}
        why = []
        hn = [f"{k}=true" for k in ("hostNetwork", "hostPID", "hostIPC") if spec.get(k)]
        if hn:
            why.append("host namespaces (" + ", ".join(hn) + ")")
        priv = [c.get("name", "") for c in (spec.get("containers") or [])
                if (c.get("securityContext") or {}).get("privileged")]
        if priv:
            why.append("privileged (" + ", ".join(f'container "{n}" must not set securityContext.privileged=true'
                                                   for n in priv) + ")")
        hp = [v.get("name", "") for v in (spec.get("volumes") or []) if "hostPath" in v]
        if hp:
            why.append("hostPath volumes (" + ", ".join(f'volume "{n}"' for n in hp) + ")")
        if not why:
            return None
        return (f'pods "{obj.get("metadata", {}).get("name", "")}" is forbidden: violates PodSecurity '
                f'"{level}:latest": ' + ", ".join(why))

    async def h_collection(self, req, key, ns):
        self.requests += 1
        if req.method == "GET":
            q = req.query
            labels = parse_selector(q.get("labelSelector", ""))
            fields = parse_selector(q.get("fieldSelector", ""))
            if q.get("watch") in ("true", "1"):
                return await self._watch(req, key, ns, labels, fields, q.get("resourceVersion"))
            items = []
            for (ons, _), o in self.objects[key].items():
                if ns is not None and ons != ns:
                    continue
                md = o.get("metadata", {})
                if match_labels(md.get("labels") or {}, labels) and match_fields(o, fields):
                    items.append(o)
            return web.json_response({"kind": RESOURCES[key][0] + "List", "apiVersion": API_VERSIONS.get(key, "v1"),
                                      "metadata": {"resourceVersion": str(self.rv)}, "items": items})
        if req.method == "POST":
            obj = await req.json()
            md = obj.setdefault("metadata", {})
            if ns is not None:
                md["namespace"] = md.get("namespace") or ns
            err = self._admit(key, obj)
            if err:
                return _status(422, "Invalid", err)
            if key == "pods":
                forbidden = self._pod_security(obj)
                if forbidden:
                    return _status(403, "Forbidden", forbidden)
            k = (md.get("namespace") if RESOURCES[key][1] else None, md["name"])
            if k in self.objects[key]:
                return _status(409, "AlreadyExists", f'{key} "{md["name"]}" already exists')
            if key == "pods":
                obj.setdefault("status", {}).setdefault("phase", "Pending")
            md.pop("resourceVersion", None)
            md.pop("uid", None)
            obj = self._store_put(key, obj, "ADDED")
            return web.json_response(obj, status=201)
        if req.method == "DELETE":
            labels = parse_selector(req.query.get("labelSelector", ""))
            gone = []
            for (ons, name), o in list(self.objects[key].items()):
                if (ns is None or ons == ns) and match_labels(o["metadata"].get("labels") or {}, labels):
                    gone.append(self._store_delete(key, ons, name))
            return web.json_response({"kind": "List", "items": gone})
        return _status(405, "MethodNotAllowed", req.method)

    async def h_item(self, req, key, ns):
        self.requests += 1
        name = req.match_info["name"]
        k = (ns, name) if RESOURCES[key][1] else (None, name)
        cur = self.objects[key].get(k)
        if req.method == "GET":
            if cur is None:
                return _status(404, "NotFound", f'{key} "{name}" not found')
            return web.json_response(cur)
        if req.method == "DELETE":
            if cur is None:
                return _status(404, "NotFound", f'{key} "{name}" not found')
            return web.json_response(self._store_delete(key, *k))
        if cur is None:
            return _status(404, "NotFound", f'{key} "{name}" not found')
        if req.method == "PUT":
            obj = await req.json()
            rv = obj.get("metadata", {}).get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                return _status(409, "Conflict", "the object has been modified; please apply your changes to the "
                                                "latest version and try again")
            new = copy.deepcopy(obj)
            new["metadata"]["uid"] = cur["metadata"]["uid"]
            new["metadata"]["creationTimestamp"] = cur["metadata"].get("creationTimestamp")
            if RESOURCES[key][2]:  # status subresource: main-resource writes never touch status
                if "status" in cur:
                    new["status"] = copy.deepcopy(cur["status"])
                else:
                    new.pop("status", None)
            err = self._admit(key, new)
            if err:
                return _status(422, "Invalid", err)
            return web.json_response(self._store_put(key, new))
        if req.method == "PATCH":
            patch = await req.json()
            new = json_merge_patch(copy.deepcopy(cur), patch)
            if RESOURCES[key][2]:
                if "status" in cur:
                    new["status"] = copy.deepcopy(cur["status"])
            new["metadata"]["uid"] = cur["metadata"]["uid"]
            err = self._admit(key, new)
            if err:
                return _status(422, "Invalid", err)
            return web.json_response(self._store_put(key, new))
        return _status(405, "MethodNotAllowed", req.method)

    async def h_status(self, req, key, ns):
        self.requests += 1
        name = req.match_info["name"]
        cur = self.objects[key].get((ns, name))
        if cur is None:
            return _status(404, "NotFound", f'{key} "{name}" not found')
        if req.method == "GET":
            return web.json_response(cur)
        body = await req.json()
        if req.method == "PUT":
            rv = body.get("metadata", {}).get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                return _status(409, "Conflict", "the object has been modified")
            new = copy.deepcopy(cur)
            new["status"] = body.get("status", {})  # status writes never touch spec/metadata
            return web.json_response(self._store_put(key, new))
        if req.method == "PATCH":
            new = copy.deepcopy(cur)
            new["status"] = json_merge_patch(new.get("status", {}), body.get("status", body))
            return web.json_response(self._store_put(key, new))
        return _status(405, "MethodNotAllowed", req.method)

    async def _watch(self, req, key, ns, labels, fields, since):
        resp = web.StreamResponse(headers={"Content-Type": "application/json", "Transfer-Encoding": "chunked"})
        await resp.prepare(req)
        q: asyncio.Queue = asyncio.Queue()
        w = {"key": key, "ns": ns, "labels": labels, "fields": fields, "queue": q}
        self.watchers.append(w)
        try:
            if since not in (None, "", "0"):
                s = int(since)
                if self.events and self.events[0][0] > s + 1 and s < self.rv - self.history:
                    await resp.write((json.dumps({"type": "ERROR", "object": {
                        "kind": "Status", "code": 410, "reason": "Expired",
                        "message": "too old resource version"}}) + "\n").encode())
                    return resp
                for rv, k2, et, o in self.events:
                    if rv > s and k2 == key and self._match(w, o):
                        await resp.write((json.dumps({"type": et, "object": o}) + "\n").encode())
            else:
                for (ons, _), o in list(self.objects[key].items()):
                    if self._match(w, o):
                        await resp.write((json.dumps({"type": "ADDED", "object": o}) + "\n").encode())
            timeout = float(req.query.get("timeoutSeconds", "0") or 0)
            deadline = time.monotonic() + timeout if timeout > 0 else None
            while True:
                wait = None if deadline is None else max(0.0, deadline - time.monotonic())
                if wait is not None and wait <= 0:
                    break
                try:
                    et, o = await asyncio.wait_for(q.get(), timeout=wait if wait is not None else 30.0)
                except asyncio.TimeoutError:
                    if deadline is None:
                        # keep-alive: a BOOKMARK keeps proxies from idling the stream out
                        await resp.write((json.dumps({"type": "BOOKMARK", "object": {
                            "metadata": {"resourceVersion": str(self.rv)}}}) + "\n").encode())
                    continue
                await resp.write((json.dumps({"type": et, "object": o}) + "\n").encode())
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            if w in self.watchers:
                self.watchers.remove(w)
        return resp

    async def h_proxy(self, req):
        ns, svc = req.match_info["ns"], req.match_info["svc"]
        name, _, port = svc.partition(":")
        if self.kubelet is None:
            return _status(503, "ServiceUnavailable", "no kubelet attached")
        addr = self.kubelet.service_address(ns, name, int(port) if port else None)
        if addr is None:
            return _status(503, "ServiceUnavailable", f"no endpoints available for service {name}")
        url = f"http://{addr[0]}:{addr[1]}/{req.match_info['path']}"
        if req.query_string:
            url += "?" + req.query_string
        try:
            async with ClientSession() as s:
                async with s.request(req.method, url, data=await req.read(), timeout=10) as r:
                    body = await r.read()
                    return web.Response(body=body, status=r.status, content_type=r.content_type)
        except Exception as e:  # the replica may exit while answering (/exit)
            return _status(502, "BadGateway", str(e))

    async def h_log(self, req):
        ns, name = req.match_info["ns"], req.match_info["name"]
        if self.kubelet is None:
            return _status(404, "NotFound", "no kubelet")
        path = self.kubelet.log_path(ns, name, req.query.get("container"))
        if path is None:
            return _status(404, "NotFound", f'pod "{name}" has no logs')
        follow = req.query.get("follow") in ("true", "1")
        if not follow:
            with open(path, "rb") as f:
                return web.Response(body=f.read(), content_type="text/plain")
        resp = web.StreamResponse(headers={"Content-Type": "text/plain"})
        await resp.prepare(req)
        with open(path, "rb") as f:
            while True:
                chunk = f.read(65536)
                if chunk:
                    await resp.write(chunk)
                    continue
                if not self.kubelet.is_running(ns, name):
                    rest = f.read()
                    if rest:
                        await resp.write(rest)
                    break
                await asyncio.sleep(0.1)
        return resp

    # ------------------------------------------------------------------ lifecycle
    async def start(self, host="127.0.0.1", port=0):
        self.runner = web.AppRunner(self.app, access_log=None)
        await self.runner.setup()
        site = web.TCPSite(self.runner, host, port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        self.url = f"http://{host}:{self.port}"
        return self.url

    async def stop(self):
        for w in list(self.watchers):
            w["queue"].put_nowait(("BOOKMARK", {"metadata": {"resourceVersion": str(self.rv)}}))
        if self.runner:
            await self.runner.cleanup()
