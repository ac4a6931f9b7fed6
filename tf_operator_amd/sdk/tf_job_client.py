"""`TFJobClient` -- the user-facing Python SDK.

Same method names, arguments and semantics as the reference SDK
(sdk/python/kubeflow/tfjob/api/tf_job_client.py:54-442): create / get /
patch / delete / wait_for_job / wait_for_condition / get_job_status
(= type of the LAST condition, :306-318) / is_job_running / is_job_succeeded
/ get_pod_names (label selection, :343-378) / get_logs (follow: one reader
thread + queue per pod, lines forwarded in batches of 50, :380-442).

The `kubernetes` package is not required: requests talks to the API server
directly (kubeconfig, in-cluster service account, or an explicit ``master``
URL such as the in-process fake API server).  ``job_kind`` makes the same
client drive PyTorchJob / MXJob / XGBoostJob.
"""
from __future__ import annotations

import base64
import json
import logging
import os
import queue
import tempfile
import threading
import time

import requests

from . import constants, utils
from .models import _Model

log = logging.getLogger("tf_operator_amd.sdk")


class ApiException(RuntimeError):
    def __init__(self, status, body):
        self.status = status
        self.body = body
        super().__init__(f"({status}) {body}")


class _Rest:
    def __init__(self, master=None, config_file=None, context=None, token=None, verify=True):
        self.session = requests.Session()
        self.verify = verify
        if master:
            self.base = master.rstrip("/")
            if token:
                self.session.headers["Authorization"] = f"Bearer {token}"
            return
        if config_file or os.environ.get("KUBECONFIG") or os.path.exists(os.path.expanduser("~/.kube/config")):
            self._from_kubeconfig(config_file, context)
        elif utils.is_running_in_k8s():
            sa = "/var/run/secrets/kubernetes.io/serviceaccount"
            self.base = f"https://{os.environ['KUBERNETES_SERVICE_HOST']}:{os.environ['KUBERNETES_SERVICE_PORT']}"
            self.session.headers["Authorization"] = "Bearer " + open(os.path.join(sa, "token")).read().strip()
            self.verify = os.path.join(sa, "ca.crt")
        else:
            raise RuntimeError("no API server: pass master=..., a kubeconfig, or run in-cluster")

    def _from_kubeconfig(self, path, context):
        import yaml

        path = path or os.environ.get("KUBECONFIG") or os.path.expanduser("~/.kube/config")
        cfg = yaml.safe_load(open(path))
        ctxn = context or cfg.get("current-context")
        ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == ctxn)
        cl = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
        user = next((u["user"] for u in cfg.get("users", []) if u["name"] == ctx.get("user")), {})
        self.base = cl["server"].rstrip("/")
        if cl.get("insecure-skip-tls-verify"):
            self.verify = False
        elif cl.get("certificate-authority-data"):
            f = tempfile.NamedTemporaryFile(delete=False, suffix=".crt")
            f.write(base64.b64decode(cl["certificate-authority-data"]))
            f.close()
            self.verify = f.name
        elif cl.get("certificate-authority"):
            self.verify = cl["certificate-authority"]
        if user.get("token"):
            self.session.headers["Authorization"] = f"Bearer {user['token']}"
        if user.get("client-certificate-data"):
            c = tempfile.NamedTemporaryFile(delete=False, suffix=".crt")
            c.write(base64.b64decode(user["client-certificate-data"]))
            c.close()
            k = tempfile.NamedTemporaryFile(delete=False, suffix=".key")
            k.write(base64.b64decode(user["client-key-data"]))
            k.close()
            self.session.cert = (c.name, k.name)
        elif user.get("client-certificate"):
            self.session.cert = (user["client-certificate"], user["client-key"])

    def call(self, method, path, body=None, params=None, stream=False, content_type="application/json",
             timeout=constants.APISERVER_TIMEOUT):
        r = self.session.request(method, self.base + path, data=json.dumps(body) if body is not None else None,
                                 params=params, headers={"Content-Type": content_type}, verify=self.verify,
                                 stream=stream, timeout=None if stream else timeout)
        if r.status_code >= 400:
            raise ApiException(r.status_code, r.text)
        if stream:
            return r
        ct = r.headers.get("Content-Type", "")
        return r.json() if "json" in ct else r.text


class TFJobClient:
    def __init__(self, config_file=None, context=None, client_configuration=None, persist_config=True,
                 master=None, token=None, job_kind="TFJob"):
        if isinstance(client_configuration, dict) and not master:
            master = client_configuration.get("host")
            token = token or client_configuration.get("api_key")
        self.rest = _Rest(master=master, config_file=config_file, context=context, token=token)
        self.kind = job_kind
        self.plural = constants.PLURALS[job_kind]

    # ------------------------------------------------------------------ paths
    def _path(self, namespace, name=None):
        p = f"/apis/{constants.TFJOB_GROUP}/{constants.TFJOB_VERSION}/namespaces/{namespace}/{self.plural}"
        return p + (f"/{name}" if name else "")

    @staticmethod
    def _body(tfjob):
        return tfjob.to_dict() if isinstance(tfjob, _Model) else tfjob

    # ------------------------------------------------------------------ CRUD
    def create(self, tfjob, namespace=None):
        body = self._body(tfjob)
        namespace = namespace or utils.set_tfjob_namespace(body)
        try:
            return self.rest.call("POST", self._path(namespace), body)
        except ApiException as e:
            raise RuntimeError(f"Exception when calling CustomObjectsApi->create_namespaced_custom_object: {e}") from e

    def get(self, name=None, namespace=None, watch=False, timeout_seconds=600):
        namespace = namespace or utils.get_default_target_namespace()
        if watch:
            from .watch import watch as _watch

            return _watch(self, name=name, namespace=namespace, timeout_seconds=timeout_seconds)
        try:
            return self.rest.call("GET", self._path(namespace, name))
        except ApiException as e:
            what = "get" if name else "list"
            raise RuntimeError(f"Exception when calling CustomObjectsApi->{what}_namespaced_custom_object: {e}") \
                from e
        except requests.RequestException as e:
            raise RuntimeError(f"There was a problem to get TFJob {name} in namespace {namespace}. Exception: {e}") \
                from e

    def patch(self, name, tfjob, namespace=None):
        body = self._body(tfjob)
        namespace = namespace or utils.set_tfjob_namespace(body)
        try:
            return self.rest.call("PATCH", self._path(namespace, name), body,
                                  content_type="application/merge-patch+json")
        except ApiException as e:
            raise RuntimeError(f"Exception when calling CustomObjectsApi->patch_namespaced_custom_object: {e}") from e

    def delete(self, name, namespace=None):
        namespace = namespace or utils.get_default_target_namespace()
        try:
            return self.rest.call("DELETE", self._path(namespace, name),
                                  {"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": "Foreground"})
        except ApiException as e:
            raise RuntimeError(f"Exception when calling CustomObjectsApi->delete_namespaced_custom_object: {e}") from e

    # ------------------------------------------------------------------ waiting / status
    def wait_for_job(self, name, namespace=None, watch=False, timeout_seconds=600, polling_interval=30,
                     status_callback=None):
        namespace = namespace or utils.get_default_target_namespace()
        if watch:
            self.get(name, namespace, watch=True, timeout_seconds=timeout_seconds)
            return self.get(name, namespace)
        return self.wait_for_condition(name, ["Succeeded", "Failed"], namespace=namespace,
                                       timeout_seconds=timeout_seconds, polling_interval=polling_interval,
                                       status_callback=status_callback)

    def wait_for_condition(self, name, expected_condition, namespace=None, timeout_seconds=600, polling_interval=30,
                           status_callback=None):
        namespace = namespace or utils.get_default_target_namespace()
        expected = [expected_condition] if isinstance(expected_condition, str) else list(expected_condition)
        deadline = time.monotonic() + timeout_seconds
        tfjob = None
        while True:
            tfjob = self.get(name, namespace=namespace)
            if tfjob:
                if status_callback:
                    status_callback(tfjob)
                for c in (tfjob.get("status") or {}).get("conditions") or []:
                    if c.get("type", "") in expected:
                        return tfjob
            if time.monotonic() + polling_interval > deadline:
                break
            time.sleep(polling_interval)
        raise RuntimeError(f"Timeout waiting for TFJob {name} in namespace {namespace} to enter one of the "
                           f"conditions {expected}.", tfjob)

    def get_job_status(self, name, namespace=None):
        tfjob = self.get(name, namespace=namespace)
        conds = (tfjob.get("status") or {}).get("conditions") or [{}]
        return conds[-1].get("type", "")

    def is_job_running(self, name, namespace=None):
        return self.get_job_status(name, namespace).lower() == "running"

    def is_job_succeeded(self, name, namespace=None):
        return self.get_job_status(name, namespace).lower() == "succeeded"

    # ------------------------------------------------------------------ pods / logs
    def get_pod_names(self, name, namespace=None, master=False, replica_type=None, replica_index=None):
        namespace = namespace or utils.get_default_target_namespace()
        labels = utils.get_labels(name, master=master, replica_type=replica_type, replica_index=replica_index)
        try:
            resp = self.rest.call("GET", f"/api/v1/namespaces/{namespace}/pods",
                                  params={"labelSelector": utils.to_selector(labels)})
        except ApiException as e:
            raise RuntimeError(f"Exception when calling CoreV1Api->list_namespaced_pod: {e}") from e
        names = [p["metadata"]["name"] for p in resp.get("items", []) if p.get("metadata", {}).get("name")]
        if not names:
            log.warning("Not found Pods of the TFJob %s with the labels %s.", name, labels)
            return None
        return set(names)

    def _read_log(self, pod, namespace):
        return self.rest.call("GET", f"/api/v1/namespaces/{namespace}/pods/{pod}/log")

    def get_logs(self, name, namespace=None, master=True, replica_type=None, replica_index=None, follow=False,
                 sink=None):
        """Logs of the job's pods (by default the `job-role=master` pod).  Returns
        {pod: text}; each line is also logged (or passed to `sink(pod, line)`)."""
        namespace = namespace or utils.get_default_target_namespace()
        pods = sorted(self.get_pod_names(name, namespace=namespace, master=master, replica_type=replica_type,
                                         replica_index=replica_index) or [])
        if not pods:
            raise RuntimeError(f"Not found Pods of the TFJob {name} in namespace {namespace}")
        emit = sink or (lambda pod, line: log.info("[Pod %s]: %s", pod, line))
        out = {p: "" for p in pods}
        if not follow:
            for p in pods:
                try:
                    out[p] = self._read_log(p, namespace)
                except ApiException as e:
                    raise RuntimeError(f"Exception when calling CoreV1Api->read_namespaced_pod_log: {e}") from e
                log.info("The logs of Pod %s:\n %s", p, out[p])
            return out
        queues = []

        def reader(pod, q):
            try:
                r = self.rest.call("GET", f"/api/v1/namespaces/{namespace}/pods/{pod}/log",
                                   params={"follow": "true"}, stream=True)
                for line in r.iter_lines(decode_unicode=True):
                    q.put(line)
            except Exception as e:  # surface and end this stream
                q.put(f"<log stream error: {e}>")
            q.put(None)

        for p in pods:
            q = queue.Queue(maxsize=50000)
            threading.Thread(target=reader, args=(p, q), daemon=True).start()
            queues.append(q)
        finished = [False] * len(pods)
        while not all(finished):
            for i, q in enumerate(queues):
                if finished[i]:
                    continue
                for _ in range(50):  # batches of 50 lines per pod
                    try:
                        line = q.get(timeout=0.2)
                    except queue.Empty:
                        break
                    if line is None:
                        finished[i] = True
                        break
                    out[pods[i]] += line + "\n"
                    emit(pods[i], line)
        return out
