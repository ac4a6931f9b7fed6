"""Local kubelet + scheduler simulator: runs Pods as local processes.

Lets the whole operator stack run end-to-end on one machine (SURVEY 7.1
item 2; replaces the reference's EKS-based E2E):

* **scheduling**: a pod is bound when its ``amd.com/gpu`` request fits the
  node's free GPUs (each pod gets exclusive device indices, exported as
  ``HIP_VISIBLE_DEVICES`` -- the role the AMD device plugin plays on a real
  node).  A pod of the operator's node-local layout (annotation
  ``amd.com/gpu-visibility=node`` with ``hostIPC``, csrc/core/nodelocal.cc;
  on a real node its /dev/kfd + /dev/dri host mounts do the same) instead
  sees every GPU of the node, with its own device named in
  ``TOA_LOCAL_DEVICE``: the single-node data-parallel layout in which RCCL
  sees all peers and picks its P2P/xGMI transport directly.
  ``device_visibility="node"`` (``TOA_KUBELET_DEVICES=node``) forces that
  view for every pod;
  ``schedulerName: volcano`` pods are gang-admitted only when their
  PodGroup's ``minMember`` pods all fit at once (Volcano semantics);
* **networking**: every per-replica headless Service name gets a unique
  localhost port; MASTER_ADDR/PORT and DMLC_PS_ROOT_* are rewritten to
  ``127.0.0.1:<port>``, cluster-spec strings (TF_CONFIG, TOA_PS_HOSTS) stay
  byte-identical and their endpoints are mapped in ``TOA_ENDPOINT_MAP``; the
  replica learns its own port from ``PORT``;
* **lifecycle**: phase Pending -> Running -> Succeeded / Failed with
  containerStatuses (exit code, restartCount, start times); restartPolicy
  Always / OnFailure restart the container IN PLACE (restartCount++, as the
  real kubelet does -- E2E replica_restart_policy_tests.py:27-156 checks
  start times), Never leaves the pod terminal; pod deletion -> SIGTERM, then
  SIGKILL after the grace period;
* logs per container, served by the fake API server (``/log``).
"""
from __future__ import annotations

import asyncio
import copy
import json
import logging
import os
import re
import signal
import socket
import subprocess
import sys
import time

from .. import core
from ..operator.kube import ApiError, KubeClient

log = logging.getLogger("tf_operator_amd.kubelet")

SVC_RE = re.compile(r"([a-z0-9]([-a-z0-9]*[a-z0-9])?)\.([a-z0-9]([-a-z0-9]*[a-z0-9])?)\.svc(\.[a-z0-9.-]+)?:(\d+)")
REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


_PORT_RNG = None


def _free_port():
    """A currently free localhost port for a service.  Drawn at random from
    [20000, 32000), below the kernel's ephemeral range: a port handed out by
    bind(0) is the next one the kernel gives ANY process, so two local
    clusters on one host (parallel test workers) would otherwise tend to get
    the same just-released port between this check and the replica's bind."""
    global _PORT_RNG
    if _PORT_RNG is None:
        import random

        _PORT_RNG = random.Random(os.getpid() ^ time.time_ns())
    for _ in range(64):
        p = _PORT_RNG.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _quantity_int(v):
    if v is None:
        return 0
    try:
        return int(float(str(v)))
    except ValueError:
        return 0


_RENDEZVOUS_VARS = {"RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                    "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TF_CONFIG",
                    "TOA_LOCAL_DEVICE", "TOA_POD_DEVICES"}


def _inherited_rendezvous(k: str) -> bool:
    return k in _RENDEZVOUS_VARS or k.startswith("TORCHELASTIC_")


def pod_gpus(pod, resource="amd.com/gpu"):
    n = 0
    for c in pod.get("spec", {}).get("containers", []):
        res = c.get("resources") or {}
        n += _quantity_int((res.get("limits") or {}).get(resource) or (res.get("requests") or {}).get(resource))
    return n


class _Proc:
    def __init__(self, pod, container, gpus):
        self.pod = pod
        self.container = container
        self.gpus = gpus
        self.proc: asyncio.subprocess.Process | None = None
        self.restart_count = 0
        self.started_at = None
        self.finished_at = None
        self.exit_code = None
        self.deleting = False


def _pid_alive(pid: int) -> bool:
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except (OSError, IndexError):
        return False


async def _kill_group_and_wait(pid: int, timeout: float = 10.0):
    try:
        os.killpg(pid, signal.SIGKILL)
    except (ProcessLookupError, PermissionError):
        pass
    deadline = time.monotonic() + timeout
    while _pid_alive(pid) and time.monotonic() < deadline:
        await asyncio.sleep(0.02)


class _ForkedProc:
    """asyncio.subprocess.Process look-alike for a child of the fork server."""

    def __init__(self, pid):
        self.pid = pid
        self.returncode = None
        self._done = asyncio.get_running_loop().create_future()

    def _exited(self, status):
        self.returncode = status
        if not self._done.done():
            self._done.set_result(status)

    async def wait(self):
        return await asyncio.shield(self._done)


class LocalKubelet:
    """warm_python (opt-in; ``TOA_KUBELET_WARM=1`` turns it on): Python
    containers start as forks of a warm interpreter that has already imported
    torch (``forkserver.py``) instead of a cold ``python`` process."""

    def __init__(self, kube: KubeClient, api=None, node_name="mi355x-node-0", gpus=0, workdir="/tmp/toa-kubelet",
                 python=sys.executable, grace_seconds=3.0, restart_backoff=0.2, gpu_resource="amd.com/gpu",
                 warm_python=None, device_visibility=None):
        self.kube = kube
        if device_visibility is None:
            device_visibility = os.environ.get("TOA_KUBELET_DEVICES", "pod")
        if device_visibility not in ("pod", "node"):
            raise ValueError(f"device_visibility must be 'pod' or 'node', not {device_visibility!r}")
        self.device_visibility = device_visibility
        if warm_python is None:
            warm_python = os.environ.get("TOA_KUBELET_WARM", "0") == "1"
        self.warm_python = warm_python
        self._fs = None
        self._pagecache = None  # fork server process
        self._fs_ready = None
        self._fs_pending: dict[int, asyncio.Future] = {}
        self._fs_procs: dict[int, _ForkedProc] = {}
        self._fs_exits: dict[int, int] = {}
        self._fs_seq = 0
        self.api = api
        if api is not None:
            api.kubelet = self
        self.node = node_name
        self.total_gpus = gpus
        self.free_gpus = list(range(gpus))
        self.workdir = workdir
        self.python = python
        self.grace = grace_seconds
        self.restart_backoff = restart_backoff
        self.gpu_resource = gpu_resource
        self.ports: dict[tuple, int] = {}
        self.running: dict[tuple, dict] = {}  # (ns, pod) -> {"procs": [...], "task": Task, "gpus": [...]}
        self.pending: dict[tuple, dict] = {}
        self._stop = asyncio.Event()
        self._tasks = []
        self.start_times: dict[tuple, list] = {}
        self.terminating: dict[tuple, asyncio.Task] = {}  # pods being killed (a same-named successor waits)

    # ---------------------------------------------------------------- service registry
    def service_port(self, ns, name):
        k = (ns, name)
        if k not in self.ports:
            self.ports[k] = _free_port()
        return self.ports[k]

    def service_address(self, ns, name, port=None):
        return ("127.0.0.1", self.service_port(ns, name))

    def log_path(self, ns, name, container=None):
        d = os.path.join(self.workdir, ns, name)
        if not os.path.isdir(d):
            return None
        if container is None:
            logs = sorted(f for f in os.listdir(d) if f.endswith(".log"))
            if not logs:
                return None
            return os.path.join(d, logs[0])
        p = os.path.join(d, f"{container}.log")
        return p if os.path.exists(p) else None

    def is_running(self, ns, name):
        r = self.running.get((ns, name))
        return bool(r and any(p.proc is not None and p.proc.returncode is None for p in r["procs"]))

    # ---------------------------------------------------------------- env rewriting
    def _rewrite_env(self, pod, env: dict) -> dict:
        ns = pod["metadata"].get("namespace", "default")
        me = pod["metadata"]["name"]

        # Cluster-spec strings (TF_CONFIG, TOA_PS_HOSTS, ...) stay byte-identical
        # to what the operator injected; every service endpoint they mention is
        # published in TOA_ENDPOINT_MAP ("svc.ns.svc:port" -> "127.0.0.1:port")
        # and resolved by tf_operator_amd.train.dist.resolve_endpoint().
        out = dict(env)
        emap = {}
        for v in env.values():
            if isinstance(v, str):
                for m in SVC_RE.finditer(v):
                    emap[m.group(0)] = f"127.0.0.1:{self.service_port(m.group(3), m.group(1))}"
        # bare service names with a separate port: MX_CONFIG urls, XGBoost WORKER_ADDRS
        import json as _json

        if env.get("MX_CONFIG"):
            try:
                for ups in (_json.loads(env["MX_CONFIG"]).get("cluster") or {}).values():
                    for u in ups:
                        emap[f"{u['url']}:{u['port']}"] = f"127.0.0.1:{self.service_port(ns, u['url'])}"
            except (ValueError, KeyError, TypeError):
                pass
        if env.get("WORKER_ADDRS"):
            for w in env["WORKER_ADDRS"].split(","):
                emap[f"{w}:{env.get('WORKER_PORT', '')}"] = f"127.0.0.1:{self.service_port(ns, w)}"
        if emap:
            out["TOA_ENDPOINT_MAP"] = _json.dumps(emap, separators=(",", ":"))

        def host_to_port(host):
            if host in ("localhost", "127.0.0.1"):
                return self.service_port(ns, me)
            parts = host.split(".")
            hns = parts[1] if len(parts) > 2 and parts[2] == "svc" else ns
            return self.service_port(hns, parts[0])

        if "MASTER_ADDR" in env:
            out["MASTER_PORT"] = str(host_to_port(env["MASTER_ADDR"]))
            out["MASTER_ADDR"] = "127.0.0.1"
        if env.get("DMLC_PS_ROOT_URI"):
            out["DMLC_PS_ROOT_PORT"] = str(host_to_port(env["DMLC_PS_ROOT_URI"]))
            out["DMLC_PS_ROOT_URI"] = "127.0.0.1"
        return out

    # ---------------------------------------------------------------- status
    async def _put_status(self, pod_key, mutate):
        ns, name = pod_key
        for _ in range(5):
            try:
                cur = await self.kube.get("pods", ns, name)
            except ApiError:
                return
            st = copy.deepcopy(cur.get("status") or {})
            mutate(st)
            cur["status"] = st
            try:
                await self.kube.update_status("pods", ns, cur)
                return
            except ApiError as e:
                if e.status != 409:
                    return

    def _container_statuses(self, procs):
        out = []
        for p in procs:
            s = {"name": p.container["name"], "restartCount": p.restart_count, "image": p.container.get("image", ""),
                 "ready": p.exit_code is None and p.proc is not None}
            if p.exit_code is None and p.proc is not None:
                s["state"] = {"running": {"startedAt": core.rfc3339(p.started_at)}}
            elif p.exit_code is not None:
                s["state"] = {"terminated": {"exitCode": p.exit_code,
                                             "reason": "Completed" if p.exit_code == 0 else "Error",
                                             "startedAt": core.rfc3339(p.started_at),
                                             "finishedAt": core.rfc3339(p.finished_at or time.time())}}
            else:
                s["state"] = {"waiting": {"reason": "ContainerCreating"}}
            out.append(s)
        return out

    # ---------------------------------------------------------------- scheduling
    def _gang_ready(self, pod):
        """Volcano admission: all minMember pods of the group fit together."""
        ann = pod["metadata"].get("annotations") or {}
        group = ann.get("scheduling.k8s.io/group-name")
        if not group or pod.get("spec", {}).get("schedulerName") != "volcano" or self.api is None:
            return True, [pod]
        ns = pod["metadata"].get("namespace", "default")
        pg = self.api.get("scheduling.volcano.sh/podgroups", ns, group)
        if pg is None:
            return False, []
        min_member = int(pg.get("spec", {}).get("minMember", 1))
        members = [p for (pns, pname), p in ((k, v["pod"]) for k, v in self.pending.items())
                   if pns == ns and (pns, pname) not in self.terminating and (p["metadata"].get("annotations") or {}).get("scheduling.k8s.io/group-name") == group]
        if len(members) < min_member:
            return False, []
        need = sum(pod_gpus(p, self.gpu_resource) for p in members)
        if need > len(self.free_gpus):
            return False, []
        pg_status = dict(pg.get("status") or {})
        pg_status.update({"phase": "Running", "running": len(members)})
        self.api.put_status("scheduling.volcano.sh/podgroups", ns, group, pg_status)
        return True, members

    async def _try_schedule(self):
        for key in list(self.pending):
            if key not in self.pending:
                continue
            if key in self.terminating:
                continue
            pod = self.pending[key]["pod"]
            ok, members = self._gang_ready(pod)
            if not ok:
                continue
            if len(members) == 1:
                need = pod_gpus(pod, self.gpu_resource)
                if need > len(self.free_gpus):
                    if not self.pending[key].get("unsched_reported"):
                        self.pending[key]["unsched_reported"] = True
                        await self._put_status(key, lambda st: st.update({
                            "phase": "Pending", "conditions": [{"type": "PodScheduled", "status": "False",
                                                                "reason": "Unschedulable",
                                                                "message": f"0/1 nodes are available: 1 Insufficient "
                                                                           f"{self.gpu_resource}."}]}))
                    continue
            for m in members:
                mk = (m["metadata"].get("namespace", "default"), m["metadata"]["name"])
                if mk not in self.pending:
                    continue
                p = self.pending.pop(mk)["pod"]
                need = pod_gpus(p, self.gpu_resource)
                gpus = [self.free_gpus.pop(0) for _ in range(need)]
                self._start_pod(p, gpus)

    # ---------------------------------------------------------------- running
    def _start_pod(self, pod, gpus):
        key = (pod["metadata"].get("namespace", "default"), pod["metadata"]["name"])
        procs = [_Proc(pod, c, gpus) for c in pod.get("spec", {}).get("containers", [])]
        rec = {"procs": procs, "gpus": gpus, "pod": pod}
        self.running[key] = rec
        rec["task"] = asyncio.create_task(self._run_pod(key, rec))

    def _node_visible(self, pod, container) -> bool:
        """Node-wide GPU visibility for this pod: the node is configured that
        way (TOA_KUBELET_DEVICES=node), or the pod qualifies the way a real
        node decides it.  A container sees the node's other GPUs only when
        they are in its device cgroup, i.e. when it is privileged; a hostPath
        mount of /dev/dri does not do it.  So: the operator's node-local mark
        (amd.com/gpu-visibility=node, csrc/core/nodelocal.cc) AND hostIPC AND
        this container privileged.  The annotation alone grants nothing."""
        if self.device_visibility == "node":
            return True
        md = pod.get("metadata") or {}
        spec = pod.get("spec") or {}
        return ((md.get("annotations") or {}).get("amd.com/gpu-visibility") == "node"
                and bool(spec.get("hostIPC"))
                and (container.get("securityContext") or {}).get("privileged") is True)

    def _field_ref(self, pod, path: str):
        """Downward API fieldRef values this kubelet can answer."""
        md = pod.get("metadata") or {}
        return {"metadata.name": md.get("name"), "metadata.namespace": md.get("namespace", "default"),
                "metadata.uid": md.get("uid"), "spec.nodeName": self.node,
                "spec.serviceAccountName": (pod.get("spec") or {}).get("serviceAccountName", "default"),
                "status.hostIP": "127.0.0.1", "status.podIP": "127.0.0.1"}.get(path)

    def _build_env(self, pod, container, gpus):
        env = {}
        for e in container.get("env") or []:
            if "value" in e:
                env[e["name"]] = str(e["value"])
            else:
                ref = ((e.get("valueFrom") or {}).get("fieldRef") or {}).get("fieldPath")
                val = self._field_ref(pod, ref) if ref else None
                if val is not None:
                    env[e["name"]] = str(val)
        env = self._rewrite_env(pod, env)
        ns = pod["metadata"].get("namespace", "default")
        # a real kubelet starts containers from the image's env, not its own:
        # never leak the host process's rendezvous (e.g. a torchrun agent's
        # TORCHELASTIC_USE_AGENT_STORE would send the replica's
        # init_process_group to a store nobody serves)
        base = {k: v for k, v in os.environ.items() if not _inherited_rendezvous(k)}
        base.update(env)
        base["HOSTNAME"] = pod["metadata"]["name"]
        # Every pod of a real node has its own UTS namespace, i.e. its own
        # hostname, and RCCL derives its host identity from the hostname
        # unless NCCL_HOSTID is set: two "pods" of this one-host kubelet would
        # otherwise share an identity a real cluster never grants them.  The
        # pod's own name stands in for its hostname; a value the pod spec
        # provides (the operator's node-local layout: spec.nodeName,
        # csrc/core/nodelocal.cc) overrides it.  A hostNetwork pod shares the
        # node's hostname, so it gets none.
        if not (pod.get("spec") or {}).get("hostNetwork") and "NCCL_HOSTID" not in env:
            base["NCCL_HOSTID"] = pod["metadata"]["name"]
        base["PORT"] = str(self.service_port(ns, pod["metadata"]["name"]))
        base["TOA_POD_NAME"] = pod["metadata"]["name"]
        base["TOA_POD_NAMESPACE"] = ns
        base["TOA_NODE_NAME"] = self.node
        base["PYTHONPATH"] = REPO_ROOT + (os.pathsep + base["PYTHONPATH"] if base.get("PYTHONPATH") else "")
        if gpus and self._node_visible(pod, container):
            base.pop("HIP_VISIBLE_DEVICES", None)
            base.pop("TOA_NO_GPU", None)
            base["TOA_LOCAL_DEVICE"] = str(gpus[0])
            base["TOA_POD_DEVICES"] = ",".join(str(g) for g in gpus)
        elif gpus:
            base["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in gpus)
        else:
            base.pop("HIP_VISIBLE_DEVICES", None)
            base["TOA_NO_GPU"] = "1"
        return base

    def _argv(self, container):
        cmd = list(container.get("command") or []) + [str(a) for a in container.get("args") or []]
        if cmd and cmd[0] in ("python", "python3"):
            cmd[0] = self.python
        return cmd

    async def _run_container(self, key, rec, p: _Proc):
        pod = rec["pod"]
        rp = pod.get("spec", {}).get("restartPolicy", "Always")
        d = os.path.join(self.workdir, key[0], key[1])
        os.makedirs(d, exist_ok=True)
        logf = os.path.join(d, f"{p.container['name']}.log")
        while True:
            argv = self._argv(p.container)
            env = self._build_env(pod, p.container, rec["gpus"])
            with open(logf, "ab") as lf:
                p.started_at = time.time()
                self.start_times.setdefault(key, []).append(p.started_at)
                p.exit_code = None
                try:
                    cold = ((pod.get("metadata") or {}).get("annotations") or {}).get("training.amd.com/start") == "cold"
                    p.proc = None if cold else await self._warm_spawn(argv, env, d, logf)
                    if p.proc is None:
                        p.proc = await asyncio.create_subprocess_exec(*argv, stdout=lf, stderr=subprocess.STDOUT,
                                                                      env=env, cwd=d, start_new_session=True)
                except (FileNotFoundError, PermissionError, IndexError) as e:
                    lf.write(f"failed to start container: {e}\n".encode())
                    p.proc = None
                    p.exit_code = 127
                    p.finished_at = time.time()
                await self._sync_status(key, rec)
                if p.proc is not None:
                    code = await p.proc.wait()
                    p.exit_code = code if code >= 0 else 128 - code  # signal N -> 128+N
                    p.finished_at = time.time()
            if p.deleting or self._stop.is_set():
                return
            restart = rp == "Always" or (rp == "OnFailure" and p.exit_code != 0)
            if not restart:
                await self._sync_status(key, rec)
                return
            p.restart_count += 1
            await self._sync_status(key, rec)
            await asyncio.sleep(min(5.0, self.restart_backoff * (2 ** min(p.restart_count - 1, 5))))
            if p.deleting or self._stop.is_set():
                return

    # ---------------------------------------------------------------- warm starts
    async def _start_forkserver(self):
        env = dict(os.environ)
        env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env.pop("HIP_VISIBLE_DEVICES", None)
        self._fs_ready = asyncio.Event()
        self._fs_lock = asyncio.Lock()
        self._fs = await asyncio.create_subprocess_exec(self.python, "-m", "tf_operator_amd.localkubelet.forkserver",
                                                        stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=env,
                                                        cwd=REPO_ROOT, start_new_session=True)
        self._tasks.append(asyncio.create_task(self._forkserver_reader()))

    async def _forkserver_reader(self):
        while True:
            line = await self._fs.stdout.readline()
            if not line:
                break
            try:
                msg = json.loads(line)
            except ValueError:
                continue
            if "ready" in msg:
                self._fs_ready.set()
            elif "exit" in msg:
                pr = self._fs_procs.pop(msg["exit"], None)
                if pr is not None:
                    pr._exited(int(msg["status"]))
                else:
                    self._fs_exits[msg["exit"]] = int(msg["status"])
            elif "id" in msg:
                fut = self._fs_pending.pop(msg["id"], None)
                if fut is not None and not fut.done():
                    fut.set_result(msg)
        self._fs_ready.clear()  # server gone: cold starts from here on
        for fut in self._fs_pending.values():
            if not fut.done():
                fut.set_result({"error": "fork server exited"})
        self._fs_pending.clear()
        # the forked containers called setsid() and outlive their parent: kill
        # each group and wait until it is really gone before reporting the
        # exit, or a restart would share GPUs/ports with an untracked orphan
        for pid, pr in list(self._fs_procs.items()):
            await _kill_group_and_wait(pid)
            pr._exited(-signal.SIGKILL)
        self._fs_procs.clear()

    def warm_ready(self) -> bool:
        """The fork server has imported torch and takes container starts."""
        return bool(self.warm_python and self._fs is not None and self._fs_ready.is_set())

    async def _warm_spawn(self, argv, env, cwd, logpath):
        """Fork the container off the warm interpreter; None = use a cold start."""
        if not (self.warm_python and self._fs is not None and self._fs_ready.is_set() and len(argv) >= 2
                and argv[0] == self.python and (argv[1] in ("-m", "-c") or argv[1].endswith(".py"))):
            return None
        self._fs_seq += 1
        rid = self._fs_seq
        fut = asyncio.get_running_loop().create_future()
        self._fs_pending[rid] = fut
        req = {"id": rid, "argv": argv[1:], "env": env, "cwd": cwd, "log": logpath}
        try:
            async with self._fs_lock:  # one drain() at a time on the pipe
                self._fs.stdin.write((json.dumps(req) + "\n").encode())
                await self._fs.stdin.drain()
            msg = await asyncio.wait_for(fut, 30)
        except (OSError, asyncio.TimeoutError) as e:
            self._fs_pending.pop(rid, None)
            log.warning("fork server: %s; cold start", e)
            return None
        if "pid" not in msg:
            return None
        pr = _ForkedProc(msg["pid"])
        if msg["pid"] in self._fs_exits:  # (cannot happen: the reply precedes the exit) defensive
            pr._exited(self._fs_exits.pop(msg["pid"]))
        else:
            self._fs_procs[msg["pid"]] = pr
        return pr

    async def _sync_status(self, key, rec):
        procs = rec["procs"]
        done = all(p.exit_code is not None and (p.proc is None or p.proc.returncode is not None) for p in procs)
        rp = rec["pod"].get("spec", {}).get("restartPolicy", "Always")
        if done and (rp == "Never" or (rp == "OnFailure" and all(p.exit_code == 0 for p in procs))):
            phase = "Succeeded" if all(p.exit_code == 0 for p in procs) else "Failed"
        else:
            phase = "Running"
        cs = self._container_statuses(procs)

        def mutate(st):
            st["phase"] = phase
            st["podIP"] = "127.0.0.1"
            st["hostIP"] = "127.0.0.1"
            st.setdefault("startTime", core.rfc3339())
            st["containerStatuses"] = cs
            st["conditions"] = [{"type": "PodScheduled", "status": "True"},
                                {"type": "Ready", "status": "True" if phase == "Running" else "False"}]

        await self._put_status(key, mutate)

    async def _run_pod(self, key, rec):
        try:
            await asyncio.gather(*(self._run_container(key, rec, p) for p in rec["procs"]))
        finally:
            if not any(p.deleting for p in rec["procs"]):
                await self._sync_status(key, rec)
            self._release(key)

    def _release(self, key):
        rec = self.running.get(key)
        if rec is None:
            return
        if all(p.proc is None or p.proc.returncode is not None for p in rec["procs"]):
            self.free_gpus.extend(g for g in rec["gpus"] if g < self.total_gpus)
            self.free_gpus.sort()
            rec["gpus"] = []
            self.running.pop(key, None)

    async def _kill(self, key):
        rec = self.running.get(key)
        if rec is None:
            return
        for p in rec["procs"]:
            p.deleting = True
            if p.proc is not None and p.proc.returncode is None:
                try:
                    os.killpg(p.proc.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.monotonic() + self.grace
        for p in rec["procs"]:
            if p.proc is None:
                continue
            try:
                await asyncio.wait_for(p.proc.wait(), timeout=max(0.0, deadline - time.monotonic()))
            except asyncio.TimeoutError:
                try:
                    os.killpg(p.proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                await p.proc.wait()
        self._release(key)

    # ---------------------------------------------------------------- watch loop
    async def _loop(self):
        while not self._stop.is_set():
            try:
                lst = await self.kube.list("pods")
                for pod in lst.get("items", []):
                    await self._on_pod("ADDED", pod)
                async for et, pod in self.kube.watch("pods", None, None, lst["metadata"]["resourceVersion"]):
                    if self._stop.is_set():
                        return
                    if et in ("BOOKMARK", "ERROR"):
                        if et == "ERROR":
                            break
                        continue
                    await self._on_pod(et, pod)
            except asyncio.CancelledError:
                return
            except Exception as e:
                if self._stop.is_set():
                    return
                log.warning("kubelet watch: %s", e)
                await asyncio.sleep(0.3)

    async def _on_pod(self, et, pod):
        key = (pod["metadata"].get("namespace", "default"), pod["metadata"]["name"])
        if et == "DELETED" or pod.get("metadata", {}).get("deletionTimestamp"):
            if et == "DELETED":
                self.pending.pop(key, None)
            if key in self.running and key not in self.terminating:
                # kill concurrently: deleting a whole elastic generation must
                # not serialise N grace periods
                t = asyncio.create_task(self._kill(key))
                self.terminating[key] = t
                t.add_done_callback(lambda _t, k=key: self.terminating.pop(k, None))
            return
        if key in self.pending:
            return
        if key in self.running and key not in self.terminating:
            return
        if (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
            return
        if (pod.get("status") or {}).get("phase") == "Running":
            return  # owned by a previous kubelet incarnation
        self.pending[key] = {"pod": pod}
        await self._try_schedule()

    async def _scheduler(self):
        while not self._stop.is_set():
            await asyncio.sleep(0.1)
            if self.pending:
                await self._try_schedule()

    # ---------------------------------------------------------------- node object
    def node_object(self):
        q = str(self.total_gpus)
        res = {self.gpu_resource: q, "cpu": str(os.cpu_count() or 1)}
        return {"apiVersion": "v1", "kind": "Node",
                "metadata": {"name": self.node, "labels": {"kubernetes.io/hostname": self.node,
                                                           "amd.com/gpu.product-name": "MI355X"}},
                "status": {"capacity": dict(res), "allocatable": dict(res),
                           "conditions": [{"type": "Ready", "status": "True"}]}}

    async def _register_node(self):
        body = self.node_object()
        try:
            cur = await self.kube.get("nodes", None, self.node)
            cur["status"] = body["status"]
            await self.kube.update_status("nodes", None, cur)
        except ApiError:
            try:
                await self.kube.create("nodes", None, body)
            except ApiError:
                pass

    # ---------------------------------------------------------------- device metrics
    def gpu_owners(self) -> dict:
        """{device index: (namespace, pod, container)} of the running pods --
        the attribution the node agent gives the accelerator series."""
        out = {}
        for (ns, name), rec in self.running.items():
            ctrs = [c.get("name", "") for c in (rec.get("pod") or {}).get("spec", {}).get("containers", [])]
            for g in rec.get("gpus") or []:
                out[g] = (ns, name, ctrs[0] if ctrs else "")
        return out

    def gpu_metrics_text(self, sysfs_root: str | None = None) -> str:
        """cAdvisor-style ``container_accelerator_*`` series for this node's
        GPUs, attributed to the pods holding them (utils/gpu_metrics.py).
        On the real sysfs only the GPUs this node can open are listed (device
        index i = the i-th of them), not every card of a shared host."""
        from ..utils import gpu_metrics

        devs = (gpu_metrics.read_devices(sysfs_root) if sysfs_root
                else gpu_metrics.read_devices(gpu_metrics.SYSFS_DRM, accessible_only=True))
        return gpu_metrics.exposition(devs, self.gpu_owners())

    async def set_capacity(self, gpus: int):
        """Change the node's allocatable GPUs (fault injection: a device or
        node slice lost / returned).  Devices >= `gpus` are not handed out
        again; pods already holding them keep running until they end."""
        self.total_gpus = int(gpus)
        used = {g for rec in self.running.values() for g in rec["gpus"]}
        self.free_gpus = sorted(g for g in range(self.total_gpus) if g not in used)
        await self._register_node()

    async def start(self):
        os.makedirs(self.workdir, exist_ok=True)
        await self._register_node()
        self._tasks = [asyncio.create_task(self._loop()), asyncio.create_task(self._scheduler())]
        if self.total_gpus > 0 and os.environ.get("TOA_KUBELET_PAGECACHE", "1") != "0":
            # node agent: GPU code objects into the page cache (pagecache.py; no GPU touched)
            try:
                self._pagecache = await asyncio.create_subprocess_exec(
                    self.python, "-m", "tf_operator_amd.localkubelet.pagecache", stdout=subprocess.DEVNULL,
                    stderr=subprocess.DEVNULL, env={**os.environ, "PYTHONPATH": REPO_ROOT}, start_new_session=True)
            except OSError as e:
                log.warning("page-cache warmer not started: %s", e)
        if self.warm_python:
            await self._start_forkserver()  # not awaited ready: cold starts until it is

    def node_warm(self) -> bool:
        """The page-cache warmer (the node's image pre-pull analogue) has
        finished, or none runs."""
        pc = self._pagecache
        return pc is None or pc.returncode is not None

    async def stop(self):
        self._stop.set()
        for key in list(self.running):
            await self._kill(key)
        pc, self._pagecache = self._pagecache, None
        if pc is not None and pc.returncode is None:  # the page-cache warmer: end it, reap it
            try:
                os.killpg(pc.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
            try:
                await asyncio.wait_for(pc.wait(), 5)
            except asyncio.TimeoutError:
                try:
                    os.killpg(pc.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                await pc.wait()
        if self._fs is not None and self._fs.returncode is None:
            self._fs.stdin.close()  # the server's loop ends on EOF
            try:
                await asyncio.wait_for(self._fs.wait(), 5)
            except asyncio.TimeoutError:
                self._fs.kill()
                await self._fs.wait()
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
