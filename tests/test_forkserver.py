"""Warm-interpreter fork server (tf_operator_amd/localkubelet/forkserver.py).

A forked child takes the container's argv / env / cwd / log file, runs in a
session of its own (the kubelet signals the process group) and its exit
status comes back over the protocol; with ``warm_python`` the local kubelet
starts Python containers through it.  The GPU case checks that HIP
initialises in the child while the server itself never opens the device."""
import json
import os
import signal
import subprocess
import sys
import time

import pytest

from tf_operator_amd.sdk import container, pod_template
from tf_operator_amd.testing.cluster import LocalCluster

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Server:
    def __init__(self):
        env = dict(os.environ, PYTHONPATH=REPO)
        self.p = subprocess.Popen([sys.executable, "-m", "tf_operator_amd.localkubelet.forkserver"],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=env, cwd=REPO)
        self.seen = []
        self.n = 0
        assert "ready" in self._read()

    def _read(self):
        line = self.p.stdout.readline()
        assert line, "fork server exited"
        return json.loads(line)

    def spawn(self, argv, tmp, env=None):
        self.n += 1
        log = str(tmp / f"c{self.n}.log")
        req = {"id": self.n, "argv": argv, "env": dict(os.environ, **(env or {})), "cwd": str(tmp), "log": log}
        self.p.stdin.write((json.dumps(req) + "\n").encode())
        self.p.stdin.flush()
        while True:
            m = self._read()
            if m.get("id") == self.n:
                assert "pid" in m, m
                return m["pid"], log
            self.seen.append(m)

    def wait(self, pid):
        while True:
            for m in self.seen:
                if m.get("exit") == pid:
                    return m["status"]
            self.seen.append(self._read())

    def close(self):
        self.p.stdin.close()
        self.p.wait(30)


@pytest.fixture(scope="module")
def server():
    s = _Server()
    yield s
    s.close()


def _read(path):
    return open(path).read() if os.path.exists(path) else ""


@pytest.mark.timeout(180)
def test_script_gets_env_cwd_argv_and_exit_code(server, tmp_path):
    (tmp_path / "c.py").write_text(
        "import os, sys\n"
        "print('env', os.environ['TOA_X'], 'cwd', os.getcwd(), 'argv', sys.argv[1:],"
        " 'leader', os.getsid(0) == os.getpid())\n"
        "sys.exit(7)\n")
    pid, log = server.spawn([str(tmp_path / "c.py"), "a", "b"], tmp_path, {"TOA_X": "42"})
    assert server.wait(pid) == 7
    assert f"env 42 cwd {tmp_path} argv ['a', 'b'] leader True" in _read(log)


@pytest.mark.timeout(120)
def test_module_and_uncaught_exception(server, tmp_path):
    (tmp_path / "toa_fs_mod.py").write_text("import sys\nprint('main', __name__, sys.argv[1:])\n")
    pid, log = server.spawn(["-m", "toa_fs_mod", "x"], tmp_path)
    assert server.wait(pid) == 0
    assert "main __main__ ['x']" in _read(log)
    pid, log = server.spawn(["-c", "raise ValueError('boom')"], tmp_path)
    assert server.wait(pid) == 1
    assert "ValueError: boom" in _read(log)


@pytest.mark.timeout(120)
def test_sigkill_reports_negative_signal(server, tmp_path):
    pid, log = server.spawn(["-c", "import time; print('up', flush=True); time.sleep(60)"], tmp_path)
    deadline = time.time() + 30
    while "up" not in _read(log) and time.time() < deadline:
        time.sleep(0.05)
    os.killpg(pid, signal.SIGKILL)  # the child leads its own process group
    assert server.wait(pid) == -signal.SIGKILL


@pytest.mark.timeout(240)
def test_kubelet_starts_python_containers_warm():
    cmd = [sys.executable, "-c", "import os, sys; print('ppid', os.getppid(), 'torch' in sys.modules)"]
    tpl = pod_template(container(image="toa/trainer:latest", command=cmd))
    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": "warm", "namespace": "default"},
           "spec": {"runPolicy": {"cleanPodPolicy": "None"}, "successPolicy": "AllWorkers",
                    "tfReplicaSpecs": {"Worker": {"replicas": 2, "restartPolicy": "Never", "template": tpl}}}}
    with LocalCluster(kinds=("TFJob",), warm_python=True) as c:
        c.wait(lambda: c.kubelet._fs_ready is not None and c.kubelet._fs_ready.is_set(), 180,
               what="fork server ready")
        c.client.create(job)

        def done():
            conds = [x["type"] for x in ((c.client.get("warm").get("status") or {}).get("conditions") or [])
                     if x.get("status") == "True"]
            return "Succeeded" in conds or "Failed" in conds

        c.wait(done, 60, what="job finished")
        want = f"ppid {c.kubelet._fs.pid} True"
        c.wait(lambda: all(want in v for v in c.client.get_logs("warm", master=False).values()), 30, what="logs")
        logs = c.client.get_logs("warm", master=False)
        assert sorted(logs) == ["warm-worker-0", "warm-worker-1"], logs


@pytest.mark.gpu
@pytest.mark.timeout(180)
def test_hip_initialises_in_the_child_not_the_server(server, tmp_path):
    code = "import torch; x = torch.ones(4, device='cuda'); print('sum', float(x.sum()))"
    pid, log = server.spawn(["-c", code], tmp_path)
    assert server.wait(pid) == 0, _read(log)[-2000:]
    assert "sum 4.0" in _read(log)
    fds = []
    for f in os.listdir(f"/proc/{server.p.pid}/fd"):
        try:
            fds.append(os.readlink(f"/proc/{server.p.pid}/fd/{f}"))
        except OSError:
            pass
    assert not any("kfd" in f for f in fds), fds
