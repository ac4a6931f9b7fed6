"""The single-node xGMI layout on a real cluster's terms (verdict r3 item 2,
ADVICE r3 high): opt-in only, privileged for peer access, the allocated GPU
bound by PCI address from the kubelet's pod-resources API (never LOCAL_RANK),
a PodSecurity rejection surfaced as an event, and the local kubelet granting
node visibility by the same rule a real node applies."""
import pytest

from tf_operator_amd.bench.flagship import transport_ok
from tf_operator_amd.sdk import container, pod_template
from tf_operator_amd.testing.cluster import LocalCluster
from tf_operator_amd.train import devices

PODS = [
    {"name": "other-job-worker-0", "namespace": "default",
     "containers": [{"name": "tensorflow", "devices": [{"resource_name": "amd.com/gpu", "device_ids": ["0000:05:00.0"]}]}]},
    {"name": "llama-worker-3", "namespace": "team-a",
     "containers": [{"name": "sidecar", "devices": []},
                    {"name": "tensorflow", "devices": [
                        {"resource_name": "amd.com/gpu", "device_ids": ["0000:c1:00.0"]},
                        {"resource_name": "rdma/hca", "device_ids": ["mlx5_0"]}]}]},
]
# HIP ordinals of an 8-GPU node, as torch.cuda.get_device_properties reports them
NODE_PCI = [(0, b, 0) for b in (0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xC1, 0xD1)]


def test_pod_resources_protobuf_roundtrip():
    assert devices.decode(devices.encode_response(PODS)) == PODS
    assert devices.decode(b"") == []


def test_allocated_device_is_the_pods_gpu_not_local_rank():
    env = {"TOA_POD_NAME": "llama-worker-3", "TOA_POD_NAMESPACE": "team-a", "LOCAL_RANK": "3"}
    idx = devices.allocated_device_index(env, lister=lambda: devices.decode(devices.encode_response(PODS)),
                                         pci=lambda: NODE_PCI)
    assert idx == 6  # bus c1 = ordinal 6, whatever LOCAL_RANK says


@pytest.mark.parametrize("env,pods,pci,err", [
    ({}, PODS, NODE_PCI, RuntimeError),                                               # no downward API
    ({"TOA_POD_NAME": "ghost", "TOA_POD_NAMESPACE": "x"}, PODS, NODE_PCI, LookupError),  # kubelet does not know it
    ({"TOA_POD_NAME": "llama-worker-3", "TOA_POD_NAMESPACE": "team-a"}, PODS, NODE_PCI[:6], LookupError),  # not visible
    ({"TOA_POD_NAME": "other-job-worker-0", "TOA_POD_NAMESPACE": "default", "TOA_GPU_RESOURCE": "x/y"},
     PODS, NODE_PCI, RuntimeError),                                                   # no GPU of that resource
])
def test_allocated_device_refuses_to_guess(env, pods, pci, err):
    with pytest.raises(err):
        devices.allocated_device_index(env, lister=lambda: pods, pci=lambda: pci)


def test_parse_bdf_forms():
    assert devices.parse_bdf("0000:c1:00.0") == (0, 0xC1, 0)
    assert devices.parse_bdf("c1:00.0") == (0, 0xC1, 0)
    with pytest.raises(ValueError):
        devices.parse_bdf("renderD128")


def test_dist_binds_pod_resources_device(monkeypatch):
    from tf_operator_amd.train import dist

    monkeypatch.delenv("TOA_LOCAL_DEVICE", raising=False)
    monkeypatch.setenv("TOA_DEVICE_SOURCE", "pod-resources")
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.setattr(dist, "_DEVICE_CACHE", {})
    monkeypatch.setattr(devices, "allocated_device_index", lambda: 6)
    assert dist.local_device_index() == 6
    monkeypatch.setenv("TOA_LOCAL_DEVICE", "2")  # the local kubelet's own answer wins
    assert dist.local_device_index() == 2


def _pod(privileged, host_ipc=True, annotated=True):
    c = {"name": "tensorflow"}
    if privileged is not None:
        c["securityContext"] = {"privileged": privileged}
    return {"metadata": {"name": "p", "annotations": {"amd.com/gpu-visibility": "node"} if annotated else {}},
            "spec": {"hostIPC": host_ipc, "containers": [c]}}


@pytest.mark.parametrize("privileged,host_ipc,annotated,visible", [
    (True, True, True, True),
    (None, True, True, False),    # annotation + hostIPC alone: a real node would not put the peers in the cgroup
    (False, True, True, False),
    (True, False, True, False),
    (True, True, False, False),
])
def test_kubelet_node_visibility_needs_privileged(privileged, host_ipc, annotated, visible):
    from tf_operator_amd.localkubelet.kubelet import LocalKubelet

    kl = LocalKubelet.__new__(LocalKubelet)
    kl.device_visibility = None
    pod = _pod(privileged, host_ipc, annotated)
    assert kl._node_visible(pod, pod["spec"]["containers"][0]) is visible


def test_podsecurity_rejection_is_an_event_not_a_silent_pending():
    with LocalCluster(gpus=2) as c:
        c.run(_put_namespace(c, "restricted", "baseline"))
        tpl = pod_template(container(image="x", command=["python", "-c", "pass"], gpus=1))
        job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
               "metadata": {"name": "nl", "namespace": "restricted", "annotations": {"amd.com/node-local": "privileged"}},
               "spec": {"tfReplicaSpecs": {"Worker": {"replicas": 2, "restartPolicy": "Never", "template": tpl}}}}
        c.client.create(job, namespace="restricted")

        def forbidden():
            return [e for e in c.events("restricted") if e.get("reason") == "NodeLocalForbidden"]

        evs = c.wait(forbidden, timeout=30, what="NodeLocalForbidden event")
        assert 'violates PodSecurity "baseline:latest"' in evs[0]["message"]
        assert "hostIPC=true" in evs[0]["message"] and "privileged" in evs[0]["message"]
        assert not c.pods("restricted")
        # the same job without the annotation runs in that namespace
        job2 = {**job, "metadata": {"name": "plain", "namespace": "restricted"}}
        c.client.create(job2, namespace="restricted")
        done = c.client.wait_for_job("plain", namespace="restricted", polling_interval=0.2, timeout_seconds=60)
        assert [x["type"] for x in done["status"]["conditions"]][-1] == "Succeeded"


async def _put_namespace(c, name, level):
    c.api._store_put("namespaces", {"apiVersion": "v1", "kind": "Namespace",
                                    "metadata": {"name": name, "labels": {
                                        "pod-security.kubernetes.io/enforce": level}}}, "ADDED")


@pytest.mark.parametrize("trans,n,ok", [
    ({"P2P/IPC": 48}, 8, True),
    ({"P2P/IPC": 40, "P2P/direct pointer": 8}, 8, True),
    ({"P2P/IPC": 40, "SHM/direct/direct": 8}, 8, False),
    ({"NET/Socket/0": 16}, 2, False),
    ({}, 8, None),
    ({"SHM/direct/direct": 4}, 1, None),
])
def test_bench_flags_a_degraded_one_node_transport(trans, n, ok):
    assert transport_ok({"channel_connections_by_transport": trans}, n) is ok
    assert transport_ok(None, 8) is None


def _kubelet():
    from tf_operator_amd.localkubelet.kubelet import LocalKubelet

    kl = LocalKubelet.__new__(LocalKubelet)
    kl.device_visibility = None
    kl.node = "node-a"
    kl._rewrite_env = lambda pod, env: env
    kl.service_port = lambda ns, name: 2222
    return kl


def test_kubelet_gives_each_pod_its_own_rccl_host_identity():
    """On a real node every pod has its own hostname, which RCCL hashes into
    its host identity: the one-host local kubelet emulates that with a
    per-pod NCCL_HOSTID, so a job that needs one identity for its ranks must
    say so (the operator's node-local layout: spec.nodeName)."""
    kl = _kubelet()
    a = {"metadata": {"name": "job-worker-0", "namespace": "ns"}, "spec": {"containers": [{"name": "c"}]}}
    b = {"metadata": {"name": "job-worker-1", "namespace": "ns"}, "spec": {"containers": [{"name": "c"}]}}
    ea = kl._build_env(a, a["spec"]["containers"][0], [])
    eb = kl._build_env(b, b["spec"]["containers"][0], [])
    assert ea["NCCL_HOSTID"] == "job-worker-0" and eb["NCCL_HOSTID"] == "job-worker-1"
    hn = {"metadata": {"name": "h", "namespace": "ns"}, "spec": {"hostNetwork": True, "containers": [{"name": "c"}]}}
    assert kl._build_env(hn, hn["spec"]["containers"][0], []).get("NCCL_HOSTID") != "h"  # shares the node's hostname


def test_kubelet_operator_node_local_env_overrides_the_per_pod_identity():
    """The node-local rank pods the C++ core builds carry NCCL_HOSTID from
    spec.nodeName: the kubelet resolves that fieldRef, so every rank reports
    the node, and RCCL sees one host."""
    from tf_operator_amd import core
    from tf_operator_amd.testing import fixtures as fx

    job = fx.new_tfjob(3, 0)
    for s in job["spec"]["tfReplicaSpecs"].values():
        s["template"]["spec"]["containers"][0]["resources"] = {"limits": {"amd.com/gpu": 1}}
    job["metadata"]["annotations"] = {"amd.com/node-local": "privileged"}
    res = core.reconcile(job, [], [], now=0.0, options={})
    pods = [a["pod"] for a in res["actions"] if a["op"] == "create_pod"]
    assert len(pods) == 3
    kl = _kubelet()
    ids = {kl._build_env(p, p["spec"]["containers"][0], [0])["NCCL_HOSTID"] for p in pods}
    assert ids == {"node-a"}
    assert all(p["spec"]["hostPID"] is True for p in pods)
