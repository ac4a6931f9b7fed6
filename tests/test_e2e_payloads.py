"""The bundled payloads run as real TFJobs on the local cluster (CPU, gloo):
the reference's example jobs (examples/v1/dist-mnist, mnist_with_summaries,
estimator-API, distribution_strategy/keras-API) submitted through the SDK,
with TF_CONFIG / WORLD_SIZE from the operator, plus gang scheduling of
GPU-requesting workers (BASELINE config #4)."""
import os
import sys
import time

import pytest

from tf_operator_amd.sdk import container, pod_template
from tf_operator_amd.testing.cluster import LocalCluster

ENV = {"OMP_NUM_THREADS": "1"}


def payload(module, *args, gpus=0, env=None):
    cmd = [sys.executable, "-m", f"tf_operator_amd.examples.{module}", *[str(a) for a in args]]
    return pod_template(container(image="toa/examples:latest", command=cmd, gpus=gpus, env={**ENV, **(env or {})}))


def tfjob(name, specs, annotations=None, **spec):
    md = {"name": name, "namespace": "default"}
    if annotations:
        md["annotations"] = annotations
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": md,
            "spec": {"tfReplicaSpecs": specs, **spec}}


def rs(n, tpl, restart="Never"):
    return {"replicas": n, "restartPolicy": restart, "template": tpl}


def conds(job):
    return [c["type"] for c in (job.get("status") or {}).get("conditions") or [] if c.get("status") == "True"]


@pytest.fixture(scope="module")
def cluster():
    with LocalCluster(gpus=0) as c:
        yield c


def _run(cluster, job, timeout=180):
    c = cluster.client
    c.create(job)
    name = job["metadata"]["name"]
    done = c.wait_for_job(name, polling_interval=0.2, timeout_seconds=timeout)
    logs = {}
    for p in cluster.kubelet.start_times:
        if p[1].startswith(name + "-"):
            path = cluster.kubelet.log_path(p[0], p[1])
            if path:
                logs[p[1]] = open(path).read()
    return done, logs


def test_dist_mnist_allreduce(cluster):
    args = ("--train_steps", 300, "--log_every", 100, "--min_accuracy", 0.3)
    job = tfjob("mnist-ar", {"Chief": rs(1, payload("dist_mnist", *args)),
                             "Worker": rs(2, payload("dist_mnist", *args))})
    done, logs = _run(cluster, job)
    assert "Succeeded" in conds(done), (conds(done), logs)
    chief = logs["mnist-ar-chief-0"]
    assert "rank 0/3" in chief and "accuracy" in chief


def test_dist_mnist_node_local_auto_oneshot():
    """The node-local layout (annotation amd.com/node-local: privileged, one
    GPU per rank) reaches the payload: both ranks get LOCAL_WORLD_SIZE=2 from
    the operator (no TOA_IPC_ALLREDUCE in their env), the local kubelet grants
    node-wide visibility to the privileged containers and names each pod's
    allocated device, and GradBucketer's automatic selection finds the job
    eligible for the one-shot IPC all-reduce -- here only the CPU gradients
    keep it on gloo; on GPUs with RCCL the same decision turns it on."""
    args = ("--train_steps", 40, "--log_every", 20, "--min_accuracy", 0.0)
    job = tfjob("mnist-nl", {"Worker": rs(2, payload("dist_mnist", *args, gpus=1,
                                                      env={"TOA_NO_GPU": "1"}))},
                annotations={"amd.com/node-local": "privileged"})
    names = ("mnist-nl-worker-0", "mnist-nl-worker-1")
    with LocalCluster(gpus=2) as c2:
        c2.client.create(job)
        # the pods as the operator created them (they may be cleaned up once the job ends)
        pods = c2.wait(lambda: [c2.api.get("pods", "default", n) for n in names]
                       if all(c2.api.get("pods", "default", n) for n in names) else None, 60, what="pods")
        envs = {n: c2.kubelet._build_env(p, p["spec"]["containers"][0], [int(n[-1])]) for n, p in zip(names, pods)}
        done = c2.client.wait_for_job("mnist-nl", polling_interval=0.2, timeout_seconds=180)
        logs = {p[1]: open(c2.kubelet.log_path(p[0], p[1])).read() for p in c2.kubelet.start_times
                if p[1].startswith("mnist-nl-") and c2.kubelet.log_path(p[0], p[1])}
    assert "Succeeded" in conds(done), (conds(done), logs)
    for name in ("mnist-nl-worker-0", "mnist-nl-worker-1"):
        assert "one-shot IPC off (eligible (2 ranks on this node" in logs[name], logs[name]
        assert envs[name]["TOA_LOCAL_DEVICE"] == name[-1] and "HIP_VISIBLE_DEVICES" not in envs[name]


@pytest.mark.parametrize("sync", [False, True])
def test_dist_mnist_parameter_server(cluster, sync):
    args = ["--train_steps", 200, "--log_every", 50, "--min_accuracy", 0.2]
    if sync:
        args += ["--sync_replicas", "--replicas_to_aggregate", 2]
    name = "mnist-ps-sync" if sync else "mnist-ps"
    job = tfjob(name, {"PS": rs(1, payload("dist_mnist", *args)), "Worker": rs(2, payload("dist_mnist", *args))})
    done, logs = _run(cluster, job)
    assert "Succeeded" in conds(done), (conds(done), logs)
    w0 = logs[f"{name}-worker-0"]
    assert "ps" in w0.lower() and "accuracy" in w0


def test_tf_smoke_in_graph_replication(cluster):
    """tf_smoke.py analog: the chief checks a 10x10
    multiply from every task of Chief + 2 Workers (all-gather); the PS
    replica never exits and the job still succeeds on the chief."""
    tpl = payload("smoke")
    job = tfjob("smoke", {"Chief": rs(1, tpl), "Worker": rs(2, tpl), "PS": rs(1, tpl)},
                runPolicy={"cleanPodPolicy": "All"})
    done, logs = _run(cluster, job)
    assert "Succeeded" in conds(done), (conds(done), logs)
    assert "smoke ok on 3 task(s)" in logs["smoke-chief-0"], logs["smoke-chief-0"]


def test_mnist_with_summaries(cluster, tmp_path):
    job = tfjob("summaries", {"Worker": rs(1, payload("mnist_with_summaries", "--max_steps", 60,
                                                      "--log_dir", tmp_path))})
    done, logs = _run(cluster, job)
    assert "Succeeded" in conds(done), logs
    assert any(f.endswith(".jsonl") or "events" in f for _, _, fs in os.walk(tmp_path) for f in fs)


def test_estimator_with_evaluator(cluster, tmp_path):
    ck = str(tmp_path / "est")
    tpl = payload("estimator", "--steps", 100, "--ckpt_dir", ck, "--eval_timeout", 60)
    job = tfjob("est", {"Chief": rs(1, tpl), "Worker": rs(1, tpl), "Evaluator": rs(1, tpl)},
                successPolicy="AllWorkers")
    done, logs = _run(cluster, job)
    assert "Succeeded" in conds(done), (conds(done), logs)
    ev = logs.get("est-evaluator-0", "")
    assert "evaluated checkpoint" in ev, ev


def test_keras_cnn_multiworker_resume(cluster, tmp_path):
    ck = str(tmp_path / "keras")
    tpl = payload("keras_cnn", "--epochs", 1, "--steps_per_epoch", 5, "--batch_per_replica", 16,
                  "--saved_model_dir", ck)
    done, logs = _run(cluster, tfjob("keras", {"Worker": rs(2, tpl)}))
    assert "Succeeded" in conds(done), logs
    cluster.client.delete("keras")
    cluster.wait(lambda: not cluster.pods(labels={"job-name": "keras"}), 20, what="keras cleanup")
    tpl2 = payload("keras_cnn", "--epochs", 2, "--steps_per_epoch", 5, "--batch_per_replica", 16,
                   "--saved_model_dir", ck)
    done, logs = _run(cluster, tfjob("keras2", {"Worker": rs(2, tpl2)}))
    assert "Succeeded" in conds(done), logs
    assert "resumed" in logs["keras2-worker-0"]


def test_gang_scheduling_all_or_nothing(tmp_path):
    """Two Worker=2 jobs on a 3-GPU node with gang scheduling: the second
    job's PodGroup is never partially admitted; it runs once the first ends."""
    sleep = pod_template(container(image="x", command=[sys.executable, "-c", "import time; time.sleep(2.5)"],
                                   gpus=1))
    with LocalCluster(gpus=3, enable_gang_scheduling=True) as c:
        c.client.create(tfjob("gang-a", {"Worker": rs(2, sleep)}))
        c.wait(lambda: len([p for p in c.pods(labels={"job-name": "gang-a"})
                            if (p.get("status") or {}).get("phase") == "Running"]) == 2, 30, what="gang-a running")
        c.client.create(tfjob("gang-b", {"Worker": rs(2, sleep)}))
        time.sleep(1.0)
        b = c.pods(labels={"job-name": "gang-b"})
        assert len(b) == 2 and all((p.get("status") or {}).get("phase") in (None, "Pending") for p in b)
        pg = c.api.get("scheduling.volcano.sh/podgroups", "default", "gang-b")
        assert pg["spec"]["minMember"] == 2 and pg["spec"]["minResources"]["amd.com/gpu"] == "2"
        for p in b:
            assert p["spec"]["schedulerName"] == "volcano"
        done = c.client.wait_for_job("gang-b", polling_interval=0.2, timeout_seconds=60)
        assert "Succeeded" in conds(done)
        sa = min(t[0] for k, t in c.kubelet.start_times.items() if k[1].startswith("gang-b"))
        starts_b = [t[0] for k, t in c.kubelet.start_times.items() if k[1].startswith("gang-b")]
        assert max(starts_b) - sa < 0.5  # admitted together
