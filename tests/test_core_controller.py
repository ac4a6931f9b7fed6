"""Ported controller tests (reference: pkg/controller.v1/tensorflow/*_test.go).

Same style as the reference's fake-indexer + FakePodControl tests: feed the
pure C++ reconcile engine observed pods/services and assert on the returned
actions and status.
"""
import json
import os

import pytest

from tf_operator_amd import core
from tf_operator_amd.testing import fixtures as fx

NOW = 1_700_000_000.0


def ops(res, op):
    return [a for a in res["actions"] if a["op"] == op]


def run(job, pods=(), svcs=(), now=NOW, **opt):
    return core.reconcile(job, list(pods), list(svcs), now=now, options=opt)


# ---------------------------------------------------------------------------
# controller_test.go TestNormalPath (8 table cases)
# ---------------------------------------------------------------------------
NORMAL = {
    # name: (worker, ps, wpods(pend,act,succ,fail), pspods(...), wsvc, pssvc,
    #        creates, deletes, svc_creates, wstat(act,succ,fail), psstat, cond)
    "local created": (1, 0, (0, 0, 0, 0), (0, 0, 0, 0), 0, 0, 1, 0, 1, (0, 0, 0), (0, 0, 0), None),
    "dist created": (4, 2, (0, 0, 0, 0), (0, 0, 0, 0), 0, 0, 6, 0, 6, (0, 0, 0), (0, 0, 0), None),
    "all pending": (4, 2, (4, 0, 0, 0), (2, 0, 0, 0), 4, 2, 0, 0, 0, (0, 0, 0), (0, 0, 0), None),
    "all running": (4, 2, (0, 4, 0, 0), (0, 2, 0, 0), 4, 2, 0, 0, 0, (4, 0, 0), (2, 0, 0), "Running"),
    "2w 1ps pending": (4, 2, (2, 0, 0, 0), (1, 0, 0, 0), 2, 1, 3, 0, 3, (0, 0, 0), (0, 0, 0), None),
    "1 worker running": (4, 2, (2, 1, 0, 0), (1, 0, 0, 0), 3, 1, 2, 0, 2, (1, 0, 0), (0, 0, 0), "Running"),
    "1 worker succeeded": (4, 2, (2, 0, 1, 0), (1, 0, 0, 0), 3, 1, 2, 0, 2, (0, 1, 0), (0, 0, 0), None),
    "succeeded": (4, 2, (0, 0, 4, 0), (0, 0, 2, 0), 4, 2, 0, 0, 0, (0, 4, 0), (0, 2, 0), "Succeeded"),
}


@pytest.mark.parametrize("name", list(NORMAL))
def test_normal_path(name):
    w, ps, wp, pp, wsvc, pssvc, creates, deletes, screates, wstat, psstat, cond = NORMAL[name]
    job = fx.new_tfjob(w, ps)
    pods = fx.pods_with_statuses(job, "worker", *wp) + fx.pods_with_statuses(job, "ps", *pp)
    svcs = fx.services(job, "worker", wsvc) + fx.services(job, "ps", pssvc)
    res = run(job, pods, svcs)
    assert len(ops(res, "create_pod")) == creates
    assert len(ops(res, "delete_pod")) == deletes
    assert len(ops(res, "create_service")) == screates
    rs = res["status"]["replicaStatuses"]
    got_w = (rs["Worker"]["active"], rs["Worker"]["succeeded"], rs["Worker"]["failed"])
    assert got_w == wstat
    if ps:
        assert (rs["PS"]["active"], rs["PS"]["succeeded"], rs["PS"]["failed"]) == psstat
    if cond:
        assert fx.check_condition(res["status"], cond, "TFJob" + cond)
    # ControllerRef on every created pod (controller_test.go:270-287)
    for a in ops(res, "create_pod"):
        ref = a["pod"]["metadata"]["ownerReferences"][0]
        assert ref == {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "name": fx.TEST_TFJOB_NAME,
                       "uid": job["metadata"]["uid"], "controller": True, "blockOwnerDeletion": True}
    # startTime is always set on a non-terminal sync
    assert res["status"].get("startTime")


def test_created_pod_contract():
    job = fx.new_tfjob(2, 1, chief=1)
    res = run(job)
    pods = {a["pod"]["metadata"]["name"]: a["pod"] for a in ops(res, "create_pod")}
    assert sorted(pods) == ["test-tfjob-chief-0", "test-tfjob-ps-0", "test-tfjob-worker-0", "test-tfjob-worker-1"]
    chief = pods["test-tfjob-chief-0"]
    lb = chief["metadata"]["labels"]
    assert lb["group-name"] == "kubeflow.org" and lb["job-name"] == "test-tfjob"
    assert lb["replica-type"] == "chief" and lb["replica-index"] == "0" and lb["job-role"] == "master"
    assert "job-role" not in pods["test-tfjob-worker-0"]["metadata"]["labels"]
    assert chief["spec"]["restartPolicy"] == "Never"
    svcs = {a["service"]["metadata"]["name"]: a["service"] for a in ops(res, "create_service")}
    s = svcs["test-tfjob-worker-1"]
    assert s["spec"]["clusterIP"] == "None"
    assert s["spec"]["ports"] == [{"name": "tfjob-port", "port": 2222}]
    assert s["spec"]["selector"]["replica-index"] == "1"
    # expectations to raise for the shell
    keys = {e["key"]: e["add"] for e in res["expect"]}
    assert keys["default/test-tfjob/worker/pods"] == 2
    assert keys["default/test-tfjob/worker/services"] == 2


def test_worker0_is_master_role_without_chief():
    res = run(fx.new_tfjob(2, 0))
    pods = {a["pod"]["metadata"]["name"]: a["pod"] for a in ops(res, "create_pod")}
    assert pods["test-tfjob-worker-0"]["metadata"]["labels"]["job-role"] == "master"
    assert "job-role" not in pods["test-tfjob-worker-1"]["metadata"]["labels"]


def test_copy_labels_and_annotations():
    """job_test.go TestCopyLabelsAndAnnotation: template metadata is preserved."""
    job = fx.new_tfjob(1, 0)
    job["spec"]["tfReplicaSpecs"]["Worker"]["template"]["metadata"] = {"labels": {"label1": "1"},
                                                                       "annotations": {"annotation1": "1"}}
    res = run(job)
    md = ops(res, "create_pod")[0]["pod"]["metadata"]
    assert md["labels"]["label1"] == "1" and md["annotations"]["annotation1"] == "1"


# ---------------------------------------------------------------------------
# pod_test.go TestClusterSpec: byte-exact TF_CONFIG
# ---------------------------------------------------------------------------
CLUSTER_CASES = [
    (fx.new_tfjob(1, 0, namespace="ns0"), "", ""),
    (fx.new_tfjob(1, 0, namespace="ns1"), "tf.training.com", ""),
    (fx.new_tfjob(1, 1, namespace="ns2"), "tf.training.org",
     '{"cluster":{"ps":["test-tfjob-ps-0.ns2.svc.tf.training.org:2222"],"worker":["test-tfjob-worker-0.ns2.svc.'
     'tf.training.org:2222"]},"task":{"type":"worker","index":0},"environment":"cloud"}'),
    (fx.new_tfjob(1, 1, evaluator=1, namespace="ns3"), "tf.training.io",
     '{"cluster":{"evaluator":["test-tfjob-evaluator-0.ns3.svc.tf.training.io:2222"],"ps":["test-tfjob-ps-0.ns3.'
     'svc.tf.training.io:2222"],"worker":["test-tfjob-worker-0.ns3.svc.tf.training.io:2222"]},"task":{"type":'
     '"worker","index":0},"environment":"cloud"}'),
    (fx.new_tfjob(1, 1, evaluator=1, namespace="ns3"), "",
     '{"cluster":{"evaluator":["test-tfjob-evaluator-0.ns3.svc:2222"],"ps":["test-tfjob-ps-0.ns3.svc:2222"],'
     '"worker":["test-tfjob-worker-0.ns3.svc:2222"]},"task":{"type":"worker","index":0},"environment":"cloud"}'),
]


@pytest.mark.parametrize("case", range(len(CLUSTER_CASES)))
def test_cluster_spec(case):
    job, domain, expected = CLUSTER_CASES[case]
    res = run(job, cluster_domain=domain)
    pod = [a["pod"] for a in ops(res, "create_pod") if a["pod"]["metadata"]["name"] == "test-tfjob-worker-0"][0]
    env = {e["name"]: e["value"] for e in pod["spec"]["containers"][0].get("env", [])}
    if expected == "":
        assert "TF_CONFIG" not in env
    else:
        assert env["TF_CONFIG"] == expected
    # the direct generator agrees
    if expected:
        assert core.gen_tf_config(job, "worker", 0, {"cluster_domain": domain}) == expected


def test_sparse_cluster_spec():
    """tensorflow_test.go: EnableDynamicWorker -> sparse TF_CONFIG."""
    job = fx.new_tfjob(2, 2)
    job["spec"]["enableDynamicWorker"] = True
    w = json.loads(core.gen_tf_config(job, "worker", 0))
    assert w == {"sparseCluster": {"worker": {"0": "test-tfjob-worker-0.default.svc:2222"},
                                   "ps": ["test-tfjob-ps-0.default.svc:2222", "test-tfjob-ps-1.default.svc:2222"]},
                 "task": {"type": "worker", "index": 0}}
    p = json.loads(core.gen_tf_config(job, "ps", 0))
    assert p["sparseCluster"] == {"worker": {}, "ps": ["test-tfjob-ps-0.default.svc:2222"]}
    # Go struct field order is preserved
    assert core.gen_tf_config(job, "ps", 1).startswith('{"sparseCluster":{"worker":{},"ps":[')


def test_is_distributed():
    assert not core.tf_is_distributed(fx.new_tfjob(1, 0))
    assert core.tf_is_distributed(fx.new_tfjob(2, 0))
    assert core.tf_is_distributed(fx.new_tfjob(1, 1))
    assert not core.tf_is_distributed(fx.new_tfjob(0, 0, chief=1))


def test_rocm_env_block():
    job = fx.new_tfjob(4, 1, chief=1)
    env = {e["name"]: e["value"] for e in core.gen_env(job, "Worker", 2)}
    assert env["MASTER_ADDR"] == "test-tfjob-chief-0.default.svc"
    assert env["MASTER_PORT"] == "2222"
    assert env["WORLD_SIZE"] == "5"  # chief + 4 workers; PS outside the RCCL world
    assert env["RANK"] == "3"
    assert env["LOCAL_RANK"] == "0" and env["TOA_ROLE"] == "worker"
    assert env["TOA_PS_HOSTS"] == "test-tfjob-ps-0.default.svc:2222"
    ps = {e["name"]: e["value"] for e in core.gen_env(job, "PS", 0)}
    assert "RANK" not in ps and ps["TOA_ROLE"] == "ps"
    off = core.gen_env(job, "Worker", 0, {"inject_rocm_env": False})
    assert [e["name"] for e in off] == ["TF_CONFIG"]
    knobs = {e["name"]: e["value"] for e in core.gen_env(job, "Worker", 0, {"nccl_env": {"NCCL_MIN_NCHANNELS": "32"}})}
    assert knobs["NCCL_MIN_NCHANNELS"] == "32"


def test_rccl_defaults_never_override_user_env():
    """xGMI defaults (envgen.cc kRcclDefaults) are injected into TFJob and
    PyTorchJob trainers unless --nccl-env or the container already sets them."""
    job = fx.new_tfjob(2, 0)
    env = {e["name"]: e["value"] for e in core.gen_env(job, "Worker", 0)}
    assert env["TORCH_NCCL_HIGH_PRIORITY"] == "1"
    assert env["TORCH_NCCL_AVOID_RECORD_STREAMS"] == "1"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    over = {e["name"]: e["value"] for e in core.gen_env(job, "Worker", 0, {"nccl_env": {"TORCH_NCCL_HIGH_PRIORITY": "0"}})}
    assert over["TORCH_NCCL_HIGH_PRIORITY"] == "0"
    assert [e["name"] for e in core.gen_env(job, "Worker", 0, {"nccl_env": {"TORCH_NCCL_HIGH_PRIORITY": "0"}})].count(
        "TORCH_NCCL_HIGH_PRIORITY") == 1
    off = {e["name"] for e in core.gen_env(job, "Worker", 0, {"rccl_defaults": False})}
    assert "TORCH_NCCL_HIGH_PRIORITY" not in off
    # a container that sets one keeps its own value (and gets no duplicate entry)
    tpl = job["spec"]["tfReplicaSpecs"]["Worker"]["template"]
    tpl["spec"]["containers"][0].setdefault("env", []).append({"name": "TORCH_NCCL_HIGH_PRIORITY", "value": "0"})
    out = core.set_cluster_spec(job, tpl, "Worker", 0)
    names = [e["name"] for e in out["spec"]["containers"][0]["env"]]
    assert names.count("TORCH_NCCL_HIGH_PRIORITY") == 1
    assert {e["name"]: e["value"] for e in out["spec"]["containers"][0]["env"]}["TORCH_NCCL_HIGH_PRIORITY"] == "0"
    assert "TORCH_NCCL_AVOID_RECORD_STREAMS" in names


# ---------------------------------------------------------------------------
# status_test.go TestStatus -- assert the LAST condition
# ---------------------------------------------------------------------------
# (job, ps(f,s,a), worker(f,s,a), chief(f,s,a), extra, expected_last)
STATUS = [
    ("c1w", None, (0, 1, 0), (0, 1, 0), None, "Succeeded"),
    ("c1w", None, (0, 0, 0), (0, 0, 1), None, "Running"),
    ("c1w", None, (0, 0, 0), (1, 0, 0), None, "Failed"),
    ("1w", None, (1, 0, 0), None, None, "Failed"),
    ("1w", None, (0, 1, 0), None, None, "Succeeded"),
    ("1w", None, (0, 0, 1), None, None, "Running"),
    ("4w2ps", (0, 0, 2), (0, 2, 2), None, None, "Running"),
    ("4w2ps", (0, 0, 2), (2, 0, 2), None, None, "Failed"),
    ("4w2ps", (0, 0, 2), (2, 2, 0), None, None, "Failed"),
    ("4w2ps", (0, 0, 2), (0, 1, 3), None, "w0", "Succeeded"),
    ("4wall", None, (0, 1, 3), None, "w0", "Running"),
    ("4wall", None, (0, 4, 0), None, None, "Succeeded"),
    ("4wall", None, (1, 1, 2), None, None, "Failed"),
    ("c4w2ps", (0, 0, 2), (4, 0, 0), (0, 0, 1), None, "Failed"),
    ("c4w2ps", (0, 0, 2), (0, 4, 0), (0, 0, 1), None, "Running"),
    ("c4w2ps", (1, 0, 1), (0, 4, 0), (0, 0, 1), None, "Failed"),
    ("c4w2ps", (0, 0, 2), (0, 4, 0), (1, 0, 0), None, "Failed"),
    ("c4w2ps", (0, 0, 2), (4, 0, 0), (0, 1, 0), None, "Succeeded"),
    ("c4w2ps", (0, 0, 2), (4, 0, 0), (1, 0, 0), "restart", "Restarting"),
]


def _status_job(kind):
    return {"c1w": lambda: fx.new_tfjob(1, 0, chief=1), "1w": lambda: fx.new_tfjob(1, 0),
            "4w2ps": lambda: fx.new_tfjob(4, 2),
            "4wall": lambda: fx.new_tfjob_with_success_policy(4, 0, "AllWorkers"),
            "c4w2ps": lambda: fx.new_tfjob(4, 2, chief=1)}[kind]()


def _typed_pods(job, typ, counts, w0=False, restart=False):
    if counts is None:
        return []
    failed, succeeded, active = counts
    out, idx = [], 0
    for _ in range(succeeded):
        p = fx.new_pod(job, typ, idx, "Succeeded")
        if w0 and typ == "worker" and idx == 0:
            fx.set_exit_code(p, 0)
        out.append(p)
        idx += 1
    for _ in range(failed):
        p = fx.new_pod(job, typ, idx, "Failed")
        if restart:
            fx.set_exit_code(p, 130)
        out.append(p)
        idx += 1
    for _ in range(active):
        out.append(fx.new_pod(job, typ, idx, "Running"))
        idx += 1
    return out


@pytest.mark.parametrize("i", range(len(STATUS)))
def test_status_truth_table(i):
    kind, ps, w, chief, extra, expected = STATUS[i]
    job = _status_job(kind)
    if extra == "restart":
        for s in job["spec"]["tfReplicaSpecs"].values():
            s["restartPolicy"] = "ExitCode"
    pods = (_typed_pods(job, "ps", ps, restart=extra == "restart")
            + _typed_pods(job, "worker", w, w0=extra == "w0", restart=extra == "restart")
            + _typed_pods(job, "chief", chief, restart=extra == "restart"))
    res = run(job, pods)
    st = res["status"]
    assert fx.last_condition(st) == expected, st["conditions"]
    # filterOutConditionTest: Running is never True next to Succeeded/Failed
    if fx.check_condition(st, "Succeeded") or fx.check_condition(st, "Failed"):
        assert not fx.check_condition(st, "Running")


# ---------------------------------------------------------------------------
# job_test.go TestDeletePodsAndServices / ActiveDeadline / Backoff / TTL
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("policy,wp,pp,expected", [
    ("All", (0, 4, 0, 0), (0, 2, 0, 0), 6),
    ("Running", (0, 4, 0, 0), (0, 2, 0, 0), 6),
    ("Running", (0, 0, 4, 0), (0, 0, 2, 0), 0),
    ("None", (0, 0, 4, 0), (0, 0, 2, 0), 0),
])
def test_delete_pods_and_services(policy, wp, pp, expected):
    job = fx.new_tfjob_with_clean_policy(0, 4, 2, policy)
    st, _ = core.update_job_conditions({}, "Succeeded", "TFJobSucceeded", "", NOW)
    job["status"] = st
    pods = fx.pods_with_statuses(job, "worker", *wp) + fx.pods_with_statuses(job, "ps", *pp)
    svcs = fx.services(job, "worker", 4) + fx.services(job, "ps", 2)
    res = run(job, pods, svcs)
    assert len(ops(res, "delete_pod")) == expected
    assert len(ops(res, "delete_service")) == expected


def test_cleanpod_running_kills_only_running_ps():
    """E2E cleanpod_policy_tests: policy Running -> only still-running PS go."""
    job = fx.new_tfjob_with_clean_policy(0, 2, 1, "Running")
    job["status"], _ = core.update_job_conditions({}, "Succeeded", "TFJobSucceeded", "", NOW)
    pods = fx.pods_with_statuses(job, "worker", 0, 0, 2, 0) + fx.pods_with_statuses(job, "ps", 0, 1, 0, 0)
    res = run(job, pods, fx.services(job, "worker", 2) + fx.services(job, "ps", 1))
    assert [a["name"] for a in ops(res, "delete_pod")] == ["ps-0"]


@pytest.mark.parametrize("ads,elapsed,expected", [(None, 10, 0), (2, 1, 0), (2, 3, 6)])
def test_active_deadline_seconds(ads, elapsed, expected):
    job = fx.new_tfjob_with_active_deadline(0, 4, 2, ads)
    job["status"] = {"startTime": core.rfc3339(NOW), "conditions": [], "replicaStatuses": {}}
    pods = fx.pods_with_statuses(job, "worker", 0, 4, 0, 0) + fx.pods_with_statuses(job, "ps", 0, 2, 0, 0)
    svcs = fx.services(job, "worker", 4) + fx.services(job, "ps", 2)
    res = run(job, pods, svcs, now=NOW + elapsed)
    assert len(ops(res, "delete_pod")) == expected
    assert len(ops(res, "delete_service")) == expected
    if expected:
        assert fx.last_condition(res["status"]) == "Failed"
    elif ads:
        # deadline fix: the engine asks for a requeue
        assert res["requeue_after"] == pytest.approx(ads - elapsed)


def test_backoff_for_on_failure():
    job = fx.new_tfjob_with_backoff_limit(0, 4, 2, 4)
    pods = (fx.pods_with_statuses(job, "worker", 0, 4, 0, 0, restart_counts=[1, 1, 1, 1])
            + fx.pods_with_statuses(job, "ps", 0, 2, 0, 0))
    res = run(job, pods, fx.services(job, "worker", 4) + fx.services(job, "ps", 2))
    assert len(ops(res, "delete_pod")) == 6
    assert fx.last_condition(res["status"]) == "Failed"
    # below the limit nothing happens
    pods2 = (fx.pods_with_statuses(job, "worker", 0, 4, 0, 0, restart_counts=[1, 1, 1, 0])
             + fx.pods_with_statuses(job, "ps", 0, 2, 0, 0))
    res2 = run(job, pods2, fx.services(job, "worker", 4) + fx.services(job, "ps", 2))
    assert ops(res2, "delete_pod") == []


def test_ttl_seconds_after_finished():
    job = fx.new_tfjob_with_ttl(0, 1, 0, 10)
    st, _ = core.update_job_conditions({}, "Succeeded", "TFJobSucceeded", "", NOW)
    st["completionTime"] = core.rfc3339(NOW)
    job["status"] = st
    early = run(job, now=NOW + 3)
    assert ops(early, "delete_job") == [] and early["requeue_after"] == pytest.approx(7)
    late = run(job, now=NOW + 11)
    assert len(ops(late, "delete_job")) == 1


def test_succeeded_moves_active_to_succeeded():
    job = fx.new_tfjob(2, 1)
    job["status"], _ = core.update_job_conditions({}, "Succeeded", "TFJobSucceeded", "", NOW)
    job["status"]["replicaStatuses"] = {"PS": {"active": 1, "succeeded": 0, "failed": 0}}
    res = run(job)
    assert res["status"]["replicaStatuses"]["PS"] == {"active": 0, "succeeded": 1, "failed": 0}


# ---------------------------------------------------------------------------
# pod_test.go TestExitCode / TestScaleDown / TestScaleUp / TestRestartPolicy
# ---------------------------------------------------------------------------
def test_exit_code_restart():
    job = fx.new_tfjob(1, 0)
    job["spec"]["tfReplicaSpecs"]["Worker"]["restartPolicy"] = "ExitCode"
    pod = fx.set_exit_code(fx.new_pod(job, "worker", 0, "Failed"), 130)
    res = run(job, [pod])
    assert [a["name"] for a in ops(res, "delete_pod")] == ["worker-0"]
    assert fx.last_condition(res["status"]) == "Restarting"
    assert res["metrics"]["restarted"] == 1
    # a permanent error (1) is not restarted and fails the job
    pod1 = fx.set_exit_code(fx.new_pod(job, "worker", 0, "Failed"), 1)
    res1 = run(job, [pod1])
    assert ops(res1, "delete_pod") == []
    assert fx.last_condition(res1["status"]) == "Failed"


@pytest.mark.parametrize("code,retry", [(0, False), (1, False), (127, False), (128, True), (130, True), (137, True)])
def test_retryable_exit_code(code, retry):
    assert core.is_retryable_exit_code(code) == retry


def test_scale_down():
    job = fx.new_tfjob(2, 0)
    job["spec"]["enableDynamicWorker"] = True
    pods = [fx.new_pod(job, "worker", i, "Running") for i in range(3)]
    res = run(job, pods)
    assert [a["name"] for a in ops(res, "delete_pod")] == ["worker-2"]


def test_scale_up():
    job = fx.new_tfjob(3, 0)
    job["spec"]["enableDynamicWorker"] = True
    res = run(job, [fx.new_pod(job, "worker", 0, "Running")])
    names = [a["pod"]["metadata"]["name"] for a in ops(res, "create_pod")]
    assert names == ["test-tfjob-worker-1", "test-tfjob-worker-2"]


@pytest.mark.parametrize("rp,expected", [("Always", "Always"), ("OnFailure", "OnFailure"), ("Never", "Never"),
                                         ("ExitCode", "Never")])
def test_restart_policy(rp, expected):
    job = fx.new_tfjob(1, 0)
    job["spec"]["tfReplicaSpecs"]["Worker"]["restartPolicy"] = rp
    res = run(job)
    assert ops(res, "create_pod")[0]["pod"]["spec"]["restartPolicy"] == expected


def test_is_worker0_completed_success_policy():
    job = fx.new_tfjob(4, 0)
    pods = [fx.set_exit_code(fx.new_pod(job, "worker", 0, "Succeeded"), 0)] + [
        fx.new_pod(job, "worker", i, "Running") for i in range(1, 4)]
    assert fx.last_condition(run(job, pods)["status"]) == "Succeeded"
    job2 = fx.new_tfjob_with_success_policy(4, 0, "AllWorkers")
    assert fx.last_condition(run(job2, pods)["status"]) == "Running"


def test_invalid_spec_fails_job():
    job = fx.new_tfjob(1, 0)
    job["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]["image"] = ""
    res = run(job)
    assert res["actions"] == []
    assert fx.check_condition(res["status"], "Failed", "InvalidTFJobSpec")


def test_deleting_job_is_skipped():
    job = fx.new_tfjob(1, 0)
    job["metadata"]["deletionTimestamp"] = core.rfc3339(NOW)
    res = run(job)
    assert res["skipped"] == "deleting" and res["actions"] == []


# ---------------------------------------------------------------------------
# gang scheduling
# ---------------------------------------------------------------------------
def test_gang_scheduling_podgroup_and_annotations():
    job = fx.new_tfjob(8, 0)
    c = job["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]
    c["resources"] = {"limits": {"amd.com/gpu": 1, "memory": "64Gi"}, "requests": {"cpu": "500m"}}
    job["spec"]["tfReplicaSpecs"]["Worker"]["restartPolicy"] = "OnFailure"
    res = run(job, enable_gang_scheduling=True)
    pg = ops(res, "sync_podgroup")[0]["podgroup"]
    assert pg["kind"] == "PodGroup" and pg["apiVersion"] == "scheduling.volcano.sh/v1beta1"
    assert pg["spec"]["minMember"] == 8
    assert pg["spec"]["minResources"] == {"amd.com/gpu": "8", "memory": "512Gi", "cpu": "4"}
    pod = ops(res, "create_pod")[0]["pod"]
    assert pod["spec"]["schedulerName"] == "volcano"
    assert pod["metadata"]["annotations"]["scheduling.k8s.io/group-name"] == "test-tfjob"
    assert pod["metadata"]["annotations"]["volcano.sh/task-spec"] == "worker"
    job["spec"]["runPolicy"]["schedulingPolicy"] = {"minAvailable": 4, "queue": "q1", "priorityClass": "high"}
    pg2 = core.gen_podgroup(job)
    assert pg2["spec"]["minMember"] == 4 and pg2["spec"]["queue"] == "q1"
    assert pg2["spec"]["priorityClassName"] == "high"
    # terminal job deletes its PodGroup
    job["status"], _ = core.update_job_conditions({}, "Succeeded", "TFJobSucceeded", "", NOW)
    assert len(ops(run(job, enable_gang_scheduling=True), "delete_podgroup")) == 1


def test_gang_keeps_user_scheduler():
    job = fx.new_tfjob(1, 0)
    job["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["schedulerName"] = "my-sched"
    res = run(job, enable_gang_scheduling=True)
    assert ops(res, "create_pod")[0]["pod"]["spec"]["schedulerName"] == "my-sched"
    assert any(e["reason"] == "SettedPodTemplateSchedulerName" for e in res["events"])


# ---------------------------------------------------------------------------
# expectations (pod_test.go TestExpectation)
# ---------------------------------------------------------------------------
def test_expectations():
    e = core.Expectations(ttl_seconds=300)
    key = core.native().expectation_pods_key("default/test-tfjob", "worker")
    assert key == "default/test-tfjob/worker/pods"
    assert e.satisfied(key, NOW)
    e.expect_creations(key, 2, NOW)
    assert not e.satisfied(key, NOW) and e.get(key) == (2, 0)
    e.creation_observed(key)
    assert not e.satisfied(key, NOW)
    e.creation_observed(key)
    assert e.satisfied(key, NOW)
    e.expect_creations(key, 1, NOW)
    assert e.get(key) == (1, 0)
    assert e.satisfied(key, NOW + 301)  # TTL expiry
    e.delete_key(key)
    assert not e.exists(key)


# ---------------------------------------------------------------------------
# ControllerRef claiming (client-go ClaimObject via GetPodsForJob,
# tfjob_controller.go:251-289)
# ---------------------------------------------------------------------------
def test_claim_adopts_orphans_keeps_own_releases_mismatch_ignores_foreign():
    job = fx.new_tfjob(3, 0)
    own = fx.new_pod(job, "worker", 0)
    orphan = fx.new_pod(job, "worker", 1)
    orphan["metadata"].pop("ownerReferences", None)
    foreign = fx.new_pod(job, "worker", 2)
    foreign["metadata"]["ownerReferences"] = [{"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "name": "other",
                                               "uid": "someone-else", "controller": True}]
    drifted = fx.new_pod(job, "worker", 3, name="drifted")
    drifted["metadata"]["labels"]["job-name"] = "not-this-job"
    deleting_orphan = fx.new_pod(job, "worker", 4, name="going")
    deleting_orphan["metadata"].pop("ownerReferences", None)
    deleting_orphan["metadata"]["deletionTimestamp"] = "2024-01-01T00:00:00Z"
    res = core.claim_objects(job, [own, orphan, foreign, drifted, deleting_orphan])
    names = [o["metadata"]["name"] for o in res["claimed"]]
    assert names == [own["metadata"]["name"], orphan["metadata"]["name"]]
    assert res["adopt"] == [orphan["metadata"]["name"]]
    assert res["release"] == ["drifted"]
    adopted = res["claimed"][1]["metadata"]["ownerReferences"][-1]
    assert adopted["uid"] == job["metadata"]["uid"] and adopted["controller"] is True


def test_claim_nothing_adopted_while_job_deleting():
    job = fx.new_tfjob(1, 0)
    job["metadata"]["deletionTimestamp"] = "2024-01-01T00:00:00Z"
    orphan = fx.new_pod(job, "worker", 0)
    orphan["metadata"].pop("ownerReferences", None)
    res = core.claim_objects(job, [orphan])
    assert res["claimed"] == [] and res["adopt"] == []


# ---------------------------------------------------------------------------
# node-local xGMI layout (csrc/core/nodelocal.cc)
# ---------------------------------------------------------------------------
def _gpu_job(workers, chief=0, ps=0, gpus=1, annotation=None):
    job = fx.new_tfjob(workers, ps, chief=chief)
    for rt, s in job["spec"]["tfReplicaSpecs"].items():
        if rt != "PS":
            s["template"]["spec"]["containers"][0]["resources"] = {"limits": {"amd.com/gpu": gpus}}
    if annotation is not None:
        job["metadata"]["annotations"] = {"amd.com/node-local": annotation}
    return job


def test_node_local_pod_spec_and_env():
    """Worker=8 with amd.com/node-local: privileged, one GPU each: every rank
    pod is co-located by a required hostname podAffinity, gets hostIPC, a
    PRIVILEGED training container (a hostPath /dev/dri mount is not in the
    device cgroup, so peers could not be opened), the kubelet's pod-resources
    socket read-only and its own name / namespace from the downward API (the
    trainer binds the GPU the device plugin allocated, not LOCAL_RANK), and
    LOCAL_RANK / LOCAL_WORLD_SIZE of the node."""
    job = _gpu_job(7, chief=1, ps=1, annotation="privileged")
    res = run(job, enable_gang_scheduling=True)
    pods = {p["pod"]["metadata"]["name"]: p["pod"] for p in ops(res, "create_pod")}
    w3 = pods["test-tfjob-worker-3"]
    spec = w3["spec"]
    assert spec["hostIPC"] is True
    # DMA-BUF IPC handles travel between rank processes by PID (nodelocal.cc)
    assert spec["hostPID"] is True
    term = spec["affinity"]["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"][0]
    assert term["topologyKey"] == "kubernetes.io/hostname"
    assert term["labelSelector"]["matchLabels"] == {"group-name": "kubeflow.org", "job-name": "test-tfjob",
                                                    "training.amd.com/node-local": "true"}
    assert w3["metadata"]["labels"]["training.amd.com/node-local"] == "true"
    assert w3["metadata"]["annotations"]["amd.com/gpu-visibility"] == "node"
    # no host device mounts: the privileged container's device cgroup is what grants peer access
    assert [v["hostPath"]["path"] for v in spec["volumes"]] == ["/var/lib/kubelet/pod-resources"]
    c = spec["containers"][0]
    assert c["securityContext"]["privileged"] is True
    assert c["volumeMounts"] == [{"name": "toa-pod-resources", "mountPath": "/var/lib/kubelet/pod-resources",
                                  "readOnly": True}]
    env = {e["name"]: e.get("value") for e in c["env"]}
    downward = {e["name"]: e["valueFrom"]["fieldRef"]["fieldPath"] for e in c["env"] if "valueFrom" in e}
    # NCCL_HOSTID = the node's name: one RCCL hostHash for every co-located rank
    # (each pod has its own hostname), so RCCL takes P2P / SHM, not the socket transport
    assert downward == {"TOA_POD_NAME": "metadata.name", "TOA_POD_NAMESPACE": "metadata.namespace",
                        "NCCL_HOSTID": "spec.nodeName"}
    assert env["RANK"] == "4" and env["LOCAL_RANK"] == "4"  # chief is rank 0
    assert env["LOCAL_WORLD_SIZE"] == "8" and env["WORLD_SIZE"] == "8" and env["TOA_NODE_LOCAL"] == "1"
    assert env["TOA_DEVICE_SOURCE"] == "pod-resources"
    chief = {e["name"]: e.get("value") for e in pods["test-tfjob-chief-0"]["spec"]["containers"][0]["env"]}
    assert chief["LOCAL_RANK"] == "0" and chief["LOCAL_WORLD_SIZE"] == "8"
    ps = pods["test-tfjob-ps-0"]  # outside the RCCL world: unchanged
    assert "hostIPC" not in ps["spec"] and "affinity" not in ps["spec"] and "hostPID" not in ps["spec"]
    assert "securityContext" not in ps["spec"]["containers"][0]
    assert "NCCL_HOSTID" not in {e["name"] for e in ps["spec"]["containers"][0]["env"]}
    assert "LOCAL_RANK" not in {e["name"] for e in ps["spec"]["containers"][0]["env"]}


def _gpu_ps_job(workers=2, ps=1, annotation=None):
    job = _gpu_job(workers, ps=ps, annotation=annotation)
    job["spec"]["tfReplicaSpecs"]["PS"]["template"]["spec"]["containers"][0]["resources"] = {
        "limits": {"amd.com/gpu": 1}}
    return job


def test_gpu_ps_is_in_the_rccl_world():
    """BASELINE config #2 (PS=1 Worker=2, one MI355X each): a PS replica that
    requests a GPU is an RCCL rank the operator owns -- WORLD_SIZE counts it
    and PS p is rank W + p (reference: the PS is a first-class member of the
    cluster spec, tensorflow.go:142-173).  A CPU PS stays outside."""
    job = _gpu_ps_job(2, ps=2)
    envs = {(rt, i): {e["name"]: e["value"] for e in core.gen_env(job, rt, i)}
            for rt, i in (("Worker", 0), ("Worker", 1), ("PS", 0), ("PS", 1))}
    assert {e["WORLD_SIZE"] for e in envs.values()} == {"4"}
    assert [envs[k]["RANK"] for k in sorted(envs)] == ["2", "3", "0", "1"]  # PS 0/1, Worker 0/1
    assert {e["TOA_PS_IN_WORLD"] for e in envs.values()} == {"1"}
    assert {e["TOA_NUM_TRAINERS"] for e in envs.values()} == {"2"}
    assert {e["MASTER_ADDR"] for e in envs.values()} == {"test-tfjob-worker-0.default.svc"}
    cpu = _gpu_job(2, ps=1)  # PS without a GPU request
    w = {e["name"]: e["value"] for e in core.gen_env(cpu, "Worker", 1)}
    p = {e["name"]: e["value"] for e in core.gen_env(cpu, "PS", 0)}
    assert w["WORLD_SIZE"] == "2" and w["TOA_PS_IN_WORLD"] == "0" and "RANK" not in p


def test_gpu_ps_node_local_layout():
    """PS=1 Worker=2 GPU TFJob with amd.com/node-local: all three pods are
    co-located rank pods with identical WORLD_SIZE / LOCAL_WORLD_SIZE, the same
    affinity term, privileged + hostIPC + hostPID and NCCL_HOSTID from the
    node's name, so the PS's pushes and pulls take xGMI, not the socket
    transport; and the trainer's join_ps_world accepts that env as is."""
    from tf_operator_amd.parallel import ps_collective

    job = _gpu_ps_job(2, ps=1, annotation="privileged")
    assert core.node_local(job, {})
    pods = {p["pod"]["metadata"]["name"]: p["pod"] for p in ops(run(job), "create_pod")}
    assert sorted(pods) == ["test-tfjob-ps-0", "test-tfjob-worker-0", "test-tfjob-worker-1"]
    terms, ranks = [], {}
    for name, pod in pods.items():
        spec, c = pod["spec"], pod["spec"]["containers"][0]
        env = {e["name"]: e.get("value") for e in c["env"]}
        downward = {e["name"]: e["valueFrom"]["fieldRef"]["fieldPath"] for e in c["env"] if "valueFrom" in e}
        assert spec["hostIPC"] is True and spec["hostPID"] is True, name
        assert c["securityContext"]["privileged"] is True, name
        assert downward["NCCL_HOSTID"] == "spec.nodeName", name
        assert env["WORLD_SIZE"] == "3" and env["LOCAL_WORLD_SIZE"] == "3", name
        assert env["LOCAL_RANK"] == env["RANK"] and env["TOA_NODE_LOCAL"] == "1", name
        terms.append(spec["affinity"]["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"])
        ranks[name] = int(env["RANK"])
        assert pod["metadata"]["labels"]["training.amd.com/node-local"] == "true"
        # the trainer's check passes on exactly this env, and fails on a tampered one
        saved = dict(os.environ)
        try:
            os.environ.update({k: v for k, v in env.items() if v is not None})
            w, s_, role, idx = ps_collective.ps_world_env()
            assert (w, s_) == (2, 1)
            ps_collective.join_ps_world(w, s_, role, idx)
            os.environ["WORLD_SIZE"] = "2"
            with pytest.raises(RuntimeError, match="inconsistent"):
                ps_collective.join_ps_world(w, s_, role, idx)
        finally:
            os.environ.clear()
            os.environ.update(saved)
    assert all(t == terms[0] for t in terms)
    assert ranks == {"test-tfjob-worker-0": 0, "test-tfjob-worker-1": 1, "test-tfjob-ps-0": 2}
    # 8 GPU ranks fit one node; 7 workers + 2 GPU servers do not
    assert core.node_local(_gpu_ps_job(7, ps=1, annotation="privileged"), {})
    assert not core.node_local(_gpu_ps_job(7, ps=2, annotation="privileged"), {})


def test_node_local_keeps_user_security_context_and_env():
    job = _gpu_job(2, annotation="privileged")
    c0 = job["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]
    c0["securityContext"] = {"runAsUser": 1000}
    c0["env"] = [{"name": "TOA_POD_NAME", "value": "explicit"}]
    pod = ops(run(job), "create_pod")[0]["pod"]
    c = pod["spec"]["containers"][0]
    assert c["securityContext"] == {"runAsUser": 1000, "privileged": True}
    names = [e["name"] for e in c["env"]]
    assert names.count("TOA_POD_NAME") == 1 and names.count("TOA_POD_NAMESPACE") == 1
    assert names.count("NCCL_HOSTID") == 1


def test_node_local_keeps_operator_nccl_hostid():
    """An NCCL_HOSTID the operator's --nccl-env sets wins over the downward-API
    default; without the annotation no rank pod gets NCCL_HOSTID or hostPID."""
    job = _gpu_job(2, annotation="privileged")
    pod = ops(run(job, nccl_env={"NCCL_HOSTID": "rack7-node3"}), "create_pod")[0]["pod"]
    env = [e for e in pod["spec"]["containers"][0]["env"] if e["name"] == "NCCL_HOSTID"]
    assert env == [{"name": "NCCL_HOSTID", "value": "rack7-node3"}]
    plain = ops(run(_gpu_job(2)), "create_pod")[0]["pod"]
    assert "hostPID" not in plain["spec"]
    assert "NCCL_HOSTID" not in {e["name"] for e in plain["spec"]["containers"][0]["env"]}


@pytest.mark.parametrize("workers,gpus,annotation,gang,expected", [
    (2, 1, None, False, False),          # no annotation: the reference layout
    (2, 1, None, True, False),           # gang scheduling alone never selects it (opt-in only)
    (2, 1, "privileged", False, True),   # opt in
    (2, 1, "true", True, True),          # "true" is an alias of "privileged"
    (8, 1, "false", True, False),        # explicit off
    (8, 1, "host-mounts", True, False),  # unknown mode: off
    (9, 1, "privileged", True, False),   # does not fit one 8-GPU node
    (1, 1, "privileged", True, False),   # a single rank has no peers
    (4, 2, "privileged", True, False),   # exactly one GPU per rank pod
])
def test_node_local_selection(workers, gpus, annotation, gang, expected):
    job = _gpu_job(workers, gpus=gpus, annotation=annotation)
    opts = {"enable_gang_scheduling": gang}
    assert core.node_local(job, opts) is expected
    env = {e["name"]: e["value"] for e in core.gen_env(job, "Worker", workers - 1, opts)}
    assert env["LOCAL_WORLD_SIZE"] == (str(workers) if expected else "1")
    assert env["LOCAL_RANK"] == (str(workers - 1) if expected else "0")
    assert ("TOA_DEVICE_SOURCE" in env) is expected
    assert not core.node_local(_gpu_job(4, annotation="privileged"), {"gpus_per_node": 2})


def test_node_local_pytorchjob_env():
    tpl = fx.replica_template()
    tpl["spec"]["containers"][0]["name"] = "pytorch"
    tpl["spec"]["containers"][0]["resources"] = {"limits": {"amd.com/gpu": 1}}
    job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "metadata": {"name": "pt", "namespace": "default", "annotations": {"amd.com/node-local": "privileged"}},
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "template": tpl},
                                            "Worker": {"replicas": 3, "template": tpl}}}}
    env = {e["name"]: e["value"] for e in core.gen_env(job, "Worker", 1)}
    assert env["RANK"] == "2" and env["LOCAL_RANK"] == "2"
    assert env["LOCAL_WORLD_SIZE"] == env["WORLD_SIZE"] == "4"


def test_oneshot_selection_under_operator_env():
    """The operator's node-local env makes GradBucketer's one-shot IPC path
    auto-selectable (no TOA_IPC_ALLREDUCE=1); the classic env does not."""
    from tf_operator_amd.parallel.ddp import ipc_decision

    job = _gpu_job(2, annotation="true")
    env = {e["name"]: e["value"] for e in core.gen_env(job, "Worker", 1)}
    ok, why = ipc_decision("auto", int(env["WORLD_SIZE"]), True, True, True, 1, env["LOCAL_WORLD_SIZE"])
    assert ok, why
    classic = {e["name"]: e["value"] for e in core.gen_env(_gpu_job(2), "Worker", 1)}
    ok, why = ipc_decision("auto", 2, True, True, True, 1, classic["LOCAL_WORLD_SIZE"])
    assert not ok and "span nodes" in why
    assert not ipc_decision("auto", 2, True, True, True, 0, "2")[0]  # nothing small enough
    assert not ipc_decision("0", 2, True, True, True, 1, "2")[0]
    # a gloo group with GPU gradients (replicas possibly sharing one device): never automatic
    ok, why = ipc_decision("auto", 2, True, True, True, 1, "2", backend="gloo")
    assert not ok and "gloo" in why
    assert ipc_decision("1", 2, True, True, True, 1, "2", backend="gloo")[0]  # forced still works
