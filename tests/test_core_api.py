"""API defaulting / validation tests (reference: pkg/apis/*/v1/defaults_test.go,
pkg/apis/*/validation/validation_test.go, pkg/apis/tensorflow/v1/util_test.go)."""
import copy

import pytest

from tf_operator_amd import core
from tf_operator_amd.testing import fixtures as fx


def tpl(container="tensorflow", image="img", ports=None):
    c = {"name": container, "image": image}
    if ports is not None:
        c["ports"] = ports
    return {"spec": {"containers": [c]}}


def test_tf_defaults():
    job = {"kind": "TFJob", "metadata": {"name": "j", "namespace": "ns"},
           "spec": {"tfReplicaSpecs": {"worker": {"template": tpl()}, "ps": {"replicas": 2, "template": tpl()}}}}
    d = core.set_defaults(job)
    s = d["spec"]
    assert s["runPolicy"]["cleanPodPolicy"] == "Running"
    assert s["successPolicy"] == ""
    assert set(s["tfReplicaSpecs"]) == {"Worker", "PS"}  # camel-case normalisation
    w = s["tfReplicaSpecs"]["Worker"]
    assert w["replicas"] == 1 and w["restartPolicy"] == "Never"
    assert w["template"]["spec"]["containers"][0]["ports"] == [{"name": "tfjob-port", "containerPort": 2222}]
    assert s["tfReplicaSpecs"]["PS"]["replicas"] == 2
    # existing port is kept, not duplicated
    job2 = copy.deepcopy(job)
    job2["spec"]["tfReplicaSpecs"]["worker"]["template"] = tpl(ports=[{"name": "tfjob-port", "containerPort": 1}])
    p = core.set_defaults(job2)["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]["ports"]
    assert p == [{"name": "tfjob-port", "containerPort": 1}]


@pytest.mark.parametrize("key,canon", [("WORKER", "Worker"), ("Ps", "PS"), ("chief", "Chief"), ("MASTER", "Master"),
                                       ("evaluator", "Evaluator")])
def test_tf_camel_case(key, canon):
    job = {"kind": "TFJob", "metadata": {"name": "j"}, "spec": {"tfReplicaSpecs": {key: {"template": tpl()}}}}
    assert list(core.set_defaults(job)["spec"]["tfReplicaSpecs"]) == [canon]


def test_port_added_to_default_container_or_first():
    job = {"kind": "TFJob", "metadata": {"name": "j"},
           "spec": {"tfReplicaSpecs": {"Worker": {"template": {"spec": {"containers": [
               {"name": "sidecar", "image": "a"}, {"name": "tensorflow", "image": "b"}]}}}}}}
    cs = core.set_defaults(job)["spec"]["tfReplicaSpecs"]["Worker"]["template"]["spec"]["containers"]
    assert "ports" not in cs[0] and cs[1]["ports"][0]["name"] == "tfjob-port"


def test_legacy_flat_runpolicy_fields():
    """SDK/YAML examples put cleanPodPolicy at spec root."""
    job = {"kind": "TFJob", "metadata": {"name": "j"},
           "spec": {"cleanPodPolicy": "None", "backoffLimit": 3, "tfReplicaSpecs": {"Worker": {"template": tpl()}}}}
    s = core.set_defaults(job)["spec"]
    assert s["runPolicy"]["cleanPodPolicy"] == "None" and s["runPolicy"]["backoffLimit"] == 3
    assert "cleanPodPolicy" not in s


@pytest.mark.parametrize("kind,field,container,port_name,port,restart,clean", [
    ("PyTorchJob", "pytorchReplicaSpecs", "pytorch", "pytorchjob-port", 23456, "OnFailure", "None"),
    ("MXJob", "mxReplicaSpecs", "mxnet", "mxjob-port", 9091, "Never", "All"),
    ("XGBoostJob", "xgbReplicaSpecs", "xgboost", "xgboostjob-port", 9999, "Never", "All"),
])
def test_other_kind_defaults(kind, field, container, port_name, port, restart, clean):
    first = "Scheduler" if kind == "MXJob" else "Master"
    job = {"kind": kind, "metadata": {"name": "j"},
           "spec": {field: {first.lower(): {"template": tpl(container)}, "worker": {"template": tpl(container)}}}}
    d = core.set_defaults(job)
    s = d["spec"]
    assert s["runPolicy"]["cleanPodPolicy"] == clean
    specs = s[field]
    assert set(specs) == {first, "Worker"}
    for rt, sp in specs.items():
        assert sp["restartPolicy"] == restart and sp["replicas"] == 1
        ports = sp["template"]["spec"]["containers"][0].get("ports")
        if kind == "PyTorchJob" and rt == "Worker":
            assert ports is None  # port only on Master (pytorch/v1/defaults.go:98-105)
        else:
            assert ports == [{"name": port_name, "containerPort": port}]


def test_kind_info_table():
    assert core.supported_kinds() == ["TFJob", "PyTorchJob", "MXJob", "XGBoostJob"]
    ki = core.kind_info("TFJob")
    assert ki["plural"] == "tfjobs" and ki["container"] == "tensorflow" and ki["port"] == 2222
    assert core.kind_info("pytorchjobs")["kind"] == "PyTorchJob"


# ---------------------------------------------------------------------------
# validation
# ---------------------------------------------------------------------------
def tfjob(specs):
    return {"kind": "TFJob", "metadata": {"name": "j"}, "spec": {"tfReplicaSpecs": specs}}


@pytest.mark.parametrize("specs,msg", [
    (None, "TFJobSpec is not valid"),
    ({"Worker": {"template": {"spec": {"containers": []}}}}, "containers definition expected in Worker"),
    ({"Worker": {"template": tpl(image="")}}, "Image is undefined in the container of Worker"),
    ({"Worker": {"template": tpl(container="foo")}}, "There is no container named tensorflow in Worker"),
    ({"Chief": {"template": tpl()}, "Master": {"template": tpl()}}, "more than 1 chief/master found"),
])
def test_tf_validation_errors(specs, msg):
    assert msg in core.validate(tfjob(specs))


def test_tf_validation_ok():
    assert core.validate(fx.new_tfjob(2, 1, chief=1)) == ""


@pytest.mark.parametrize("kind,field,c", [("PyTorchJob", "pytorchReplicaSpecs", "pytorch"),
                                          ("XGBoostJob", "xgbReplicaSpecs", "xgboost")])
def test_master_worker_validation(kind, field, c):
    def job(specs):
        return {"kind": kind, "metadata": {"name": "j"}, "spec": {field: specs}}

    assert core.validate(job({"Master": {"replicas": 1, "template": tpl(c)},
                              "Worker": {"replicas": 3, "template": tpl(c)}})) == ""
    assert "Master ReplicaSpec must be present" in core.validate(job({"Worker": {"template": tpl(c)}}))
    assert "only 1 master" in core.validate(job({"Master": {"replicas": 2, "template": tpl(c)}}))
    assert "must be one of" in core.validate(job({"Master": {"template": tpl(c)}, "PS": {"template": tpl(c)}}))
    assert "no container named " + c in core.validate(job({"Master": {"template": tpl("x")}}))
    assert "Image is undefined" in core.validate(job({"Master": {"template": tpl(c, image="")}}))


def test_mx_validation():
    def job(specs):
        return {"kind": "MXJob", "metadata": {"name": "j"}, "spec": {"mxReplicaSpecs": specs}}

    ok = job({"Scheduler": {"template": tpl("mxnet")}, "Server": {"template": tpl("mxnet")},
              "Worker": {"template": tpl("mxnet")}})
    assert core.validate(ok) == ""
    assert core.validate(job({"Worker": {"template": tpl("foo")}})) == "MXJobSpec is not valid"


# ---------------------------------------------------------------------------
# env generators for the other kinds
# ---------------------------------------------------------------------------
def test_pytorch_env():
    job = {"kind": "PyTorchJob", "metadata": {"name": "pt", "namespace": "ns"},
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "template": tpl("pytorch")},
                                            "Worker": {"replicas": 3, "template": tpl("pytorch")}}}}
    m = {e["name"]: e["value"] for e in core.gen_env(job, "Master", 0)}
    assert m["MASTER_ADDR"] == "localhost" and m["RANK"] == "0" and m["WORLD_SIZE"] == "4"
    assert m["MASTER_PORT"] == "23456" and m["PYTHONUNBUFFERED"] == "0"
    w = {e["name"]: e["value"] for e in core.gen_env(job, "Worker", 2)}
    assert w["MASTER_ADDR"] == "pt-master-0" and w["RANK"] == "3"
    names = [e["name"] for e in core.gen_env(job, "Worker", 0, {"inject_rocm_env": False})]
    assert names == ["MASTER_PORT", "MASTER_ADDR", "WORLD_SIZE", "RANK", "PYTHONUNBUFFERED"]


def test_xgboost_env():
    job = {"kind": "XGBoostJob", "metadata": {"name": "xg"},
           "spec": {"xgbReplicaSpecs": {"Master": {"replicas": 1, "template": tpl("xgboost")},
                                        "Worker": {"replicas": 2, "template": tpl("xgboost")}}}}
    w = {e["name"]: e["value"] for e in core.gen_env(job, "Worker", 1)}
    assert w["RANK"] == "2" and w["WORLD_SIZE"] == "3" and w["MASTER_ADDR"] == "xg-master-0"
    assert w["WORKER_PORT"] == "9999" and w["WORKER_ADDRS"] == "xg-worker-0,xg-worker-1"


def test_mxnet_env():
    job = {"kind": "MXJob", "metadata": {"name": "mx"},
           "spec": {"mxReplicaSpecs": {
               "Scheduler": {"replicas": 1, "template": tpl("mxnet")},
               "Server": {"replicas": 1, "template": tpl("mxnet")},
               "Worker": {"replicas": 2, "template": {"metadata": {"annotations": {"tuner-server-key": "k"}},
                                                       "spec": {"containers": [{"name": "mxnet", "image": "i"}]}}}}}}
    e = {x["name"]: x["value"] for x in core.gen_env(job, "Worker", 1)}
    assert e["MX_CONFIG"] == ('{"cluster":{"scheduler":[{"url":"mx-scheduler-0","port":9091}],"server":[{"url":'
                              '"mx-server-0","port":9091}],"worker":[{"url":"mx-worker-0","port":9091},{"url":'
                              '"mx-worker-1","port":9091}]},"labels":{"scheduler":"","server":"","worker":"k"},'
                              '"task":{"type":"worker","index":1}}')
    assert e["DMLC_PS_ROOT_URI"] == "mx-scheduler-0" and e["DMLC_PS_ROOT_PORT"] == "9091"
    assert e["DMLC_NUM_SERVER"] == "1" and e["DMLC_NUM_WORKER"] == "2" and e["DMLC_ROLE"] == "worker"
    assert e["DMLC_USE_KUBERNETES"] == "1" and e["DMLC_WORKER_ID"] == "1"


@pytest.mark.parametrize("kind,field,c,first", [("PyTorchJob", "pytorchReplicaSpecs", "pytorch", "Master"),
                                                ("XGBoostJob", "xgbReplicaSpecs", "xgboost", "Master"),
                                                ("MXJob", "mxReplicaSpecs", "mxnet", "Scheduler")])
def test_other_kind_status(kind, field, c, first):
    job = {"kind": kind, "metadata": {"name": "j", "namespace": "default", "uid": "u"},
           "spec": {field: {first: {"replicas": 1, "template": tpl(c)}, "Worker": {"replicas": 2,
                                                                                    "template": tpl(c)}}}}
    res = core.reconcile(job, [], [], now=1e9)
    assert len([a for a in res["actions"] if a["op"] == "create_pod"]) == 3
    pods = [fx.new_pod(job, first.lower(), 0, "Running"), fx.new_pod(job, "worker", 0, "Running"),
            fx.new_pod(job, "worker", 1, "Running")]
    assert fx.last_condition(core.reconcile(job, pods, [], now=1e9)["status"]) == "Running"
    pods[0]["status"]["phase"] = "Succeeded"
    if kind == "MXJob":
        for p in pods:
            p["status"]["phase"] = "Succeeded"
    st = core.reconcile(job, pods, [], now=1e9)["status"]
    assert fx.last_condition(st) == "Succeeded" and st.get("completionTime")
    pods[0]["status"]["phase"] = "Running"
    pods[1]["status"]["phase"] = "Failed"
    st = core.reconcile(job, pods, [], now=1e9)["status"]
    assert fx.last_condition(st) == "Failed"


def test_conditions_semantics():
    st, ch = core.update_job_conditions({}, "Created", "TFJobCreated", "m", 1.0)
    assert ch and [c["type"] for c in st["conditions"]] == ["Created"]
    st, ch = core.update_job_conditions(st, "Running", "TFJobRunning", "m", 2.0)
    st, ch = core.update_job_conditions(st, "Running", "TFJobRunning", "m", 3.0)
    assert not ch  # same type/status/reason -> no-op
    st, _ = core.update_job_conditions(st, "Restarting", "TFJobRestarting", "m", 4.0)
    assert [c["type"] for c in st["conditions"]] == ["Created", "Restarting"]  # Running removed
    st, _ = core.update_job_conditions(st, "Running", "TFJobRunning", "m", 5.0)
    assert [c["type"] for c in st["conditions"]] == ["Created", "Running"]
    st, _ = core.update_job_conditions(st, "Failed", "TFJobFailed", "m", 6.0)
    run = [c for c in st["conditions"] if c["type"] == "Running"][0]
    assert run["status"] == "False" and st["conditions"][-1]["type"] == "Failed"
    st2, ch = core.update_job_conditions(st, "Running", "TFJobRunning", "m", 7.0)
    assert not ch and st2 == st  # a failed job is frozen


def test_on_job_created():
    j = core.on_job_created(fx.new_tfjob(1, 0), now=1e9)
    c = j["status"]["conditions"][-1]
    assert c["type"] == "Created" and c["reason"] == "TFJobCreated"
    assert c["message"] == "TFJob default/test-tfjob is created."


def test_rfc3339_roundtrip():
    assert core.rfc3339(0) == "1970-01-01T00:00:00Z"
    assert core.parse_rfc3339("2024-05-01T10:00:00Z") == core.parse_rfc3339("2024-05-01T12:00:00+02:00")


def test_store_and_workqueue():
    s = core.Store()
    a = fx.new_pod(fx.new_tfjob(1, 0), "worker", 0, "Running")
    a["metadata"]["resourceVersion"] = "1"
    assert s.upsert(a)
    assert not s.upsert(a)  # same resourceVersion -> resync, not a change
    assert len(s.list("default", {"replica-type": "worker"})) == 1
    assert s.list("default", {"replica-type": "ps"}) == []
    assert s.get("default/worker-0")["status"]["phase"] == "Running"
    assert s.remove("default/worker-0") and len(s) == 0
    q = core.WorkQueue(0.001, 0.1)
    q.add("a")
    q.add("a")  # de-duplicated
    assert len(q) == 1
    assert q.get(0.1) == "a"
    q.add("a")  # while processing -> re-queued on done()
    assert len(q) == 0
    q.done("a")
    assert q.get(0.1) == "a"
    q.done("a")
    q.add_rate_limited("b")
    q.add_rate_limited("b")
    assert q.num_requeues("b") == 2
    assert q.get(0.5) == "b"
    q.forget("b")
    assert q.num_requeues("b") == 0
    q.shutdown()
    assert q.get(0.01) is None
