"""Deploy artefacts and the example job YAMLs:
generated CRDs match the schema module, the SDK models cover the schema,
kustomize trees are complete, every example job validates, and the CPU-sized
examples (dist-mnist PS, MXJob ps-lite, XGBoostJob Rabit) run to Succeeded on
the local cluster from their YAML."""
import copy
import dataclasses
import glob
import os
import sys

import pytest
import yaml

from tf_operator_amd import core
from tf_operator_amd.api import schema
from tf_operator_amd.sdk import models
from tf_operator_amd.testing.cluster import LocalCluster

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAN = os.path.join(ROOT, "manifests")


def _camel(s):
    p = s.split("_")
    return p[0] + "".join(x.title() for x in p[1:])


def test_generated_crds_are_current():
    for kind, (plural, *_r) in schema.KINDS.items():
        path = os.path.join(MAN, "base", f"kubeflow.org_{plural}.yaml")
        body = open(path).read().split("\n", 1)[1]
        assert body == schema.render(kind), f"{path} is stale: run python -m tf_operator_amd.api.schema"
        crd = yaml.safe_load(body)
        assert crd["spec"]["names"]["kind"] == kind
        v = crd["spec"]["versions"][0]
        assert v["subresources"] == {"status": {}}
        spec = v["schema"]["openAPIV3Schema"]["properties"]["spec"]
        assert schema.KINDS[kind][2] in spec["properties"]
        assert "elasticPolicy" in spec["properties"] and "runPolicy" in spec["properties"]


def test_sdk_models_cover_schema():
    sp = schema.spec_schema("TFJob")["properties"]
    for f in dataclasses.fields(models.V1TFJobSpec):
        if f.metadata.get("skip"):
            continue
        assert _camel(f.name) in sp, f.name
    rp = schema.RUN_POLICY["properties"]
    for f in dataclasses.fields(models.V1RunPolicy):
        assert _camel(f.name) in rp, f.name
    ep = schema.ELASTIC_POLICY["properties"]
    for f in dataclasses.fields(models.V1ElasticPolicy):
        assert _camel(f.name) in ep, f.name
    st = schema.JOB_STATUS["properties"]
    for f in dataclasses.fields(models.V1JobStatus):
        assert _camel(f.name) in st, f.name
    es = schema.ELASTIC_STATUS["properties"]
    for f in dataclasses.fields(models.V1ElasticStatus):
        assert _camel(f.name) in es, f.name


@pytest.mark.parametrize("tree", ["base", "overlays/standalone", "overlays/kubeflow"])
def test_kustomize_resources_exist(tree):
    k = yaml.safe_load(open(os.path.join(MAN, tree, "kustomization.yaml")))
    for r in k["resources"]:
        p = os.path.normpath(os.path.join(MAN, tree, r))
        assert os.path.exists(p), p
        if p.endswith(".yaml"):
            for doc in yaml.safe_load_all(open(p)):
                assert doc is None or "kind" in doc


def test_rbac_covers_what_the_operator_touches():
    rules = yaml.safe_load(open(os.path.join(MAN, "base", "cluster-role.yaml")))["rules"]
    granted = {(g, r) for rule in rules for g in rule["apiGroups"] for r in rule["resources"]}
    for need in [("kubeflow.org", "tfjobs/status"), ("", "pods"), ("", "services"), ("", "events"),
                 ("", "nodes"), ("scheduling.volcano.sh", "podgroups"), ("coordination.k8s.io", "leases")]:
        assert need in granted, need


EXAMPLES = sorted(glob.glob(os.path.join(MAN, "examples", "*.yaml")))


@pytest.mark.parametrize("path", EXAMPLES, ids=[os.path.basename(p) for p in EXAMPLES])
def test_example_jobs_validate(path):
    job = yaml.safe_load(open(path))
    assert core.validate(job) == "", core.validate(job)
    d = core.set_defaults(job)
    field = core.kind_info(job["kind"])["specs_field"]
    for rt, spec in d["spec"][field].items():
        assert spec["replicas"] >= 1 and spec["restartPolicy"]
    res = core.reconcile(core.on_job_created(job), [], [], options={})
    assert [a for a in res["actions"] if a["op"] == "create_pod"]


def _localize(job, overrides):
    job = copy.deepcopy(job)
    field = core.kind_info(job["kind"])["specs_field"]
    for rt, spec in job["spec"][field].items():
        for c in spec["template"]["spec"]["containers"]:
            c["command"] = [sys.executable] + c["command"][1:]
            c["args"] = overrides.get(rt, overrides.get("*", c.get("args", [])))
            c.setdefault("env", []).append({"name": "OMP_NUM_THREADS", "value": "1"})
            c.get("resources", {}).get("limits", {}).pop("amd.com/gpu", None)
    return job


def _conds(job):
    return [c["type"] for c in (job.get("status") or {}).get("conditions") or [] if c.get("status") == "True"]


@pytest.fixture(scope="module")
def cluster():
    with LocalCluster(gpus=0) as c:
        yield c


@pytest.mark.parametrize("name,overrides,kind", [
    ("tfjob-dist-mnist.yaml", {"*": ["--train_steps", "200", "--log_every", "100"]}, "TFJob"),
    ("mxjob-dist.yaml", {"*": ["--steps", "60"]}, "MXJob"),
    ("xgboostjob-dist.yaml", {"*": ["--rounds", "10", "--rows", "5000"]}, "XGBoostJob"),
])
def test_example_runs_from_yaml(cluster, name, overrides, kind):
    job = _localize(yaml.safe_load(open(os.path.join(MAN, "examples", name))), overrides)
    client = cluster.sdk(kind)
    client.create(job)
    done = client.wait_for_job(job["metadata"]["name"], polling_interval=0.2, timeout_seconds=180)
    logs = {}
    for (ns, pod) in list(cluster.kubelet.start_times):
        if pod.startswith(job["metadata"]["name"] + "-"):
            p = cluster.kubelet.log_path(ns, pod)
            logs[pod] = open(p).read()[-1500:] if p else ""
    assert "Succeeded" in _conds(done), (_conds(done), logs)
    if kind == "XGBoostJob":
        assert "round 10 logloss" in logs[job["metadata"]["name"] + "-master-0"]
    if kind == "MXJob":
        assert "accuracy" in logs[job["metadata"]["name"] + "-worker-0"]


def test_pod_template_schema_is_structural_and_admits_examples():
    """The replica pod template is validated (not preserve-unknown at the
    top): every example job passes; the API server refuses malformed
    containers with the API server's field paths."""
    from tf_operator_amd.api.validate import job_errors

    tpl = schema.spec_schema("TFJob")["properties"]["tfReplicaSpecs"]["additionalProperties"]["properties"]["template"]
    assert "x-kubernetes-preserve-unknown-fields" not in tpl
    assert tpl["properties"]["spec"]["required"] == ["containers"]
    n = 0
    for path in sorted(glob.glob(os.path.join(MAN, "examples", "*.yaml"))):
        for doc in yaml.safe_load_all(open(path)):
            if doc and doc.get("kind") in schema.KINDS:
                assert job_errors(doc, doc["kind"]) == [], path
                n += 1
    assert n >= 3


@pytest.mark.parametrize("mutate,field", [
    (lambda c: c.pop("name"), "spec.tfReplicaSpecs.Worker.template.spec.containers[0].name: Required value"),
    (lambda c: c.update(command="python train.py"),
     "spec.tfReplicaSpecs.Worker.template.spec.containers[0].command: Invalid value"),
    (lambda c: c.update(ports=[{"name": "tfjob-port"}]),
     "spec.tfReplicaSpecs.Worker.template.spec.containers[0].ports[0].containerPort: Required value"),
    (lambda c: c.update(resources={"limits": {"amd.com/gpu": "one"}}),
     "spec.tfReplicaSpecs.Worker.template.spec.containers[0].resources.limits.amd.com/gpu: Invalid value"),
    (lambda c: c.update(env=[{"value": "1"}]),
     "spec.tfReplicaSpecs.Worker.template.spec.containers[0].env[0].name: Required value"),
    (lambda c: c.update(imagePullPolicy="Sometimes"),
     "spec.tfReplicaSpecs.Worker.template.spec.containers[0].imagePullPolicy: Unsupported value"),
])
def test_api_server_rejects_malformed_container(mutate, field):
    from tf_operator_amd.sdk import container, pod_template

    c = container(image="toa/trainer", command=["python", "-c", "pass"], gpus=1)
    mutate(c)
    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": "bad", "namespace": "default"},
           "spec": {"tfReplicaSpecs": {"Worker": {"replicas": 1, "template": pod_template(c)}}}}
    with LocalCluster(gpus=0) as cl:
        with pytest.raises(Exception) as ei:
            cl.client.create(job)
        assert field in str(ei.value), str(ei.value)
        assert 'TFJob.kubeflow.org \\"bad\\" is invalid' in str(ei.value) and "(422)" in str(ei.value)
        assert cl.api.get("kubeflow.org/tfjobs", "default", "bad") is None


def test_api_server_rejects_empty_container_list():
    from tf_operator_amd.api.validate import job_errors

    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": "x"},
           "spec": {"tfReplicaSpecs": {"Worker": {"replicas": 1, "template": {"spec": {"containers": []}}}}}}
    errs = job_errors(job, "TFJob")
    assert errs == ["spec.tfReplicaSpecs.Worker.template.spec.containers: Invalid value: 0: "
                    "spec.tfReplicaSpecs.Worker.template.spec.containers in body should have at least 1 items"]
