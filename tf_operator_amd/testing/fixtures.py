"""Job / pod / service fixture builders (reference: pkg/common/util/v1/testutil/
{tfjob,pod,service,util,const}.go).  Used by the ported controller tests and
the E2E suites."""
from __future__ import annotations

import copy
import uuid

TEST_TFJOB_NAME = "test-tfjob"
TEST_IMAGE = "test-image-for-kubeflow-tf-operator:latest"
LABEL_GROUP_NAME = "group-name"
JOB_NAME_LABEL = "job-name"
REPLICA_TYPE_LABEL = "replica-type"
REPLICA_INDEX_LABEL = "replica-index"
LABEL_WORKER, LABEL_PS, LABEL_CHIEF, LABEL_EVALUATOR = "worker", "ps", "chief", "evaluator"


def replica_template(container="tensorflow", port_name="tfjob-port", port=2222, image=TEST_IMAGE):
    return {"spec": {"containers": [{"name": container, "image": image, "args": ["Fake", "Fake"],
                                     "ports": [{"name": port_name, "containerPort": port}]}]}}


def new_tfjob(worker=0, ps=0, chief=0, master=0, evaluator=0, name=TEST_TFJOB_NAME, namespace="default"):
    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
           "metadata": {"name": name, "namespace": namespace, "uid": str(uuid.uuid5(uuid.NAMESPACE_DNS, name + namespace))},
           "spec": {"runPolicy": {"cleanPodPolicy": "Running"}, "successPolicy": "", "tfReplicaSpecs": {}}}
    specs = job["spec"]["tfReplicaSpecs"]
    for rt, n in (("Worker", worker), ("PS", ps), ("Chief", chief), ("Master", master), ("Evaluator", evaluator)):
        if n > 0:
            specs[rt] = {"replicas": n, "template": replica_template()}
    return job


def new_tfjob_with_clean_policy(chief, worker, ps, policy):
    j = new_tfjob(worker, ps, chief=chief)
    j["spec"]["runPolicy"]["cleanPodPolicy"] = policy
    return j


def new_tfjob_with_active_deadline(chief, worker, ps, ads):
    j = new_tfjob(worker, ps, chief=chief)
    if ads is not None:
        j["spec"]["runPolicy"]["activeDeadlineSeconds"] = ads
    return j


def new_tfjob_with_backoff_limit(chief, worker, ps, limit):
    j = new_tfjob(worker, ps, chief=chief)
    j["spec"]["runPolicy"]["backoffLimit"] = limit
    for s in j["spec"]["tfReplicaSpecs"].values():
        s["restartPolicy"] = "OnFailure"
    return j


def new_tfjob_with_ttl(chief, worker, ps, ttl):
    j = new_tfjob(worker, ps, chief=chief)
    if ttl is not None:
        j["spec"]["runPolicy"]["ttlSecondsAfterFinished"] = ttl
    return j


def new_tfjob_with_success_policy(worker, ps, policy):
    j = new_tfjob(worker, ps)
    j["spec"]["successPolicy"] = policy
    return j


def new_tfjob_with_chief(worker, ps):
    return new_tfjob(worker, ps, chief=1)


def new_tfjob_with_evaluator(worker, ps, evaluator):
    return new_tfjob(worker, ps, evaluator=evaluator)


def gen_labels(job_name):
    n = job_name.replace("/", "-")
    return {LABEL_GROUP_NAME: "kubeflow.org", JOB_NAME_LABEL: n, "tf-job-name": n}


def owner_ref(job):
    return {"apiVersion": "kubeflow.org/v1", "kind": job.get("kind", "TFJob"), "name": job["metadata"]["name"],
            "uid": job["metadata"].get("uid", ""), "controller": True, "blockOwnerDeletion": True}


def new_pod(job, typ, index, phase=None, name=None):
    md = job["metadata"]
    labels = gen_labels(md["name"])
    labels[REPLICA_TYPE_LABEL] = typ
    labels[REPLICA_INDEX_LABEL] = str(index)
    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"name": name or f"{typ}-{index}", "namespace": md.get("namespace", "default"),
                        "labels": labels, "ownerReferences": [owner_ref(job)]},
           "spec": {}, "status": {}}
    if phase:
        pod["status"]["phase"] = phase
    return pod


def pods_with_statuses(job, typ, pending=0, active=0, succeeded=0, failed=0, restart_counts=None):
    """SetPodsStatuses: indices assigned pending, then active, succeeded, failed."""
    out, idx = [], 0
    for phase, n in (("Pending", pending), ("Running", active), ("Succeeded", succeeded), ("Failed", failed)):
        for i in range(n):
            p = new_pod(job, typ, idx, phase)
            if phase == "Running" and restart_counts is not None:
                p["status"]["containerStatuses"] = [{"name": "tensorflow", "restartCount": restart_counts[i]}]
            out.append(p)
            idx += 1
    return out


def set_exit_code(pod, code, container="tensorflow"):
    pod.setdefault("status", {})["containerStatuses"] = [
        {"name": container, "state": {"terminated": {"exitCode": code}}}]
    return pod


def new_service(job, typ, index):
    md = job["metadata"]
    labels = gen_labels(md["name"])
    labels[REPLICA_TYPE_LABEL] = typ
    labels[REPLICA_INDEX_LABEL] = str(index)
    return {"apiVersion": "v1", "kind": "Service",
            "metadata": {"name": f"{typ}-{index}", "namespace": md.get("namespace", "default"), "labels": labels,
                         "ownerReferences": [owner_ref(job)]},
            "spec": {"clusterIP": "None"}}


def services(job, typ, n):
    return [new_service(job, typ, i) for i in range(n)]


def check_condition(job_or_status, ctype, reason=None):
    st = job_or_status.get("status", job_or_status)
    for c in st.get("conditions", []):
        if c["type"] == ctype and c.get("status") == "True" and (reason is None or c.get("reason") == reason):
            return True
    return False


def last_condition(job_or_status):
    st = job_or_status.get("status", job_or_status)
    conds = st.get("conditions") or []
    return conds[-1]["type"] if conds else None


def with_status(job, status):
    j = copy.deepcopy(job)
    j["status"] = status
    return j


def get_condition(job_or_status, ctype):
    st = job_or_status.get("status", job_or_status)
    for c in st.get("conditions", []):
        if c["type"] == ctype:
            return c
    return None


def new_pytorchjob(master=1, worker=0, name="test-pytorchjob", namespace="default"):
    """pkg/controller.v1/pytorch/pytorchjob_controller_suite_test.go style job."""
    job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "metadata": {"name": name, "namespace": namespace,
                        "uid": str(uuid.uuid5(uuid.NAMESPACE_DNS, name + namespace))},
           "spec": {"runPolicy": {}, "pytorchReplicaSpecs": {}}}
    specs = job["spec"]["pytorchReplicaSpecs"]
    for rt, n in (("Master", master), ("Worker", worker)):
        if n > 0:
            specs[rt] = {"replicas": n, "template": replica_template("pytorch", "pytorchjob-port", 23456)}
    return job
