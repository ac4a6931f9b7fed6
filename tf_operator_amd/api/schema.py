"""One schema module for the four job CRDs.

The reference generates ~6,900-line CRDs per kind with controller-gen from
Go types (manifests/base/kubeflow.org_tfjobs.yaml) plus deepcopy/OpenAPI/
swagger code.  Here the job-level schema is written once, in Python; the
CRD YAML under ``manifests/base`` is generated from it and a test checks
that the SDK dataclasses (``tf_operator_amd.sdk.models``) and the generated
files stay in sync with it.  The embedded pod template is a STRUCTURAL
schema of the PodTemplateSpec fields a training job uses (containers,
their command / env / ports / resources / volume mounts, volumes,
scheduling fields), so the API server rejects a malformed replica at
create time -- like the reference's controller-gen schema
(manifests/base/kubeflow.org_tfjobs.yaml:108-~6800) -- while nested
objects outside that set (affinity, probes, security contexts, volume
sources) keep ``x-kubernetes-preserve-unknown-fields``, which keeps each
CRD under a thousand lines.  ``api/validate.py`` applies the same schema
in the in-process API server.

    python -m tf_operator_amd.api.schema --out manifests/base
"""
from __future__ import annotations

import argparse
import copy
import os

GROUP = "kubeflow.org"
VERSION = "v1"

# kind -> (plural, singular, specs field, replica types, default restart, extra spec fields)
KINDS = {
    "TFJob": ("tfjobs", "tfjob", "tfReplicaSpecs", ["Chief", "Master", "PS", "Worker", "Evaluator"], "Never",
              {"successPolicy": {"type": "string", "enum": ["", "AllWorkers"],
                                 "description": 'Criteria to mark the job succeeded: "" (chief or worker-0 '
                                                'done) or AllWorkers.'},
               "enableDynamicWorker": {"type": "boolean",
                                       "description": "Workers may be added / removed while the job runs "
                                                      "(sparse TF_CONFIG)."}}),
    "PyTorchJob": ("pytorchjobs", "pytorchjob", "pytorchReplicaSpecs", ["Master", "Worker"], "OnFailure", {}),
    "MXJob": ("mxjobs", "mxjob", "mxReplicaSpecs", ["Scheduler", "Server", "Worker", "Tuner", "TunerTracker",
                                                    "TunerServer"], "Never",
              {"jobMode": {"type": "string", "enum": ["MXTrain", "MXTune"],
                           "description": "MXTrain (distributed training) or MXTune (auto-tuning)."}}),
    "XGBoostJob": ("xgboostjobs", "xgboostjob", "xgbReplicaSpecs", ["Master", "Worker"], "Never", {}),
}

QUANTITY = {"anyOf": [{"type": "integer"}, {"type": "string"}], "x-kubernetes-int-or-string": True,
            "pattern": r"^(\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))(([KMGTPE]i)|[numkMGTPE]|"
                       r"([eE](\+|-)?(([0-9]+(\.[0-9]*)?)|(\.[0-9]+))))?$"}


def _int(desc, fmt="int32", minimum=None):
    s = {"type": "integer", "format": fmt, "description": desc}
    if minimum is not None:
        s["minimum"] = minimum
    return s


SCHEDULING_POLICY = {
    "type": "object",
    "description": "Gang-scheduling policy (Volcano PodGroup).",
    "properties": {
        "minAvailable": _int("Minimum members the PodGroup needs to start (default: all replicas)."),
        "queue": {"type": "string", "description": "Scheduler queue."},
        "minResources": {"type": "object", "additionalProperties": QUANTITY,
                         "description": "Resources the PodGroup reserves (default: sum of replica requests, "
                                        "including amd.com/gpu)."},
        "priorityClass": {"type": "string", "description": "PriorityClass of the PodGroup."},
    },
}

RUN_POLICY = {
    "type": "object",
    "description": "Runtime policies of the distributed job: cleanup, TTL, deadlines, retries, gang scheduling.",
    "properties": {
        "cleanPodPolicy": {"type": "string", "enum": ["All", "Running", "None"],
                           "description": "Pods to delete when the job finishes (default: TFJob Running, "
                                          "PyTorchJob None, MXJob / XGBoostJob All)."},
        "ttlSecondsAfterFinished": _int("Delete the job this long after it finished (default: never)."),
        "activeDeadlineSeconds": _int("Fail the job after it was active this long.", "int64", 0),
        "backoffLimit": _int("Retries before the job is marked failed.", "int32", 0),
        "schedulingPolicy": SCHEDULING_POLICY,
    },
}

ELASTIC_POLICY = {
    "type": "object",
    "description": "tf-operator-amd extension: elastic Worker group restarted as a unit on failure, "
                   "preemption or capacity change (csrc/core/elastic.cc).",
    "properties": {
        "minReplicas": _int("Fewest workers the group runs with.", "int32", 1),
        "maxReplicas": _int("Most workers the group grows to.", "int32", 1),
        "maxRestarts": _int("Failure-driven group restarts before the job fails (default 10).", "int32", 0),
        "scaleUpCooldownSeconds": {"type": "number", "description": "Wait before growing the group (default 30)."},
        "scaleDownDelaySeconds": {"type": "number",
                                  "description": "Unschedulable time before shrinking the group when capacity is "
                                                 "unknown (default 30)."},
    },
}


def _obj(desc=None, **props):
    """Open object: listed properties are validated, others preserved."""
    o = {"type": "object", "x-kubernetes-preserve-unknown-fields": True}
    if props:
        o["properties"] = props
    if desc:
        o["description"] = desc
    return o


_STR = {"type": "string"}
_STRMAP = {"type": "object", "additionalProperties": {"type": "string"}}
_STRLIST = {"type": "array", "items": {"type": "string"}}

CONTAINER = {
    "type": "object",
    "x-kubernetes-preserve-unknown-fields": True,
    "required": ["name"],
    "description": "A container of the replica's pod (core/v1 Container).",
    "properties": {
        "name": {"type": "string", "minLength": 1, "maxLength": 63,
                 "pattern": "^[a-z0-9]([-a-z0-9]*[a-z0-9])?$", "description": "DNS-1123 label."},
        "image": _STR,
        "imagePullPolicy": {"type": "string", "enum": ["Always", "IfNotPresent", "Never"]},
        "command": _STRLIST,
        "args": _STRLIST,
        "workingDir": _STR,
        "env": {"type": "array", "items": {
            "type": "object", "required": ["name"],
            "properties": {"name": {"type": "string", "minLength": 1}, "value": _STR,
                           "valueFrom": _obj("ConfigMap / Secret / field / resource reference.")}}},
        "envFrom": {"type": "array", "items": _obj()},
        "ports": {"type": "array", "items": {
            "type": "object", "required": ["containerPort"],
            "properties": {"containerPort": _int("Port the container listens on.", "int32", 1) | {"maximum": 65535},
                           "hostPort": _int("Host port.", "int32", 0) | {"maximum": 65535},
                           "name": {"type": "string", "maxLength": 15},
                           "protocol": {"type": "string", "enum": ["TCP", "UDP", "SCTP"]},
                           "hostIP": _STR}}},
        "resources": {"type": "object", "description": "amd.com/gpu goes in limits (and requests).",
                      "properties": {"limits": {"type": "object", "additionalProperties": QUANTITY},
                                     "requests": {"type": "object", "additionalProperties": QUANTITY}}},
        "volumeMounts": {"type": "array", "items": {
            "type": "object", "required": ["name", "mountPath"],
            "properties": {"name": _STR, "mountPath": _STR, "readOnly": {"type": "boolean"}, "subPath": _STR,
                           "mountPropagation": _STR}}},
        "securityContext": _obj(),
        "livenessProbe": _obj(), "readinessProbe": _obj(), "startupProbe": _obj(), "lifecycle": _obj(),
        "stdin": {"type": "boolean"}, "tty": {"type": "boolean"},
        "terminationMessagePath": _STR,
        "terminationMessagePolicy": {"type": "string", "enum": ["File", "FallbackToLogsOnError"]},
    },
}

POD_TEMPLATE = {
    "type": "object",
    "description": "PodTemplateSpec of the replica (core/v1).",
    "properties": {
        "metadata": _obj("Labels and annotations are merged with the operator's.",
                         labels=_STRMAP, annotations=_STRMAP, name=_STR, namespace=_STR),
        "spec": {
            "type": "object",
            "x-kubernetes-preserve-unknown-fields": True,
            "required": ["containers"],
            "description": "PodSpec (core/v1); fields not listed are passed through to the pod.",
            "properties": {
                "containers": {"type": "array", "minItems": 1, "items": CONTAINER},
                "initContainers": {"type": "array", "items": CONTAINER},
                "volumes": {"type": "array", "items": {
                    "type": "object", "x-kubernetes-preserve-unknown-fields": True, "required": ["name"],
                    "properties": {"name": {"type": "string", "minLength": 1}}}},
                "restartPolicy": {"type": "string", "enum": ["Always", "OnFailure", "Never"],
                                  "description": "Overwritten by the replica spec's restartPolicy."},
                "nodeSelector": _STRMAP,
                "tolerations": {"type": "array", "items": {
                    "type": "object",
                    "properties": {"key": _STR, "operator": {"type": "string", "enum": ["Exists", "Equal"]},
                                   "value": _STR,
                                   "effect": {"type": "string",
                                              "enum": ["", "NoSchedule", "PreferNoSchedule", "NoExecute"]},
                                   "tolerationSeconds": _int("Seconds the toleration lasts.", "int64")}}},
                "affinity": _obj(),
                "schedulerName": _STR,
                "serviceAccountName": _STR,
                "priorityClassName": _STR,
                "hostNetwork": {"type": "boolean"},
                "hostIPC": {"type": "boolean"},
                "hostPID": {"type": "boolean"},
                "shareProcessNamespace": {"type": "boolean"},
                "terminationGracePeriodSeconds": _int("Grace period before SIGKILL.", "int64", 0),
                "activeDeadlineSeconds": _int("Pod deadline.", "int64", 1),
                "dnsPolicy": {"type": "string", "enum": ["ClusterFirst", "ClusterFirstWithHostNet", "Default",
                                                         "None"]},
                "imagePullSecrets": {"type": "array", "items": {"type": "object", "properties": {"name": _STR}}},
                "securityContext": _obj(),
            },
        },
    },
}


def replica_spec(default_restart):
    return {
        "type": "object",
        "description": "One replica type: count, restart policy and pod template.",
        "properties": {
            "replicas": _int("Number of replicas (default 1).", "int32", 0),
            "restartPolicy": {"type": "string", "enum": ["Always", "OnFailure", "Never", "ExitCode"],
                              "description": f"Restart policy (default {default_restart}). ExitCode restarts "
                                             "on retryable exit codes (>= 128)."},
            "template": copy.deepcopy(POD_TEMPLATE),
        },
    }


CONDITION = {
    "type": "object",
    "required": ["type", "status"],
    "properties": {
        "type": {"type": "string", "description": "Created, Running, Restarting, Succeeded or Failed."},
        "status": {"type": "string", "description": "True, False or Unknown."},
        "reason": {"type": "string"},
        "message": {"type": "string"},
        "lastUpdateTime": {"type": "string", "format": "date-time"},
        "lastTransitionTime": {"type": "string", "format": "date-time"},
    },
}

REPLICA_STATUS = {
    "type": "object",
    "properties": {"active": _int("Running pods."), "succeeded": _int("Succeeded pods."),
                   "failed": _int("Failed pods.")},
}

ELASTIC_STATUS = {
    "type": "object",
    "description": "State of an elastic Worker group.",
    "properties": {
        "generation": _int("Group generation (pods carry training.amd.com/elastic-generation).", "int64"),
        "currentReplicas": _int("Workers of the current generation."),
        "desiredReplicas": _int("Spec replicas clamped to [minReplicas, maxReplicas]."),
        "restarts": _int("Failure-driven restarts so far."),
        "launched": {"type": "boolean", "description": "All members of the generation are running."},
        "capacity": _int("Workers the node capacity allows."),
        "generationStartTime": {"type": "string", "format": "date-time"},
        "launchTime": {"type": "string", "format": "date-time"},
        "lastRestartTime": {"type": "string", "format": "date-time"},
        "lastRestartUnix": {"type": "number"},
        "lastScaleTime": {"type": "string", "format": "date-time"},
        "lastTransitionReason": {"type": "string"},
        "lastResumeSeconds": {"type": "number", "description": "Restart -> all members running."},
    },
}

JOB_STATUS = {
    "type": "object",
    "description": "Observed state of the job.",
    "properties": {
        "conditions": {"type": "array", "items": CONDITION},
        "replicaStatuses": {"type": "object", "additionalProperties": REPLICA_STATUS},
        "startTime": {"type": "string", "format": "date-time"},
        "completionTime": {"type": "string", "format": "date-time"},
        "lastReconcileTime": {"type": "string", "format": "date-time"},
        "elasticStatus": ELASTIC_STATUS,
    },
}


def spec_schema(kind):
    plural, singular, field, types, restart, extra = KINDS[kind]
    props = {
        "runPolicy": RUN_POLICY,
        field: {"type": "object", "additionalProperties": replica_spec(restart),
                "description": f"Replica specs keyed by type ({', '.join(types)})."},
        "elasticPolicy": ELASTIC_POLICY,
    }
    props.update(copy.deepcopy(extra))
    return {"type": "object", "required": [field], "properties": props,
            "description": f"Desired state of the {kind}."}


def job_schema(kind):
    return {
        "type": "object",
        "description": f"{kind} represents a {kind} resource.",
        "properties": {
            "apiVersion": {"type": "string"},
            "kind": {"type": "string"},
            "metadata": {"type": "object"},
            "spec": spec_schema(kind),
            "status": copy.deepcopy(JOB_STATUS),
        },
    }


def crd(kind):
    plural, singular = KINDS[kind][0], KINDS[kind][1]
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{plural}.{GROUP}", "labels": {"app.kubernetes.io/part-of": "tf-operator-amd"}},
        "spec": {
            "group": GROUP,
            "names": {"kind": kind, "listKind": kind + "List", "plural": plural, "singular": singular},
            "scope": "Namespaced",
            "versions": [{
                "name": VERSION, "served": True, "storage": True,
                "schema": {"openAPIV3Schema": job_schema(kind)},
                "subresources": {"status": {}},
                "additionalPrinterColumns": [
                    {"name": "State", "type": "string", "jsonPath": ".status.conditions[-1:].type"},
                    {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"},
                ],
            }],
        },
    }


def render(kind) -> str:
    import yaml

    return "---\n" + yaml.safe_dump(crd(kind), sort_keys=True, width=110)


def write_manifests(outdir):
    os.makedirs(outdir, exist_ok=True)
    paths = []
    for kind, (plural, *_rest) in KINDS.items():
        p = os.path.join(outdir, f"{GROUP}_{plural}.yaml")
        with open(p, "w") as f:
            f.write("# generated by `python -m tf_operator_amd.api.schema` -- do not edit\n")
            f.write(render(kind))
        paths.append(p)
    return paths


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="manifests/base")
    a = ap.parse_args(argv)
    for p in write_manifests(a.out):
        print(p)


if __name__ == "__main__":
    main()
