"""Typed SDK models for the kubeflow.org/v1 job CRDs.

Hand-written dataclasses that follow the Go schema (``runPolicy`` nesting,
pkg/apis/tensorflow/v1/types.go:29-111 and the CRD
manifests/base/kubeflow.org_tfjobs.yaml) -- the reference's swagger-generated
Python models carry stale flat fields (sdk/python/kubeflow/tfjob/models/
v1_tf_job_spec.py:49-63); those flat names are still
accepted here and folded into ``run_policy``.

``to_dict()`` emits Kubernetes camelCase JSON; ``from_dict()`` parses it.
Pod templates stay plain dicts (V1PodTemplateSpec-shaped).
"""
from __future__ import annotations

import dataclasses
import typing


def _camel(s: str) -> str:
    parts = s.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def _snake(s: str) -> str:
    out = []
    for ch in s:
        if ch.isupper():
            out.append("_" + ch.lower())
        else:
            out.append(ch)
    return "".join(out).lstrip("_")


_JSON_NAMES = {"api_version": "apiVersion", "tf_replica_specs": "tfReplicaSpecs",
               "pytorch_replica_specs": "pytorchReplicaSpecs", "mx_replica_specs": "mxReplicaSpecs",
               "xgb_replica_specs": "xgbReplicaSpecs", "ttl_seconds_after_finished": "ttlSecondsAfterFinished",
               "priority_class": "priorityClass"}


def _to(v):
    if dataclasses.is_dataclass(v):
        return v.to_dict()
    if isinstance(v, dict):
        return {k: _to(x) for k, x in v.items() if x is not None}
    if isinstance(v, list):
        return [_to(x) for x in v]
    return v


class _Model:
    def to_dict(self) -> dict:
        out = {}
        for f in dataclasses.fields(self):
            if f.metadata.get("skip"):
                continue
            v = getattr(self, f.name)
            if v is None:
                continue
            out[_JSON_NAMES.get(f.name, _camel(f.name))] = _to(v)
        return out

    @classmethod
    def from_dict(cls, d: dict | None):
        if d is None:
            return None
        hints = typing.get_type_hints(cls)
        kw = {}
        rev = {v: k for k, v in _JSON_NAMES.items()}
        names = {f.name for f in dataclasses.fields(cls)}
        for k, v in d.items():
            name = rev.get(k, _snake(k))
            if name not in names:
                continue
            t = hints.get(name)
            kw[name] = _from(t, v)
        return cls(**kw)

    def __getitem__(self, k):  # dict-style access for SDK ergonomics
        return self.to_dict()[k]


def _from(t, v):
    if v is None:
        return None
    origin = typing.get_origin(t)
    args = typing.get_args(t)
    if origin is typing.Union:
        non_none = [a for a in args if a is not type(None)]
        return _from(non_none[0], v) if non_none else v
    if isinstance(t, type) and issubclass(t, _Model):
        return t.from_dict(v)
    if origin is dict and len(args) == 2 and isinstance(args[1], type) and issubclass(args[1], _Model):
        return {k: args[1].from_dict(x) for k, x in v.items()}
    if origin is list and args and isinstance(args[0], type) and issubclass(args[0], _Model):
        return [args[0].from_dict(x) for x in v]
    return v


@dataclasses.dataclass
class V1SchedulingPolicy(_Model):
    min_available: typing.Optional[int] = None
    queue: typing.Optional[str] = None
    min_resources: typing.Optional[dict] = None
    priority_class: typing.Optional[str] = None


@dataclasses.dataclass
class V1RunPolicy(_Model):
    clean_pod_policy: typing.Optional[str] = None            # All | Running | None
    ttl_seconds_after_finished: typing.Optional[int] = None
    active_deadline_seconds: typing.Optional[int] = None
    backoff_limit: typing.Optional[int] = None
    scheduling_policy: typing.Optional[V1SchedulingPolicy] = None


@dataclasses.dataclass
class V1ReplicaSpec(_Model):
    replicas: typing.Optional[int] = None
    template: typing.Optional[dict] = None                   # V1PodTemplateSpec-shaped dict
    restart_policy: typing.Optional[str] = None              # Always | OnFailure | Never | ExitCode


@dataclasses.dataclass
class V1ElasticPolicy(_Model):
    """tf_operator_amd extension (BASELINE config #5; not in the reference).
    Semantics: csrc/core/elastic.cc (group restarts, resize to capacity)."""
    min_replicas: typing.Optional[int] = None
    max_replicas: typing.Optional[int] = None
    max_restarts: typing.Optional[int] = None
    scale_up_cooldown_seconds: typing.Optional[float] = None
    scale_down_delay_seconds: typing.Optional[float] = None


@dataclasses.dataclass
class V1ElasticStatus(_Model):
    generation: typing.Optional[int] = None
    current_replicas: typing.Optional[int] = None
    desired_replicas: typing.Optional[int] = None
    restarts: typing.Optional[int] = None
    launched: typing.Optional[bool] = None
    capacity: typing.Optional[int] = None
    generation_start_time: typing.Optional[str] = None
    launch_time: typing.Optional[str] = None
    last_restart_time: typing.Optional[str] = None
    last_restart_unix: typing.Optional[float] = None
    last_scale_time: typing.Optional[str] = None
    last_transition_reason: typing.Optional[str] = None
    last_resume_seconds: typing.Optional[float] = None


@dataclasses.dataclass
class V1TFJobSpec(_Model):
    tf_replica_specs: typing.Optional[typing.Dict[str, V1ReplicaSpec]] = None
    run_policy: typing.Optional[V1RunPolicy] = None
    success_policy: typing.Optional[str] = None              # "" | AllWorkers
    enable_dynamic_worker: typing.Optional[bool] = None
    elastic_policy: typing.Optional[V1ElasticPolicy] = None
    # legacy flat fields (reference SDK model) -- folded into run_policy
    clean_pod_policy: typing.Optional[str] = dataclasses.field(default=None, metadata={"skip": True})
    ttl_seconds_after_finished: typing.Optional[int] = dataclasses.field(default=None, metadata={"skip": True})
    active_deadline_seconds: typing.Optional[int] = dataclasses.field(default=None, metadata={"skip": True})
    backoff_limit: typing.Optional[int] = dataclasses.field(default=None, metadata={"skip": True})

    def __post_init__(self):
        flat = {"clean_pod_policy": self.clean_pod_policy, "ttl_seconds_after_finished": self.ttl_seconds_after_finished,
                "active_deadline_seconds": self.active_deadline_seconds, "backoff_limit": self.backoff_limit}
        if any(v is not None for v in flat.values()):
            if self.run_policy is None:
                self.run_policy = V1RunPolicy()
            for k, v in flat.items():
                if v is not None and getattr(self.run_policy, k) is None:
                    setattr(self.run_policy, k, v)


@dataclasses.dataclass
class V1JobCondition(_Model):
    type: typing.Optional[str] = None
    status: typing.Optional[str] = None
    reason: typing.Optional[str] = None
    message: typing.Optional[str] = None
    last_update_time: typing.Optional[str] = None
    last_transition_time: typing.Optional[str] = None


@dataclasses.dataclass
class V1ReplicaStatus(_Model):
    active: typing.Optional[int] = None
    succeeded: typing.Optional[int] = None
    failed: typing.Optional[int] = None


@dataclasses.dataclass
class V1JobStatus(_Model):
    conditions: typing.Optional[typing.List[V1JobCondition]] = None
    replica_statuses: typing.Optional[typing.Dict[str, V1ReplicaStatus]] = None
    start_time: typing.Optional[str] = None
    completion_time: typing.Optional[str] = None
    last_reconcile_time: typing.Optional[str] = None
    elastic_status: typing.Optional[V1ElasticStatus] = None


@dataclasses.dataclass
class V1ObjectMeta(_Model):
    name: typing.Optional[str] = None
    namespace: typing.Optional[str] = None
    labels: typing.Optional[dict] = None
    annotations: typing.Optional[dict] = None
    uid: typing.Optional[str] = None
    resource_version: typing.Optional[str] = None
    creation_timestamp: typing.Optional[str] = None
    generate_name: typing.Optional[str] = None


@dataclasses.dataclass
class V1TFJob(_Model):
    api_version: typing.Optional[str] = "kubeflow.org/v1"
    kind: typing.Optional[str] = "TFJob"
    metadata: typing.Optional[V1ObjectMeta] = None
    spec: typing.Optional[V1TFJobSpec] = None
    status: typing.Optional[V1JobStatus] = None


@dataclasses.dataclass
class V1TFJobList(_Model):
    api_version: typing.Optional[str] = "kubeflow.org/v1"
    kind: typing.Optional[str] = "TFJobList"
    items: typing.Optional[typing.List[V1TFJob]] = None
    metadata: typing.Optional[dict] = None


def container(name="tensorflow", image="", command=None, args=None, env=None, gpus=0, ports=None, resources=None):
    """Convenience V1Container-shaped dict; ``gpus`` requests ``amd.com/gpu``."""
    c = {"name": name, "image": image}
    if command:
        c["command"] = list(command)
    if args:
        c["args"] = [str(a) for a in args]
    if env:
        c["env"] = [{"name": k, "value": str(v)} for k, v in env.items()]
    if ports:
        c["ports"] = ports
    res = dict(resources or {})
    if gpus:
        res.setdefault("limits", {})["amd.com/gpu"] = gpus
    if res:
        c["resources"] = res
    return c


def pod_template(*containers, labels=None, annotations=None, **spec):
    t = {"spec": {"containers": list(containers), **spec}}
    md = {}
    if labels:
        md["labels"] = labels
    if annotations:
        md["annotations"] = annotations
    if md:
        t["metadata"] = md
    return t
