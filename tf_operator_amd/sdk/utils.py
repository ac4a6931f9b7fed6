"""SDK helpers (reference: sdk/python/kubeflow/tfjob/utils/utils.py:19-74)."""
from __future__ import annotations

import os

from . import constants

SA_DIR = "/var/run/secrets/kubernetes.io/"


def is_running_in_k8s() -> bool:
    return os.path.isdir(SA_DIR)


def get_current_k8s_namespace() -> str:
    with open(os.path.join(SA_DIR, "serviceaccount", "namespace")) as f:
        return f.readline().strip()


def get_default_target_namespace() -> str:
    return get_current_k8s_namespace() if is_running_in_k8s() else "default"


def set_tfjob_namespace(tfjob) -> str:
    md = tfjob.get("metadata", {}) if isinstance(tfjob, dict) else (tfjob.metadata or {})
    ns = md.get("namespace") if isinstance(md, dict) else getattr(md, "namespace", None)
    return ns or get_default_target_namespace()


def get_labels(name, master=False, replica_type=None, replica_index=None) -> dict:
    labels = {constants.TFJOB_GROUP_LABEL: "kubeflow.org", constants.TFJOB_NAME_LABEL: name}
    if master:
        labels[constants.TFJOB_ROLE_LABEL] = "master"
    if replica_type:
        labels[constants.TFJOB_TYPE_LABEL] = str(replica_type).lower()
    if replica_index is not None:
        labels[constants.TFJOB_INDEX_LABEL] = str(replica_index)
    return labels


def to_selector(labels: dict) -> str:
    return ",".join(f"{k}={v}" for k, v in labels.items())
