"""Small Kubernetes object helpers shared by the shell, SDK, fake API server
and local kubelet (selectors, merge-patch, owner references, phases).
Reference glue: pkg/common/util/util.go:9-38, reconciler.go:112-128."""
from __future__ import annotations

import copy


def parse_selector(s: str | dict | None) -> dict:
    """'a=b,c=d' (also '==') -> {'a': 'b', 'c': 'd'}; dicts pass through."""
    if not s:
        return {}
    if isinstance(s, dict):
        return dict(s)
    out = {}
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "==" in part:
            k, v = part.split("==", 1)
        elif "=" in part:
            k, v = part.split("=", 1)
        else:
            k, v = part, None
        out[k.strip()] = None if v is None else v.strip()
    return out


def format_selector(d: dict) -> str:
    return ",".join(f"{k}={v}" for k, v in d.items())


def match_labels(labels: dict, sel: dict) -> bool:
    for k, v in sel.items():
        if v is None:
            if k not in labels:
                return False
        elif labels.get(k) != v:
            return False
    return True


def _field(obj, path):
    cur = obj
    for p in path.split("."):
        if not isinstance(cur, dict):
            return None
        cur = cur.get(p)
    return cur


def match_fields(obj: dict, sel: dict) -> bool:
    for k, v in sel.items():
        if str(_field(obj, k)) != str(v):
            return False
    return True


def json_merge_patch(target, patch):
    """RFC 7386 JSON merge patch (what `kubectl patch --type=merge` sends)."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    if not isinstance(target, dict):
        target = {}
    for k, v in patch.items():
        if v is None:
            target.pop(k, None)
        else:
            target[k] = json_merge_patch(target.get(k), v)
    return target


def key_of(obj: dict) -> str:
    md = obj.get("metadata", {})
    ns = md.get("namespace", "")
    return f"{ns}/{md.get('name', '')}" if ns else md.get("name", "")


def controller_ref(obj: dict):
    for r in obj.get("metadata", {}).get("ownerReferences") or []:
        if r.get("controller"):
            return r
    return None


def pod_phase(pod: dict) -> str:
    return (pod.get("status") or {}).get("phase", "")


def is_terminal(pod: dict) -> bool:
    return pod_phase(pod) in ("Succeeded", "Failed")


def last_condition(job: dict):
    conds = (job.get("status") or {}).get("conditions") or []
    return conds[-1] if conds else None
