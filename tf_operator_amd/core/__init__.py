"""Python face of the C++17 operator core (``_toa_core``, built from csrc/core/).

Every function takes / returns plain dicts; JSON text is the wire format to
C++.  The core is pure: no Kubernetes I/O happens here (see
:mod:`tf_operator_amd.operator` for the asyncio shell that executes the
returned actions).
"""
from __future__ import annotations

import importlib
import json
import time

_mod = None


def native():
    """Return the compiled pybind11 module; raise if it has not been built."""
    global _mod
    if _mod is None:
        try:
            _mod = importlib.import_module("tf_operator_amd.core._toa_core")
        except ImportError:
            # build on first use (CPU-only toolchain, ~10 s)
            from .. import _build

            _build.build_core()
            try:
                _mod = importlib.import_module("tf_operator_amd.core._toa_core")
            except ImportError as e:  # pragma: no cover
                raise RuntimeError("C++ operator core not built: run `python -m tf_operator_amd._build --only core`") \
                    from e
    return _mod


def _d(x):
    return json.dumps(x, separators=(",", ":")) if x is not None else ""


def _now(now):
    return time.time() if now is None else float(now)


def supported_kinds():
    return list(native().supported_kinds())


def kind_info(kind):
    return dict(native().kind_info(kind))


def set_defaults(job: dict) -> dict:
    return json.loads(native().set_defaults(_d(job)))


def validate(job: dict) -> str:
    """'' when valid, else the reference-compatible error message."""
    return native().validate(_d(job))


def on_job_created(job: dict, now=None) -> dict:
    return json.loads(native().on_job_created(_d(job), _now(now)))


def claim_objects(job: dict, objs) -> dict:
    """ControllerRef claim (adopt orphans / release mismatches): see csrc/core/claim.cc."""
    return json.loads(native().claim_objects(_d(job), _d(list(objs))))


def reconcile(job: dict, pods=(), services=(), now=None, options: dict | None = None) -> dict:
    return json.loads(native().reconcile(_d(job), _d(list(pods)), _d(list(services)), _now(now), _d(options or {})))


def gen_tf_config(job: dict, rtype: str, index: int, options: dict | None = None) -> str:
    return native().gen_tf_config(_d(job), rtype, int(index), _d(options or {}))


def node_local(job: dict, options: dict | None = None) -> bool:
    """Does the job's RCCL world run in the single-node xGMI layout
    (csrc/core/nodelocal.cc)?"""
    return bool(native().node_local(_d(job), _d(options or {})))


def gen_env(job: dict, rtype: str, index: int, options: dict | None = None) -> list:
    return json.loads(native().gen_env(_d(job), rtype, int(index), _d(options or {})))


def set_cluster_spec(job: dict, template: dict, rtype: str, index: int, options: dict | None = None) -> dict:
    """The pod template with the replica's environment applied (what the
    reconciler does to every pod it creates)."""
    return json.loads(native().set_cluster_spec(_d(job), _d(template), rtype, int(index), _d(options or {})))


def tf_is_distributed(job: dict) -> bool:
    return bool(native().tf_is_distributed(_d(job)))


def gen_podgroup(job: dict, options: dict | None = None) -> dict:
    return json.loads(native().gen_podgroup(_d(job), _d(options or {})))


def update_job_conditions(status: dict, ctype: str, reason: str, message: str, now=None):
    s, changed = native().update_job_conditions(_d(status), ctype, reason, message, _now(now))
    return json.loads(s), bool(changed)


def is_retryable_exit_code(code: int) -> bool:
    return bool(native().is_retryable_exit_code(int(code)))


def rfc3339(t=None) -> str:
    return native().rfc3339(_now(t))


def parse_rfc3339(s: str) -> float:
    return native().parse_rfc3339(s)


def gen_general_name(job, rt, index):
    return native().gen_general_name(job, rt, str(index))


def Expectations(ttl_seconds=300.0):
    return native().Expectations(ttl_seconds)


def WorkQueue(base_delay=0.005, max_delay=1000.0):
    return native().WorkQueue(base_delay, max_delay)


class Store:
    """dict-level wrapper over the native indexed cache."""

    def __init__(self):
        self._s = native().Store()

    def upsert(self, obj: dict) -> bool:
        return self._s.upsert(_d(obj))

    def remove(self, key: str) -> bool:
        return self._s.remove(key)

    def get(self, key: str):
        v = self._s.get(key)
        return None if v is None else json.loads(v)

    def list(self, namespace: str = "", selector: dict | None = None) -> list:
        return json.loads(self._s.list(namespace, _d(selector or {})))

    def keys(self):
        return list(self._s.keys())

    def __len__(self):
        return len(self._s)

    @staticmethod
    def key_of(obj: dict) -> str:
        md = obj.get("metadata", {})
        ns = md.get("namespace", "")
        return f"{ns}/{md.get('name', '')}" if ns else md.get("name", "")
