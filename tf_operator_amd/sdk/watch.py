"""Table watch of TFJobs until Succeeded/Failed (reference:
sdk/python/kubeflow/tfjob/api/tf_job_watch.py:23-59 -- NAME/STATE/TIME
table, stops on a terminal state, retried up to 20 x 1 s)."""
from __future__ import annotations

import json
import sys
import time

from . import utils

COLS = (("NAME", 30), ("STATE", 20), ("TIME", 30))


def _row(vals, out):
    out.write("".join(str(v).ljust(w) for v, (_, w) in zip(vals, COLS)) + "\n")
    out.flush()


def watch(client, name=None, namespace=None, timeout_seconds=600, out=None, retries=20):
    out = out or sys.stdout
    namespace = namespace or utils.get_default_target_namespace()
    last = None
    for attempt in range(retries):
        try:
            _row([c for c, _ in COLS], out)
            r = client.rest.call("GET", client._path(namespace), params={"watch": "true",
                                                                          "timeoutSeconds": str(timeout_seconds)},
                                 stream=True)
            for line in r.iter_lines(decode_unicode=True):
                if not line:
                    continue
                ev = json.loads(line)
                job = ev.get("object") or {}
                jname = job.get("metadata", {}).get("name")
                if ev.get("type") == "BOOKMARK" or not jname or (name and name != jname):
                    continue
                conds = (job.get("status") or {}).get("conditions") or [{}]
                state, ts = conds[-1].get("type", ""), conds[-1].get("lastTransitionTime", "")
                if (jname, state) != last:
                    _row([jname, state, ts], out)
                    last = (jname, state)
                if name == jname and state in ("Succeeded", "Failed"):
                    return state
            return last[1] if last else None
        except Exception:
            if attempt == retries - 1:
                raise
            time.sleep(1)
    return None
