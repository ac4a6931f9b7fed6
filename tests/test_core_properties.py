"""Property tests (hypothesis) on the C++ status/condition and reconcile
engines -- SURVEY section 5 "Race detection / sanitizers": the reference
pins these behaviours with a fixed table only (status_test.go:120-425,
:585-592); here random sequences and random pod populations check the
invariants every table row relies on."""
import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from tf_operator_amd import core  # noqa: E402
from tf_operator_amd.testing import fixtures as fx  # noqa: E402

NOW = 1_700_000_000.0
CTYPES = ["Created", "Running", "Restarting", "Succeeded", "Failed"]


def _true(status, t):
    return any(c["type"] == t and c["status"] == "True" for c in status.get("conditions") or [])


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(CTYPES), st.sampled_from(["A", "B"])), min_size=1, max_size=12))
def test_condition_sequences_keep_invariants(seq):
    """UpdateJobConditions (kubeflow/common): one condition per type, the
    newest appended last, Running never True next to Succeeded/Failed,
    Running and Restarting mutually exclusive, and a repeated
    (type, reason) is a no-op."""
    status = {"conditions": []}
    for i, (ctype, reason) in enumerate(seq):
        before = status
        status, changed = core.update_job_conditions(status, ctype, reason, f"m{i}", now=NOW + i)
        conds = status["conditions"]
        types = [c["type"] for c in conds]
        assert len(types) == len(set(types)), types
        if changed:
            assert conds[-1]["type"] == ctype and conds[-1]["reason"] == reason
        else:
            assert status == before
        if _true(status, "Succeeded") or _true(status, "Failed"):
            assert not _true(status, "Running")
        assert not (_true(status, "Running") and _true(status, "Restarting"))
    again, changed = core.update_job_conditions(status, seq[-1][0], seq[-1][1], "again", now=NOW + 99)
    if status["conditions"] and status["conditions"][-1]["type"] == seq[-1][0]:
        assert not changed and again == status


PHASES = ["Pending", "Running", "Succeeded", "Failed"]


@settings(max_examples=200, deadline=None)
@given(workers=st.integers(1, 5), ps=st.integers(0, 3), chief=st.integers(0, 1),
       wph=st.lists(st.sampled_from(PHASES + [None]), min_size=5, max_size=5),
       pph=st.lists(st.sampled_from(PHASES + [None]), min_size=3, max_size=3),
       cph=st.sampled_from(PHASES + [None]))
def test_reconcile_invariants(workers, ps, chief, wph, pph, cph):
    """For any observed pod population of a TFJob: exactly the missing
    replica indices get a pod, created names follow <job>-<rtype>-<index>,
    the status never has Running True next to Succeeded/Failed, and once a
    sync has made the job terminal the next sync creates nothing (the
    terminal check reads the job's stored status, as ReconcileJobs does)."""
    job = fx.new_tfjob(workers, ps, chief=chief)
    pods = []
    have = {}
    for typ, n, phases in (("worker", workers, wph), ("ps", ps, pph), ("chief", chief, [cph])):
        have[typ] = set()
        for i in range(n):
            ph = phases[i]
            if ph is None:
                continue
            pods.append(fx.new_pod(job, typ, i, ph))
            have[typ].add(i)
    res = core.reconcile(job, pods, [], now=NOW, options={})
    status = res["status"]
    if _true(status, "Succeeded") or _true(status, "Failed"):
        assert not _true(status, "Running")
    creates = [a for a in res["actions"] if a["op"] == "create_pod"]
    if _true(status, "Succeeded") or _true(status, "Failed"):
        job2 = dict(job, status=status)
        res2 = core.reconcile(job2, pods, [], now=NOW + 1, options={})
        assert not [a for a in res2["actions"] if a["op"] == "create_pod"]
    name = job["metadata"]["name"]
    got = {}
    for a in creates:
        pod = a.get("pod") or a.get("object") or {}
        labels = pod.get("metadata", {}).get("labels", {})
        typ, idx = labels[fx.REPLICA_TYPE_LABEL], int(labels[fx.REPLICA_INDEX_LABEL])
        assert pod["metadata"]["name"] == f"{name}-{typ}-{idx}"
        got.setdefault(typ, set()).add(idx)
    for typ, n in (("worker", workers), ("ps", ps), ("chief", chief)):
        assert got.get(typ, set()) == set(range(n)) - have[typ], (typ, got, have)
