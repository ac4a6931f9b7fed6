"""Elastic worker groups (csrc/core/elastic.cc): group restart on retryable
failure / preemption, resize to capacity, maxRestarts, validation.

Drives the pure reconcile engine with a tiny in-memory "cluster" that applies
its actions, like the reference's FakePodControl tests (pod_test.go:529-685
for the EnableDynamicWorker scale cases this extends)."""
import copy

import pytest

from tf_operator_amd import core
from tf_operator_amd.testing import fixtures as fx

T0 = 1_700_000_000.0
GEN = "training.amd.com/elastic-generation"


def elastic_job(workers=4, mn=2, mx=4, gpus=1, max_restarts=3, policy="ExitCode", **ep):
    job = fx.new_tfjob(workers, 0)
    w = job["spec"]["tfReplicaSpecs"]["Worker"]
    w["restartPolicy"] = policy
    if gpus:
        w["template"]["spec"]["containers"][0]["resources"] = {"limits": {"amd.com/gpu": gpus}}
    job["spec"]["elasticPolicy"] = {"minReplicas": mn, "maxReplicas": mx, "maxRestarts": max_restarts, **ep}
    return job


class Sim:
    def __init__(self, job):
        self.job = core.on_job_created(job, now=T0)
        self.pods, self.svcs = {}, {}
        self.now = T0
        self.last = None

    def sync(self, free=None, dt=1.0):
        self.now += dt
        opt = {} if free is None else {"elastic_free_gpus": free}
        res = core.reconcile(self.job, list(self.pods.values()), list(self.svcs.values()), now=self.now,
                             options=opt)
        for a in res["actions"]:
            if a["op"] == "create_pod":
                p = copy.deepcopy(a["pod"])
                p["status"] = {"phase": "Pending"}
                self.pods[p["metadata"]["name"]] = p
            elif a["op"] == "delete_pod":
                self.pods.pop(a["name"], None)
            elif a["op"] == "create_service":
                self.svcs[a["service"]["metadata"]["name"]] = a["service"]
            elif a["op"] == "delete_service":
                self.svcs.pop(a["name"], None)
        self.job["status"] = res["status"]
        self.last = res
        return res

    def run_all(self):
        for p in self.pods.values():
            if p["status"]["phase"] == "Pending":
                p["status"] = {"phase": "Running"}

    def fail(self, name, code):
        self.pods[name]["status"] = {"phase": "Failed", "containerStatuses": [
            {"name": "tensorflow", "state": {"terminated": {"exitCode": code}}}]}

    def workers(self):
        return sorted(n for n, p in self.pods.items() if p["metadata"]["labels"]["replica-type"] == "worker")

    def es(self):
        return self.job["status"]["elasticStatus"]

    def env(self, name):
        return {e["name"]: e.get("value") for e in self.pods[name]["spec"]["containers"][0]["env"]}


def launch(sim, free=None):
    sim.sync(free)
    sim.run_all()
    sim.sync(free)
    assert sim.es()["launched"]


def test_initial_size_is_capacity_bounded():
    s = Sim(elastic_job(workers=4, mn=2, mx=4))
    s.sync(free=3)
    assert s.workers() == ["test-tfjob-worker-0", "test-tfjob-worker-1", "test-tfjob-worker-2"]
    assert s.es()["currentReplicas"] == 3 and s.es()["generation"] == 0
    assert s.env("test-tfjob-worker-2")["WORLD_SIZE"] == "3"
    assert s.pods["test-tfjob-worker-0"]["metadata"]["labels"][GEN] == "0"
    assert s.env("test-tfjob-worker-0")["TOA_ELASTIC_GENERATION"] == "0"
    assert s.pods["test-tfjob-worker-0"]["spec"]["restartPolicy"] == "Never"


def test_unknown_capacity_uses_desired():
    s = Sim(elastic_job(workers=4, mn=2, mx=8))
    s.sync()
    assert len(s.workers()) == 4


def test_retryable_failure_restarts_whole_group():
    s = Sim(elastic_job())
    launch(s, free=4)
    s.fail("test-tfjob-worker-2", 137)
    res = s.sync(free=4)
    # every member of generation 0 is deleted, nothing is created yet
    assert not s.pods and not [a for a in res["actions"] if a["op"] == "create_pod"]
    assert res["requeue_after"] == pytest.approx(0.5)
    assert s.es()["generation"] == 1 and s.es()["restarts"] == 1
    assert fx.check_condition(s.job["status"], "Restarting", "TFJobRestarting")
    assert res["metrics"]["restarted"] == 1
    s.sync(free=4)
    assert len(s.workers()) == 4
    assert all(p["metadata"]["labels"][GEN] == "1" for p in s.pods.values())
    assert s.env("test-tfjob-worker-0")["TOA_ELASTIC_RESTARTS"] == "1"
    s.run_all()
    s.sync(free=4)
    assert fx.check_condition(s.job["status"], "Running", "TFJobRunning")
    assert s.es()["launched"] and "lastResumeSeconds" in s.es()


def test_restart_reason_names_the_root_failure_not_a_lost_peer():
    # survivors of a killed worker exit 143 (PEER_LOST_EXIT), possibly first
    s = Sim(elastic_job())
    launch(s, free=4)
    s.fail("test-tfjob-worker-0", 143)
    s.fail("test-tfjob-worker-3", 137)
    s.sync(free=4)
    assert s.es()["lastTransitionReason"].endswith("test-tfjob-worker-3 failed with exit code 137")
    s2 = Sim(elastic_job())
    launch(s2, free=4)
    s2.fail("test-tfjob-worker-1", 143)
    s2.sync(free=4)
    assert "test-tfjob-worker-1 failed with exit code 143" in s2.es()["lastTransitionReason"]


def test_preemption_shrinks_to_capacity_then_grows_back():
    s = Sim(elastic_job(scaleUpCooldownSeconds=10))
    launch(s, free=4)
    # the node loses a GPU and worker-3 is evicted
    del s.pods["test-tfjob-worker-3"]
    s.sync(free=3)
    assert s.es()["generation"] == 1 and s.es()["currentReplicas"] == 3
    assert "disappeared" in s.es()["lastTransitionReason"]
    s.sync(free=3)
    assert s.workers() == ["test-tfjob-worker-0", "test-tfjob-worker-1", "test-tfjob-worker-2"]
    assert s.env("test-tfjob-worker-1")["WORLD_SIZE"] == "3"
    assert "test-tfjob-worker-3" not in s.svcs
    s.run_all()
    s.sync(free=3)
    assert s.es()["launched"]
    # capacity returns: resize after the cooldown, not counted as a restart
    s.sync(free=4, dt=2)
    assert s.es()["generation"] == 1
    s.sync(free=4, dt=10)
    assert s.es()["generation"] == 2 and s.es()["currentReplicas"] == 4 and s.es()["restarts"] == 1
    s.sync(free=4)
    assert len(s.workers()) == 4 and s.env("test-tfjob-worker-3")["WORLD_SIZE"] == "4"


def test_never_below_min():
    s = Sim(elastic_job(mn=2))
    launch(s, free=4)
    s.fail("test-tfjob-worker-0", 143)
    s.sync(free=1)
    s.sync(free=1)
    assert len(s.workers()) == 2  # pods wait for capacity rather than dropping below min


def test_permanent_failure_is_not_retried():
    s = Sim(elastic_job(policy="ExitCode"))
    launch(s, free=4)
    s.fail("test-tfjob-worker-1", 1)
    s.sync(free=4)
    assert s.es()["generation"] == 0
    assert fx.check_condition(s.job["status"], "Failed")


def test_onfailure_policy_retries_any_failure():
    s = Sim(elastic_job(policy="OnFailure"))
    launch(s, free=4)
    s.fail("test-tfjob-worker-1", 1)
    s.sync(free=4)
    assert s.es()["generation"] == 1


def test_max_restarts_fails_job():
    s = Sim(elastic_job(max_restarts=1))
    launch(s, free=4)
    s.fail("test-tfjob-worker-1", 137)
    s.sync(free=4)
    s.sync(free=4)
    s.run_all()
    s.sync(free=4)
    s.fail("test-tfjob-worker-0", 137)
    res = s.sync(free=4)
    assert fx.check_condition(s.job["status"], "Failed", "TFJobFailed")
    assert "maxRestarts=1" in fx.get_condition(s.job["status"], "Failed")["message"]
    # next pass is terminal: CleanPodPolicy removes what is left
    s.sync(free=4)
    assert res["status"]["elasticStatus"]["restarts"] == 1


def test_unschedulable_without_capacity_info_scales_down():
    s = Sim(elastic_job(gpus=0, mn=2, scaleDownDelaySeconds=5))
    s.sync()
    for n in ("test-tfjob-worker-0", "test-tfjob-worker-1"):
        s.pods[n]["status"] = {"phase": "Running"}
    for n in ("test-tfjob-worker-2", "test-tfjob-worker-3"):
        s.pods[n]["status"] = {"phase": "Pending", "conditions": [
            {"type": "PodScheduled", "status": "False", "reason": "Unschedulable"}]}
    res = s.sync(dt=1)
    assert s.es()["generation"] == 0 and res["requeue_after"] is not None
    s.sync(dt=5)
    assert s.es()["generation"] == 1 and s.es()["currentReplicas"] == 2 and s.es()["restarts"] == 0


def test_pytorchjob_master_counts_in_world():
    job = fx.new_pytorchjob(1, 4) if hasattr(fx, "new_pytorchjob") else None
    if job is None:
        pytest.skip("no pytorch fixture")
    job["spec"]["elasticPolicy"] = {"minReplicas": 1, "maxReplicas": 4}
    for rt in ("Master", "Worker"):
        job["spec"]["pytorchReplicaSpecs"][rt]["template"]["spec"]["containers"][0]["resources"] = {
            "limits": {"amd.com/gpu": 1}}
    s = Sim(job)
    s.sync(free=3)  # 1 master + 2 workers fit
    names = sorted(s.pods)
    assert len([n for n in names if "worker" in n]) == 2
    env = {e["name"]: e.get("value") for e in s.pods[names[0]]["spec"]["containers"][0]["env"]}
    assert env["WORLD_SIZE"] == "3"


@pytest.mark.parametrize("ep,msg", [({"minReplicas": 0}, "minReplicas"), ({"minReplicas": 3, "maxReplicas": 2},
                                                                          "maxReplicas"),
                                    ({"maxRestarts": -1}, "maxRestarts")])
def test_validation(ep, msg):
    job = fx.new_tfjob(2, 0)
    job["spec"]["elasticPolicy"] = ep
    assert msg in core.validate(job)


def test_validation_requires_worker():
    job = fx.new_tfjob(0, 1)
    job["spec"]["tfReplicaSpecs"].pop("Worker", None)
    job["spec"]["elasticPolicy"] = {"minReplicas": 1}
    assert "Worker" in core.validate(job)
