"""Elastic TFJob end to end (BASELINE config #5 on CPU/gloo): a 4-worker
Llama data-parallel job with elasticPolicy min=2 max=4 loses a GPU and a
worker (SIGKILL -> exit 137); the operator restarts the group with 3
workers, which resume from the checkpoint and finish.  Fault injection via
tf_operator_amd.testing.chaos."""
import os
import sys

import pytest

from tf_operator_amd.sdk import container, pod_template
from tf_operator_amd.testing import chaos
from tf_operator_amd.testing.cluster import LocalCluster


def _job(name, ckpt_dir, steps=40, workers=4):
    cmd = [sys.executable, "-m", "tf_operator_amd.examples.llama_train", "--steps", str(steps), "--seq-len", "32",
           "--micro-batch", "1", "--checkpoint-every", "2", "--step-sleep", "0.15"]
    tpl = pod_template(container(image="toa/trainer:latest", command=cmd, gpus=1,
                                 env={"OMP_NUM_THREADS": "1", "TOA_TEST_ELASTIC": "1"}),
                       annotations={"amd.com/checkpoint-dir": ckpt_dir})
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
            "metadata": {"name": name, "namespace": "default", "annotations": {"amd.com/checkpoint-dir": ckpt_dir}},
            "spec": {"elasticPolicy": {"minReplicas": 2, "maxReplicas": 4, "maxRestarts": 3},
                     "runPolicy": {"cleanPodPolicy": "None"},
                     "tfReplicaSpecs": {"Worker": {"replicas": workers, "restartPolicy": "ExitCode",
                                                   "template": tpl}}}}


def _status(cluster, name):
    return (cluster.api.get("kubeflow.org/tfjobs", "default", name) or {}).get("status") or {}


def _conds(st):
    return [c["type"] for c in st.get("conditions") or [] if c.get("status") == "True"]


@pytest.mark.timeout(300)
def test_elastic_shrink_on_preemption_and_resume(tmp_path):
    ckpt = str(tmp_path / "ckpt")
    with LocalCluster(gpus=4, grace_seconds=2.0) as c:
        c.client.create(_job("el", ckpt))
        c.wait(lambda: "Running" in _conds(_status(c, "el")), 120, what="job running")
        c.wait(lambda: os.path.exists(os.path.join(ckpt, "latest")), 120, what="first checkpoint")
        assert _status(c, "el")["elasticStatus"]["currentReplicas"] == 4
        # the node loses a device; the worker on it dies
        chaos.set_gpu_capacity(c, 3)
        assert chaos.kill_pod(c, "el-worker-3")
        c.wait(lambda: _status(c, "el").get("elasticStatus", {}).get("generation") == 1, 60, what="restart")
        st = c.wait(lambda: (lambda s: s if ("Succeeded" in _conds(s) or "Failed" in _conds(s)) else None)(
            _status(c, "el")), 240, what="job finished")
        assert "Succeeded" in _conds(st), st
        es = st["elasticStatus"]
        assert es["generation"] == 1 and es["restarts"] == 1 and es["currentReplicas"] == 3, str(es)
        assert "exit code 137" in es["lastTransitionReason"] or "disappeared" in es["lastTransitionReason"]
        logs = c.client.get_logs("el", master=False)
        w0 = logs.get("el-worker-0", "")
        assert "resumed at step" in w0 and "(world 3)" in w0, w0[-2000:]
        assert "done: 40 steps" in w0
        names = {p["metadata"]["name"] for p in c.pods(labels={"job-name": "el"})}
        assert "el-worker-3" not in names
        assert "trainop_elastic_time_to_resume_seconds_count" in c.metrics_text(), [l for l in c.metrics_text().splitlines() if "first_step_seconds_count" in l or "resume" in l]
