"""Elastic TFJob time-to-resume after preemption (BASELINE config #5:
"time-to-resume after preemption; samples/sec before and after").

Local cluster with `--node-gpus` virtual amd.com/gpu, an elastic Llama job
(minReplicas 2, maxReplicas = workers) checkpointing every few steps; after
the group has run for a while the node loses one GPU and the worker on it is
SIGKILLed.  Reports, from the operator's own records:
  * time to resume  = group restart -> first training step of the new generation
    (trainop_elastic_time_to_resume_seconds);
  * samples/sec before (world = workers) and after (world = workers - 1).

    python benchmarks/elastic_resume.py                       # CPU / gloo, llama-tiny
    python benchmarks/elastic_resume.py --model llama3-1b --gpu   # one process per GPU
    python benchmarks/elastic_resume.py --gpu --share-gpu         # every worker on GPU 0, gloo
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tf_operator_amd.sdk import container, pod_template  # noqa: E402
from tf_operator_amd.testing import chaos  # noqa: E402
from tf_operator_amd.testing.cluster import LocalCluster  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--model", default="llama-tiny")
    ap.add_argument("--seq-len", type=int, default=64)
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--gpu", action="store_true", help="workers use real GPUs (HIP_VISIBLE_DEVICES)")
    ap.add_argument("--share-gpu", action="store_true", help="with --gpu: all workers on device 0, gloo collectives")
    ap.add_argument("--warm", action="store_true", help="replicas start as forks of the kubelet's warm interpreter")
    ap.add_argument("--run-before", type=float, default=8.0, help="seconds of steady training before the fault")
    ap.add_argument("--workdir", default=None, help="local kubelet workdir (pod logs land under it)")
    a = ap.parse_args()
    ckpt = tempfile.mkdtemp(prefix="toa-elastic-")
    cmd = [sys.executable, "-m", "tf_operator_amd.examples.llama_train", "--model", a.model, "--steps", str(a.steps),
           "--seq-len", str(a.seq_len), "--micro-batch", str(a.micro_batch), "--checkpoint-every", "10",
           "--report-every", "5"]
    env = {"OMP_NUM_THREADS": "1", "TOA_LOG_PHASES": "0"}
    if not a.gpu:
        env["CUDA_VISIBLE_DEVICES"] = ""
    elif a.share_gpu:
        env["TOA_DIST_BACKEND"] = "gloo"
        cmd += ["--zero", "0"]  # replicated AdamW: gloo all-reduce on device tensors
    tpl = pod_template(container(image="toa/trainer", command=cmd, gpus=1, env=env),
                       annotations={"amd.com/checkpoint-dir": ckpt})
    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
           "metadata": {"name": "elastic", "namespace": "default", "annotations": {"amd.com/checkpoint-dir": ckpt}},
           "spec": {"elasticPolicy": {"minReplicas": 2, "maxReplicas": a.workers, "maxRestarts": 3},
                    "runPolicy": {"cleanPodPolicy": "All"},
                    "tfReplicaSpecs": {"Worker": {"replicas": a.workers, "restartPolicy": "ExitCode",
                                                  "template": tpl}}}}
    key = ("default", "elastic")
    with LocalCluster(gpus=a.workers, grace_seconds=2.0, warm_python=a.warm, workdir=a.workdir,
                      device_visibility="node" if a.share_gpu else None) as c:
        if a.warm:
            c.wait(c.kubelet.warm_ready, 120, 0.05, "kubelet fork server ready")
        c.client.create(job)
        st = lambda: (c.api.get("kubeflow.org/tfjobs", "default", "elastic") or {}).get("status") or {}
        c.wait(lambda: (c.controller.reports.get(key) or {}).get("samples_per_sec"), 600, 0.1, "first throughput")
        time.sleep(a.run_before)
        before = dict(c.controller.reports[key])
        chaos.set_gpu_capacity(c, a.workers - 1)
        t_fault = time.time()
        chaos.kill_pod(c, f"elastic-worker-{a.workers - 1}")
        c.wait(lambda: st().get("elasticStatus", {}).get("generation") == 1, 120, 0.05, "group restart")
        c.wait(lambda: (c.controller.reports.get(key) or {}).get("world") == a.workers - 1, 600, 0.1,
               "throughput after resume")
        time.sleep(a.run_before)
        after = dict(c.controller.reports[key])
        es = st().get("elasticStatus", {})
        text = c.metrics_text()
        resume = [float(l.split()[-1]) for l in text.splitlines()
                  if l.startswith("trainop_elastic_time_to_resume_seconds_sum")]
        c.client.delete("elastic")
    out = {"metric": "elastic time-to-resume after preemption", "unit": "s",
           "value": round(resume[0], 3) if resume else None,
           "fault_to_restart_s": round(float(es.get("lastRestartUnix", t_fault)) - t_fault, 3),
           "relaunch_s": round(float(es.get("lastResumeSeconds", 0.0)), 3),
           "samples_per_sec_before": round(before["samples_per_sec"], 2), "world_before": before.get("world"),
           "samples_per_sec_after": round(after["samples_per_sec"], 2), "world_after": after.get("world"),
           "generation": es.get("generation"), "restarts": es.get("restarts"),
           "config": {"model": a.model, "workers": a.workers, "seq_len": a.seq_len, "micro_batch": a.micro_batch,
                      "device": ("gpu0 shared, gloo" if a.share_gpu else "gpu, rccl") if a.gpu else "cpu/gloo",
                      "replica_start": "warm fork" if a.warm else "cold process"}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
