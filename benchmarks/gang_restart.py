"""Gang-scheduled TFJob restart recovery (BASELINE config #4: Volcano
PodGroup Worker=N, restartPolicy OnFailure; metrics "submit->first-step p50;
restart recovery time").

Local cluster with gang scheduling on (PodGroup minMember = N, all-or-nothing
admission in the local kubelet), a Llama data-parallel job checkpointing
every few steps.  After steady training one worker's process is SIGKILLed
(exit 137, a crashed rank).  OnFailure restarts it in place; the surviving
ranks see their collective break, exit with the retryable peer-lost code and
are restarted too; the new group re-forms the process group and resumes from
the last checkpoint.  Reported:

  * submit -> first step of the job (create() to rank 0's first step);
  * recovery = fault -> first training step of the restarted group;
  * per-pod container restart counts (every rank restarts once);
  * samples/sec before and after.

    python benchmarks/gang_restart.py                  # CPU / gloo, llama-tiny, 4 workers
    python benchmarks/gang_restart.py --gpu --model llama3-1b --workers 8      # one GPU per worker, RCCL
    python benchmarks/gang_restart.py --gpu --share-gpu --workers 4            # every worker on GPU 0, gloo

--share-gpu runs the GPU payload (HIP init, model on the device, HIP kernels)
on a one-GPU box: the node advertises one GPU per worker, every replica
drives device 0 (node-visible devices, index modulo the device count), and
the collectives are gloo, because RCCL refuses two ranks on one device.
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


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--model", default="llama-tiny")
    ap.add_argument("--seq-len", type=int, default=64)
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--steps", type=int, default=100000)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--share-gpu", action="store_true", help="with --gpu: all workers on device 0, gloo collectives")
    ap.add_argument("--warm", action="store_true", help="replicas start as forks of the kubelet's warm interpreter")
    ap.add_argument("--run-before", type=float, default=6.0, help="seconds of steady training before the fault")
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("--workdir", default=None, help="local kubelet workdir (pod logs land under it)")
    a = ap.parse_args(argv)
    ckpt = tempfile.mkdtemp(prefix="toa-gang-")
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
    name = "gang"
    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
           "metadata": {"name": name, "namespace": "default", "annotations": {"amd.com/checkpoint-dir": ckpt}},
           "spec": {"runPolicy": {"cleanPodPolicy": "All", "schedulingPolicy": {"minAvailable": a.workers}},
                    "tfReplicaSpecs": {"Worker": {"replicas": a.workers, "restartPolicy": "OnFailure",
                                                  "template": tpl}}}}
    key = ("default", name)
    def say(msg):
        print(f"[gang_restart] {time.time() - t_start:7.2f}s {msg}", file=sys.stderr, flush=True)

    t_start = time.time()
    with LocalCluster(gpus=a.workers, enable_gang_scheduling=True, grace_seconds=2.0, warm_python=a.warm,
                      device_visibility="node" if a.share_gpu else None, workdir=a.workdir) as c:
        if a.warm:
            c.wait(c.kubelet.warm_ready, 120, 0.05, "kubelet fork server ready")
        t_submit = time.time()
        c.client.create(job)
        say("submitted")
        rep = lambda: c.controller.reports.get(key) or {}  # noqa: E731
        c.wait(lambda: rep().get("first_step_time"), a.timeout, 0.02, "first step")
        say("first step")
        first = float(rep()["first_step_time"]) - t_submit
        pg = c.api.get("scheduling.volcano.sh/podgroups", "default", name) or {}
        c.wait(lambda: rep().get("samples_per_sec"), a.timeout, 0.1, "first throughput")
        time.sleep(a.run_before)
        before = dict(rep())
        step_before = int(before.get("step") or 0)
        t_fault = time.time()
        assert chaos.kill_pod(c, f"{name}-worker-1"), "worker-1 has no running process"
        say(f"killed worker-1 at step {step_before}")
        c.wait(lambda: float(rep().get("last_first_step_time") or 0) > t_fault, a.timeout, 0.02,
               "first step after restart")
        resumed = dict(rep())
        recovery = float(resumed["last_first_step_time"]) - t_fault
        say(f"restarted group's first step after {recovery:.3f}s")
        c.wait(lambda: (rep().get("samples_per_sec") and int(rep().get("step") or 0) > int(resumed.get("step") or 0)
                        + 5), a.timeout, 0.1, "throughput after restart")
        time.sleep(a.run_before)
        after = dict(rep())
        job_now = c.client.get(name)
        restarts = {p["metadata"]["name"]: sum(cs.get("restartCount", 0) for cs in
                                               (p.get("status") or {}).get("containerStatuses") or [])
                    for p in c.pods(labels={"job-name": name})}
        conds = [x["type"] for x in (job_now.get("status") or {}).get("conditions") or []]
        c.client.delete(name)
    out = {"metric": "gang-scheduled TFJob restart recovery (fault -> first step of the restarted group)",
           "unit": "s", "value": round(recovery, 3), "submit_to_first_step_s": round(first, 3),
           "podgroup_min_member": (pg.get("spec") or {}).get("minMember"),
           "step_at_fault": step_before, "samples_per_sec_before": round(before["samples_per_sec"], 2),
           "samples_per_sec_after": round(after["samples_per_sec"], 2), "conditions": conds,
           "restarts": restarts,
           "config": {"model": a.model, "workers": a.workers, "seq_len": a.seq_len, "micro_batch": a.micro_batch,
                      "device": ("gpu0 shared, gloo" if a.share_gpu else "gpu, rccl") if a.gpu else "cpu/gloo",
                      "replica_start": "warm fork" if a.warm else "cold process",
                      "restartPolicy": "OnFailure", "gang": True}}
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    main()
