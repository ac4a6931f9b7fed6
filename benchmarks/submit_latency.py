"""Submit -> first-step latency of a TFJob (BASELINE metric, second half:
"p50 submit->first-step latency at 1/2/4/8 GPUs").

Runs the whole stack in one process -- fake API server, operator (C++ core +
asyncio shell), local kubelet that starts one process per worker pinned to a
GPU (HIP_VISIBLE_DEVICES) -- submits the same TFJob `--repeats` times and
reports, per run, the client-side clock from `create()` to rank 0's first
completed optimizer step (reported back to the operator), with a breakdown:

    submit -> all pods created (operator)  -> all processes spawned (kubelet)
           -> first step done (rendezvous + model init + step 1)

    python benchmarks/submit_latency.py --workers 1 --payload llama --model llama3-8b   # GPU
    python benchmarks/submit_latency.py --workers 1 --payload mnist                      # CPU, config #1

Prints one JSON line (p50/p90/min/max + breakdown medians)."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tf_operator_amd.bench.flagship import vram_used_bytes, wait_vram_drained, wait_vram_settled  # noqa: E402
from tf_operator_amd.sdk import container, pod_template  # noqa: E402
from tf_operator_amd.testing.cluster import LocalCluster  # noqa: E402


def payload_cmd(a):
    py = [sys.executable, "-m"]
    if a.payload == "mnist":
        return py + ["tf_operator_amd.examples.dist_mnist", "--train_steps", "5", "--log_every", "0"]
    if a.payload == "resnet":
        return py + ["tf_operator_amd.examples.resnet_train", "--steps", "2", "--warmup", "0", "--batch",
                     str(a.micro_batch)]
    return py + ["tf_operator_amd.examples.llama_train", "--model", a.model, "--steps", "2", "--seq-len",
                 str(a.seq_len), "--micro-batch", str(a.micro_batch)]


def make_job(name, a):
    gpus = 1 if a.gpus_per_worker else 0
    tpl = pod_template(container(image="toa/trainer:latest", command=payload_cmd(a), gpus=gpus,
                                 env={"OMP_NUM_THREADS": "4"}))
    specs = {"Worker": {"replicas": a.workers, "restartPolicy": "Never", "template": tpl}}
    if a.ps:
        specs["PS"] = {"replicas": a.ps, "restartPolicy": "Never", "template": tpl}
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"runPolicy": {"cleanPodPolicy": "All"}, "tfReplicaSpecs": specs}}


def one_run(c, i, a, vram_base=None):
    name = f"lat-{i}"
    t0 = time.time()
    c.client.create(make_job(name, a))
    key = ("default", name)
    n_pods = a.workers + a.ps
    c.wait(lambda: len(c.pods(labels={"job-name": name})) >= n_pods, a.timeout, 0.005, "pods created")
    t_pods = time.time()
    c.wait(lambda: sum(1 for k in c.kubelet.start_times if k[1].startswith(name + "-")) >= n_pods, a.timeout,
           0.005, "processes spawned")
    t_spawn = max(v[0] for k, v in c.kubelet.start_times.items() if k[1].startswith(name + "-"))
    rep = c.wait(lambda: (c.controller.reports.get(key) or {}).get("first_step_time") and c.controller.reports[key],
                 a.timeout, 0.01, "first step")
    t_first = float(rep["first_step_time"])
    c.client.wait_for_job(name, polling_interval=0.2, timeout_seconds=a.timeout)
    c.client.delete(name)
    c.wait(lambda: not c.pods(labels={"job-name": name}) and not any(
        k[1].startswith(name + "-") for k in c.kubelet.running), 60, 0.05, "cleanup")
    drain = wait_vram_drained(vram_base)  # the next job starts on a drained node (bench/flagship.py)
    out = {"total": t_first - t0, "to_pods": t_pods - t0, "to_spawn": t_spawn - t0,
           "spawn_to_first": t_first - t_spawn, "node_drain": drain}
    for k, v in (rep.get("phases") or {}).items():
        out["phase:" + k] = v
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workers", type=int, default=1)
    p.add_argument("--ps", type=int, default=0)
    p.add_argument("--payload", choices=["llama", "mnist", "resnet"], default="llama")
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--seq-len", type=int, default=4096)
    p.add_argument("--micro-batch", type=int, default=4)
    p.add_argument("--repeats", type=int, default=5)
    p.add_argument("--gpus", type=int, default=None, help="node GPUs (default: workers if --gpus-per-worker)")
    p.add_argument("--gpus-per-worker", type=int, default=1)
    p.add_argument("--timeout", type=float, default=600)
    p.add_argument("--warm", action="store_true", help="start replicas from the kubelet's warm fork server")
    a = p.parse_args()
    node_gpus = a.gpus if a.gpus is not None else (a.workers if a.gpus_per_worker else 0)
    runs = []
    with LocalCluster(gpus=node_gpus, grace_seconds=5.0, warm_python=a.warm) as c:
        if a.warm:
            c.wait(c.kubelet.warm_ready, 300, what="fork server ready")
        wait_vram_settled()
        base = vram_used_bytes()
        for i in range(a.repeats):
            r = one_run(c, i, a, base)
            runs.append(r)
            print(json.dumps({"run": i, **{k: round(v, 4) for k, v in r.items()}}), file=sys.stderr, flush=True)
    tot = sorted(r["total"] for r in runs)

    def med(k):
        return round(statistics.median(r[k] for r in runs), 4)

    out = {"metric": "p50 submit->first-step latency", "unit": "s", "value": med("total"),
           "p90": round(tot[min(len(tot) - 1, int(0.9 * len(tot)))], 4), "min": round(tot[0], 4),
           "max": round(tot[-1], 4), "repeats": len(runs), "warm_start": a.warm, "n_gpus": a.workers * a.gpus_per_worker,
           "breakdown_p50": {"submit_to_pods_created": med("to_pods"), "submit_to_processes_spawned": med("to_spawn"),
                             "spawn_to_first_step": med("spawn_to_first"),
                             **{k[6:]: med(k) for k in runs[0] if k.startswith("phase:")
                                and all(k in r for r in runs)}},
           "config": {"payload": a.payload, "model": a.model if a.payload == "llama" else a.payload,
                      "workers": a.workers, "ps": a.ps, "seq_len": a.seq_len, "micro_batch": a.micro_batch}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
