"""Control-plane scale benchmark: many concurrent TFJobs through the whole
operator stack (fake API server, operator = C++ core + asyncio shell, local
kubelet running each replica as a real process).

The reference states its design target as O(100) concurrent TF jobs per
cluster (docs/design/tf_job_design_doc.md:24) and publishes no numbers.
This submits `--jobs` TFJobs at once, each with `--workers` Worker replicas
that run `sleep --sleep` (so every job is Running at the same time), and
measures, per job, create -> Running and create -> Succeeded on the client's
clock, plus the operator's per-sync reconcile duration (the
trainop_reconcile_duration_seconds histogram) and the API write rate.

    python benchmarks/operator_scale.py --jobs 100 --workers 2 [--qps 5 --burst 10]

`--qps/--burst` throttle the operator's API client like the reference's
flags (options.go:81-82 defaults 5 / 10); 0 = unthrottled.  Prints one JSON
line.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tf_operator_amd.sdk import container, pod_template  # noqa: E402
from tf_operator_amd.testing.cluster import LocalCluster  # noqa: E402


def make_job(name, workers, sleep_s):
    tpl = pod_template(container(image="toa/trainer:latest", command=["sleep", str(sleep_s)]))
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"runPolicy": {"cleanPodPolicy": "All"},
                     "tfReplicaSpecs": {"Worker": {"replicas": workers, "restartPolicy": "Never", "template": tpl}}}}


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q * (len(xs) - 1))))]


def _hist_quantile(hist, q):
    """Quantile (upper bucket bound) from a prometheus_client Histogram."""
    buckets = []
    for metric in hist.collect():
        for s in metric.samples:
            if s.name.endswith("_bucket"):
                buckets.append((float(s.labels["le"]), s.value))
    agg = {}
    for le, v in buckets:
        agg[le] = agg.get(le, 0.0) + v
    items = sorted(agg.items())
    if not items or items[-1][1] == 0:
        return None
    target = q * items[-1][1]
    for le, v in items:
        if v >= target:
            return le
    return items[-1][0]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--jobs", type=int, default=100)
    p.add_argument("--workers", type=int, default=2)
    p.add_argument("--sleep", type=float, default=3.0)
    p.add_argument("--threadiness", type=int, default=4)
    p.add_argument("--qps", type=float, default=0.0)
    p.add_argument("--burst", type=int, default=0)
    p.add_argument("--timeout", type=float, default=600)
    a = p.parse_args()
    with LocalCluster(gpus=0, kinds=("TFJob",), threadiness=a.threadiness, qps=a.qps, grace_seconds=1.0) as c:
        if a.burst:
            c.kube_op.limiter.burst = c.kube_op.limiter.tokens = float(a.burst)
        names = [f"scale-{i}" for i in range(a.jobs)]
        t_create = {}
        t0 = time.time()
        for n in names:
            t_create[n] = time.time()
            c.client.create(make_job(n, a.workers, a.sleep))
        t_submitted = time.time()
        running, done = {}, {}
        deadline = t0 + a.timeout
        while len(done) < len(names) and time.time() < deadline:
            for n in names:
                if n in done:
                    continue
                conds = [x["type"] for x in ((c.client.get(n).get("status") or {}).get("conditions") or [])
                         if x.get("status") == "True"]
                now = time.time()
                if n not in running and ("Running" in conds or "Succeeded" in conds):
                    running[n] = now
                if "Succeeded" in conds or "Failed" in conds:
                    done[n] = (now, "Succeeded" in conds)
            time.sleep(0.05)
        t_end = time.time()
        ok = sum(1 for v in done.values() if v[1])
        to_run = [running[n] - t_create[n] for n in running]
        to_done = [done[n][0] - t_create[n] for n in done]
        hist = c.metrics.reconcile_seconds
        out = {
            "metric": "concurrent TFJobs: create -> Running p50", "unit": "s",
            "value": round(statistics.median(to_run), 3) if to_run else None,
            "jobs": a.jobs, "workers_per_job": a.workers, "succeeded": ok,
            "submit_seconds": round(t_submitted - t0, 3),
            "wall_seconds": round(t_end - t0, 3),
            "create_to_running_s": {"p50": round(statistics.median(to_run), 3), "p99": round(_pct(to_run, .99), 3),
                                    "max": round(max(to_run), 3)} if to_run else None,
            "create_to_succeeded_s": {"p50": round(statistics.median(to_done), 3),
                                      "p99": round(_pct(to_done, .99), 3)} if to_done else None,
            "reconcile_s": {"p50_le": _hist_quantile(hist, .5), "p99_le": _hist_quantile(hist, .99)},
            "pods": a.jobs * a.workers, "sleep_s": a.sleep,
            "operator": {"threadiness": a.threadiness, "qps": a.qps or "unthrottled", "burst": a.burst or None},
        }
    print(json.dumps(out))
    if ok != a.jobs:
        sys.exit(1)


if __name__ == "__main__":
    main()
