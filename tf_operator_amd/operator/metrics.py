"""Prometheus metrics (reference names kept: docs/monitoring/README.md:52-91,
pkg/controller.v1/tensorflow/{job.go:29-37, controller.go:70-76,
status.go:47-62, pod.go:57-65}, cmd/tf-operator.v1/app/server.go:64-69)
plus the new ones BASELINE.json needs (submit->first-step latency,
samples/sec, reconcile duration)."""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

LATENCY_BUCKETS = (0.5, 1, 2, 3, 5, 7.5, 10, 15, 20, 30, 45, 60, 90, 120, 180, 300, 600)


class OperatorMetrics:
    def __init__(self, registry: CollectorRegistry | None = None, prefix="tf_operator"):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.created = Counter(f"{prefix}_jobs_created", "Counts number of jobs created", ["job_namespace"],
                               registry=r)
        self.deleted = Counter(f"{prefix}_jobs_deleted", "Counts number of jobs deleted", ["job_namespace"],
                               registry=r)
        self.successful = Counter(f"{prefix}_jobs_successful", "Counts number of jobs successful",
                                  ["job_namespace"], registry=r)
        self.failed = Counter(f"{prefix}_jobs_failed", "Counts number of jobs failed", ["job_namespace"], registry=r)
        self.restarted = Counter(f"{prefix}_jobs_restarted", "Counts number of jobs restarted", ["job_namespace"],
                                 registry=r)
        self.is_leader = Gauge(f"{prefix}_is_leader", "Is this client the leader of this tf-operator client set?",
                               registry=r)
        self.reconcile_seconds = Histogram("trainop_reconcile_duration_seconds", "Duration of one job sync",
                                           ["kind"], registry=r,
                                           buckets=(.0005, .001, .0025, .005, .01, .025, .05, .1, .25, .5, 1, 2.5))
        self.first_step = Histogram("trainop_job_submit_to_first_step_seconds",
                                    "Job creationTimestamp -> first completed training step (rank 0)",
                                    ["job_namespace", "kind"], registry=r, buckets=LATENCY_BUCKETS)
        self.time_to_resume = Histogram("trainop_elastic_time_to_resume_seconds",
                                        "Elastic group restart -> first training step of the new generation",
                                        ["job_namespace", "kind"], registry=r, buckets=LATENCY_BUCKETS)
        self.samples_per_sec = Gauge("trainop_samples_per_second", "Training throughput reported by rank 0",
                                     ["job_namespace", "job_name"], registry=r)

    def expose(self) -> bytes:
        return generate_latest(self.registry)
