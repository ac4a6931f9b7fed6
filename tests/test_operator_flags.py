"""Scheme registry (register_controller.go:52-76) and the client's QPS/burst
token bucket (clientset.go:62) — SURVEY.md §2 D10 and B1."""
import asyncio
import time

import pytest

from tf_operator_amd.operator.kube import TokenBucket
from tf_operator_amd.operator.main import enabled_kinds


def test_enable_scheme_all_when_empty():
    assert set(enabled_kinds([])) == {"TFJob", "PyTorchJob", "MXJob", "XGBoostJob"}


def test_enable_scheme_case_insensitive_and_dedup():
    assert enabled_kinds(["TFJob", "tfjob,PYTORCHJOB"]) == ["TFJob", "PyTorchJob"]


def test_enable_scheme_rejects_unknown():
    with pytest.raises(SystemExit):
        enabled_kinds(["caffejob"])


def test_token_bucket_burst_then_rate():
    async def run():
        tb = TokenBucket(qps=50, burst=5)
        t0 = time.monotonic()
        for _ in range(5):
            await tb.acquire()
        burst_s = time.monotonic() - t0
        for _ in range(5):
            await tb.acquire()
        return burst_s, time.monotonic() - t0
    burst_s, total_s = asyncio.run(run())
    assert burst_s < 0.05           # the burst is free
    assert total_s >= 5 / 50 * 0.8  # then 50 QPS
