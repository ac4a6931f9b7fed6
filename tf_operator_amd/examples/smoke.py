"""Cluster smoke test (reference: examples/tf_sample/tf_smoke.py): the chief
places a 10x10 integer multiply on EVERY task.  Here every rank of the
RCCL/gloo world computes a 10x10 product on its own device, the results are
all-gathered to the chief, which checks them (in-graph replication analog,
SURVEY P8 / K18).  PS replicas just wait (server.join analog)."""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from tf_operator_amd.examples.common import pick_device
from tf_operator_amd.train.runtime import Runtime


def main():
    rt = Runtime()
    if rt.role == "ps":
        while True:
            time.sleep(3600)
    info = rt.init_dist()
    dev = pick_device() if info.backend != "gloo" else torch.device("cpu")
    a = torch.arange(100, dtype=torch.int64, device=dev).view(10, 10) + rt.rank
    prod = (a * 2).to(torch.int64)
    if dist.is_initialized():
        outs = [torch.empty_like(prod) for _ in range(rt.world)]
        dist.all_gather(outs, prod)
    else:
        outs = [prod]
    for r, o in enumerate(outs):
        want = (torch.arange(100, dtype=torch.int64, device=dev).view(10, 10) + r) * 2
        assert torch.equal(o, want), f"rank {r} mismatch"
    rt.first_step_done()
    rt.log(f"smoke ok on {rt.world} task(s), device {dev}")


if __name__ == "__main__":
    main()
