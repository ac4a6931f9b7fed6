"""One-GPU emulation of a world-N ZeRO-1 step's collective traffic.

The N=8 headline depends on the bucketed reduce-scatter / all-gather
(parallel/zero.py) overlapping the backward and forward GEMMs.  A one-GPU
box cannot run RCCL at world 8, but what those collectives do to THIS GPU
can be reproduced: RCCL's ring kernel holds `channels` workgroups for the
whole collective, streams (N-1)/N of the bucket through HBM and lasts as
long as the xGMI links need.  With ``TOA_EMULATE_WORLD=N`` at world 1 the
trainer runs exactly rank 0's world-N step --

* the gradient buckets are "reduce-scattered" during backward and the
  weights "all-gathered" bucket by bucket before the next forward, at the
  same points and with the same per-bucket waits as the real path
  (``GradBucketer._launch``, ``ParamGather.launch`` / ``wait``);
* AdamW runs over rank 0's 1/N shards only (``FlatParams.shard_state``);

-- with each collective replaced by ``toa_emulate_xfer`` (csrc/hip/comm.hip)
on a high-priority side stream (bench.py runs RCCL's streams at high
priority too): (N-1)/N x bucket bytes, paced to ``TOA_EMULATE_GBPS`` GB/s
(default 350, an assumed RCCL bus bandwidth for 8 x MI355X over xGMI)
on ``TOA_EMULATE_CHANNELS`` workgroups (default 32).  ``TOA_EMULATE_AG=sdma``
moves the all-gathers' bytes with a copy engine instead
(``toa_emulate_copy_nocu``: no workgroup on any CU, unpaced), the stand-in
for pulling the peers' weight shards over xGMI by SDMA.  ``TOA_EMULATE_RS=sdma``
does the same for the reduce-scatters -- each rank pulls the peers' slices of
its own shard into a staging area by SDMA -- and moves the reduction into
the optimizer: before each bucket's AdamW the compute stream reads the N-1
staged slices once (:meth:`CommEmulator.fused_reduce`, the extra HBM read
an AdamW that sums N gradient slices would do).  Then no collective holds a
CU during backward; the reduce costs one read of (N-1)/N of the gradients.

The other ranks' shards are never updated (their "gathered" weights stay
as they were), so the loss is meaningless; the TIME is rank 0's.  Compare
against ``TOA_EMULATE_GBPS=0`` with ``TOA_EMULATE_BYTES=0`` (same step, no
traffic) to read what the overlap costs.  scripts/overlap_emulation.py runs
the policies side by side.

Reference parity: the reference's only collective is the payloads' per-step
gradient all-reduce (``examples/v1/distribution_strategy/keras-API/
multi_worker_strategy-with-keras.py:76-77, 117-120``); this
module measures what that step's collectives cost on MI355X at world 8.
"""
from __future__ import annotations

import os

import torch

from ..ops import _lib


def world_from_env() -> int:
    try:
        return max(1, int(os.environ.get("TOA_EMULATE_WORLD", "1")))
    except ValueError:
        return 1


class _Done:
    """Work-like handle: ``wait()`` makes the current stream wait for the
    emulated collective (as RCCL's Work.wait does), the host never blocks."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True


class CommEmulator:
    def __init__(self, world: int, device, gbps: float | None = None, channels: int | None = None,
                 move_bytes: bool | None = None):
        self.world = int(world)
        self.device = torch.device(device)
        self.gbps = float(os.environ.get("TOA_EMULATE_GBPS", "350")) if gbps is None else float(gbps)
        self.channels = int(os.environ.get("TOA_EMULATE_CHANNELS", "32")) if channels is None else int(channels)
        self.move = (os.environ.get("TOA_EMULATE_BYTES", "1") != "0") if move_bytes is None else bool(move_bytes)
        self.ag_mode = os.environ.get("TOA_EMULATE_AG", "ring")
        if self.ag_mode not in ("ring", "sdma"):
            raise ValueError(f"TOA_EMULATE_AG={self.ag_mode!r}: expected ring or sdma")
        self.rs_mode = os.environ.get("TOA_EMULATE_RS", "ring")
        if self.rs_mode not in ("ring", "sdma"):
            raise ValueError(f"TOA_EMULATE_RS={self.rs_mode!r}: expected ring or sdma")
        self.sum_out = None
        self.stream = torch.cuda.Stream(device=self.device, priority=-1) if self.device.type == "cuda" else None
        self.scratch = None
        self.calls = 0
        self.bytes = 0

    def _scratch(self, nbytes):
        if self.scratch is None or self.scratch.numel() < nbytes:
            self.scratch = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return self.scratch

    def collective(self, buf: torch.Tensor, kind: str = "reduce_scatter"):
        """Emulate one rank's share of a reduce-scatter / all-gather of
        `buf` (the whole bucket): (N-1)/N of its bytes, paced (an all-gather
        under TOA_EMULATE_AG=sdma: by a copy engine, unpaced)."""
        nbytes = buf.numel() * buf.element_size() * (self.world - 1) // self.world // 16 * 16
        self.calls += 1
        if self.stream is None:
            return _NullWork()
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)  # the bucket's producers are done
        with torch.cuda.stream(self.stream):
            if self.move and nbytes > 0:
                dst = self._scratch(nbytes)
                buf.record_stream(self.stream)
                if (self.ag_mode if kind == "all_gather" else self.rs_mode) == "sdma":
                    _lib.call("toa_emulate_copy_nocu", _lib.ptr(buf), _lib.ptr(dst), int(nbytes), _lib.stream(dst))
                else:
                    _lib.call("toa_emulate_xfer", _lib.ptr(buf), _lib.ptr(dst), int(nbytes), self.channels,
                              float(self.gbps), _lib.stream(dst))
                self.bytes += nbytes
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return _Done(ev)


    def fused_reduce(self, bucket: torch.Tensor):
        """TOA_EMULATE_RS=sdma: the optimizer's extra read of the N-1 staged
        gradient slices of this rank's shard of `bucket` (bf16), on the
        current (compute) stream, before the shard's AdamW."""
        if self.rs_mode != "sdma" or not self.move or self.stream is None:
            return
        n = bucket.numel() // self.world
        k = self.world - 1
        if n == 0 or k == 0:
            return
        staged = self._scratch(k * n * 2)[:k * n * 2].view(torch.bfloat16).view(k, n)
        if self.sum_out is None or self.sum_out.numel() < n:
            self.sum_out = torch.empty(n, dtype=torch.float32, device=self.device)
        torch.sum(staged, dim=0, dtype=torch.float32, out=self.sum_out[:n])


class _NullWork:
    def wait(self):
        return True
