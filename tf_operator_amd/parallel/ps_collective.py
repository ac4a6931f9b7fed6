"""Parameter servers on the GPU, over RCCL (BASELINE
config #2: TFJob PS=1 Worker=2 ResNet-50, each replica on one MI355X).

Reference semantics (``examples/v1/dist-mnist/dist_mnist.py:149-219``):
``replica_device_setter`` places the variables on ``/job:ps`` (the PS owns
the parameters and applies the optimizer); workers compute gradients and
fetch fresh parameters every step, either asynchronously (each push is
applied as it arrives) or through ``SyncReplicasOptimizer``
(``replicas_to_aggregate`` gradients are averaged into one update).

MI355X design -- the PS is a GPU rank in the same RCCL world as the
workers (world = W workers + P servers; PS p is rank W + p), holding the
fp32 master, Adam m and v of its contiguous shard of the flat parameter
vector (``FlatParams.shard_state``) and running the fused HIP AdamW kernel
on it (``FlatAdamW(owned=...)``).  No host round trip, no pickling: the
wire is xGMI.

* **sync** (SyncReplicas, replicas_to_aggregate = W): during the workers'
  backward each gradient bucket is ``reduce``-d (SUM) onto the PS owning
  it, bucket by bucket in flat order as the buckets complete -- the same
  backward overlap as the all-reduce path.  The PS applies one AdamW step
  with the mean and ``broadcast``-s its shard back, piece by piece (a
  bucket's part on that server) in FORWARD order.  The workers issue the
  matching broadcasts asynchronously at the end of their step and return;
  the next forward waits per bucket in module pre-hooks
  (:meth:`CollectivePS.wait_bucket`), so the pull of late layers runs under
  the compute of early ones (``TOA_PS_BLOCKING_PULL=1``: wait at the end of
  the step instead).  One collective group per PS (the W workers + that PS).
* **async**: every worker ``isend``-s its gradient shard to each PS and
  ``irecv``-s the parameters back; each PS polls one pending ``irecv`` per
  worker and applies every gradient as it arrives (stale by whatever the
  other workers pushed meanwhile), answering that worker with the
  parameters it just produced.

The TCP parameter server (:mod:`.ps`) stays as the CPU / numpy parity path.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from .flat import ALIGN, FlatParams


def ps_world_env():
    """(workers, servers, role, index) from the operator's TFJob env block.

    ``TOA_PS_HOSTS`` lists the servers and ``TOA_ROLE`` / ``TOA_REPLICA_INDEX``
    name this replica.  When the PS replicas request a GPU the operator puts
    them into the RCCL world itself (csrc/core/nodelocal.cc ``gpu_ps``):
    ``TOA_PS_IN_WORLD=1``, ``WORLD_SIZE`` = trainers + servers, PS p has
    ``RANK`` = trainers + p, and ``TOA_NUM_TRAINERS`` counts the trainers.
    Otherwise (a CPU PS: the gloo parity path) ``WORLD_SIZE`` counts only the
    trainers."""
    hosts = [h for h in os.environ.get("TOA_PS_HOSTS", "").split(",") if h]
    w = int(os.environ.get("WORLD_SIZE", "1"))
    if os.environ.get("TOA_PS_IN_WORLD") == "1":
        w = int(os.environ.get("TOA_NUM_TRAINERS", w - len(hosts)))
    role = os.environ.get("TOA_ROLE", "worker")
    idx = int(os.environ.get("TOA_REPLICA_INDEX", os.environ.get("RANK", "0")))
    return w, len(hosts), role, idx


def join_ps_world(workers: int, servers: int, role: str, index: int):
    """Make sure the process group about to be created spans workers AND
    servers (PS p = rank workers + p); call before ``Runtime.init_dist``.

    Operator-owned world (``TOA_PS_IN_WORLD=1``, GPU parameter servers): a
    consistency check only -- ``WORLD_SIZE`` / ``RANK`` must already be what
    the protocol needs, and a mismatch (an operator and a payload that
    disagree about the world) fails loudly instead of forming a wrong group.
    CPU PS replicas (``TOA_PS_IN_WORLD`` unset or 0) are outside the
    operator's world, so the payload extends it here for its gloo group."""
    want_world = workers + servers
    if os.environ.get("TOA_PS_IN_WORLD") == "1":
        world = int(os.environ.get("WORLD_SIZE", "-1"))
        rank = int(os.environ.get("RANK", "-1"))
        problems = []
        if world != want_world:
            problems.append(f"WORLD_SIZE={world}, expected {workers} trainers + {servers} servers = {want_world}")
        if role == "ps" and rank != workers + index:
            problems.append(f"PS {index} has RANK={rank}, expected {workers + index}")
        if role != "ps" and not 0 <= rank < workers:
            problems.append(f"{role} {index} has RANK={rank}, outside the trainers' ranks [0, {workers})")
        if problems:
            raise RuntimeError("parameter-server world from the operator is inconsistent: " + "; ".join(problems))
        return
    if role == "ps":
        os.environ["RANK"] = str(workers + index)
    os.environ["WORLD_SIZE"] = str(want_world)


def shard_ranges(numel: int, servers: int) -> list[tuple[int, int]]:
    """Contiguous, ALIGN-aligned [lo, hi) of the flat vector per server."""
    units = numel // ALIGN
    base, rem = divmod(units, servers)
    out, lo = [], 0
    for p in range(servers):
        hi = lo + (base + (1 if p < rem else 0)) * ALIGN
        out.append((lo, hi))
        lo = hi
    out[-1] = (out[-1][0], numel)
    return out


def flat_buckets(flat: FlatParams, bucket_mb: float) -> list[list[int]]:
    """[start, end, uses] backward-order gradient buckets of ~bucket_mb
    (flat order = reverse registration order = the order backward fills them)."""
    nb = max(1, int(bucket_mb * (1 << 20)) // flat.grad.element_size())
    out, cur = [], None
    for s in flat.segments:
        end = s.offset + -(-s.numel // ALIGN) * ALIGN
        if cur is None or cur[1] - cur[0] >= nb:
            cur = [s.offset, end, 0]
            out.append(cur)
        cur[1] = end
        cur[2] += getattr(s.param, "_toa_uses", 1)
    out[-1][1] = flat.numel
    return out


def bucket_pieces(buckets, ranges) -> list[tuple[int, int, int, int]]:
    """(bucket, server, lo, hi): each bucket split at the server shard bounds."""
    out = []
    for b, (a, e, _) in enumerate(buckets):
        for p, (lo, hi) in enumerate(ranges):
            a2, e2 = max(a, lo), min(e, hi)
            if a2 < e2:
                out.append((b, p, a2, e2))
    return out


class CollectivePS:
    """One per process (worker or server).  ``flat`` must have the same
    layout on every rank (same model code)."""

    def __init__(self, flat: FlatParams, workers: int, servers: int, mode: str = "sync", lr: float = 1e-3,
                 betas=(0.9, 0.999), eps=1e-8, weight_decay: float = 0.0, bucket_mb: float = 64.0):
        from ..ops.optim import FlatAdamW

        if mode not in ("sync", "async"):
            raise ValueError(f"mode {mode!r}")
        self.flat, self.W, self.P, self.mode = flat, int(workers), int(servers), mode
        self.rank = dist.get_rank()
        if dist.get_world_size() != self.W + self.P:
            raise RuntimeError(f"process group has {dist.get_world_size()} ranks, expected {self.W}+{self.P}")
        self.is_ps = self.rank >= self.W
        self.ranges = shard_ranges(flat.numel, self.P)
        # every rank creates every group, in the same order (torch.distributed rule)
        self.groups = [dist.new_group(list(range(self.W)) + [self.W + p]) for p in range(self.P)]
        self.buckets = flat_buckets(flat, bucket_mb)
        self.pieces = bucket_pieces(self.buckets, self.ranges)
        # the parameter pull, piece by piece in forward order (flat order is
        # backward order: the forward needs the last bucket first)
        self.pull_order = sorted(self.pieces, key=lambda t: (-t[0], t[1]))
        self.pulls = {}
        self.blocking_pull = os.environ.get("TOA_PS_BLOCKING_PULL", "0") == "1"
        # everyone starts from worker 0's weights
        dist.broadcast(flat.param, 0)
        self.updates = 0
        if self.is_ps:
            self.p = self.rank - self.W
            lo, hi = self.ranges[self.p]
            flat.shard_state([(lo, hi)])
            flat.master_from_param()
            self.opt = FlatAdamW(flat, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, max_grad_norm=0.0,
                                 owned=[(lo, hi)])
            if mode == "async":
                self.rbuf = [torch.zeros(hi - lo, device=flat.device, dtype=flat.grad.dtype) for _ in range(self.W)]
        else:
            # gradient buckets are reduced as backward completes them, strictly
            # in flat order, so every server sees its reduces in one fixed order
            for s in flat.segments:
                s.param._toa_bucket = next(i for i, (a, e, _) in enumerate(self.buckets) if a <= s.offset < e)
                if mode == "sync":
                    s.param._toa_ready = self._ready
            self._reset()

    # ------------------------------------------------------------------ worker
    def _reset(self):
        self.pending = [b[2] for b in self.buckets]
        self.ready = [False] * len(self.buckets)
        self.next_bucket = 0
        self.works = []

    def _ready(self, param):
        b = param._toa_bucket
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self.ready[b] = True
            while self.next_bucket < len(self.buckets) and self.ready[self.next_bucket]:
                self._launch(self.next_bucket)
                self.next_bucket += 1

    def _launch(self, b):
        g = self.flat.grad
        for (bb, p, lo, hi) in self.pieces:
            if bb == b:
                self.works.append(dist.reduce(g[lo:hi], self.W + p, op=dist.ReduceOp.SUM, group=self.groups[p],
                                              async_op=True))

    @torch.no_grad()
    def worker_step(self):
        """After backward: the gradients go to the servers, the servers'
        new parameters come back into ``flat.param``."""
        f = self.flat
        if self.mode == "sync":
            # pulls of the previous step that no forward hook waited for
            # (buckets whose modules did not run): the broadcasts below write
            # the same parameters
            self.wait_params()
            while self.next_bucket < len(self.buckets):  # buckets whose params got no gradient
                self._launch(self.next_bucket)
                self.next_bucket += 1
            for w in self.works:  # the next backward overwrites these gradients
                w.wait()
            self._reset()
            for (b, p, lo, hi) in self.pull_order:
                self.pulls.setdefault(b, []).append(
                    dist.broadcast(f.param[lo:hi], self.W + p, group=self.groups[p], async_op=True))
            if self.blocking_pull:
                self.wait_params()
            self.updates += 1
            return
        else:
            works = []
            for p, (lo, hi) in enumerate(self.ranges):
                works.append(dist.isend(f.grad[lo:hi].contiguous(), self.W + p))
                works.append(dist.irecv(f.param[lo:hi], self.W + p))
            for w in works:
                w.wait()
        self.updates += 1
        f.params_changed()

    def wait_bucket(self, b: int):
        """Block until bucket b's fresh parameters have arrived (sync mode;
        RCCL: the current stream waits, the host does not)."""
        works = self.pulls.pop(b, None)
        if not works:
            return
        for w in works:
            w.wait()
        # per bucket: a cache keyed on the parameters (e.g. a bf16 copy) must
        # not wait for buckets no forward touches
        self.flat.params_changed()

    def wait_params(self):
        for b in list(self.pulls):
            self.wait_bucket(b)

    # ------------------------------------------------------------------ server
    @torch.no_grad()
    def serve(self, steps: int):
        """Apply `steps` updates per worker (sync: `steps` aggregated
        updates; async: steps x W individual ones), then return."""
        if self.mode == "sync":
            self._serve_sync(steps)
        else:
            self._serve_async(steps)

    def _serve_sync(self, steps):
        f, p = self.flat, self.p
        lo, hi = self.ranges[p]
        mine = [(a, b) for (_, pp, a, b) in self.pieces if pp == p]
        for _ in range(steps):
            f.grad[lo:hi].zero_()  # the server's own contribution to the SUM
            works = [dist.reduce(f.grad[a:b], self.rank, op=dist.ReduceOp.SUM, group=self.groups[p], async_op=True)
                     for a, b in mine]
            for w in works:
                w.wait()
            self.opt.step(grad_scale=1.0 / self.W)  # SyncReplicas: the mean of W gradients
            # the same pieces, in the same (forward) order as the workers' pulls
            outs = [dist.broadcast(f.param[a:bb], self.rank, group=self.groups[p], async_op=True)
                    for (_, pp, a, bb) in self.pull_order if pp == p]
            for w in outs:
                w.wait()
            self.updates += 1

    def _serve_async(self, steps):
        f = self.flat
        lo, hi = self.ranges[self.p]

        def apply(w, buf):
            f.grad[lo:hi].copy_(buf)
            self.opt.step(grad_scale=1.0)  # async PS: every push is its own update
            self.updates += 1

        if dist.get_backend() == "gloo":
            # gloo receives from ANY source: serve pushes in arrival order
            for _ in range(steps * self.W):
                w = dist.recv(self.rbuf[0])
                apply(w, self.rbuf[0])
                dist.send(f.param[lo:hi], w)
            return
        # RCCL has no any-source receive: one pending irecv per worker, polled
        recvs = [dist.irecv(self.rbuf[w], w) for w in range(self.W)]
        left = [steps] * self.W
        while any(left):
            progressed = False
            for w in range(self.W):
                if not left[w] or not recvs[w].is_completed():
                    continue
                recvs[w].wait()  # orders the copy below after the receive on this stream
                apply(w, self.rbuf[w])
                dist.isend(f.param[lo:hi], w).wait()  # the next update may not overwrite an in-flight send
                left[w] -= 1
                progressed = True
                if left[w]:
                    recvs[w] = dist.irecv(self.rbuf[w], w)
            if not progressed:
                time.sleep(20e-6)
