"""Copy-engine all-gather of the ZeRO-1 weights (verdict r4 item 5).

With the optimizer sharded (parallel/zero.py), every rank updates 1/N of
each gradient bucket and the bf16 weights are then all-gathered bucket by
bucket under the next forward.  RCCL's ring all-gather does that with a
kernel holding workgroups on the CUs the forward's GEMMs want; on one
node the same bytes can be PULLED by the copy engines (SDMA) instead:
every rank maps its peers' flat weight buffers once (IPC), and per bucket

  owner (compute stream):  AdamW on its shard -> publish epoch in its flag
                           word for the bucket (system-scope release)
  puller (copy stream):    wait until every peer published the epoch
                           (one wave, bounded spin) -> N-1 SDMA copies of
                           the peers' shards into its own buffer -> event
  next forward:            the compute stream waits the bucket's event

No workgroup of a collective sits on a CU during the forward.  The reverse
hazard (an owner overwriting its shard of step t+1 while a peer still pulls
step t's) cannot occur: the owner updates a shard only after that bucket's
reduce-scatter of step t+1, which every peer enters after its forward of
step t+1 consumed the pulled bucket.

Emulated on one GPU first (parallel/emulate.py ``TOA_EMULATE_AG=sdma``,
``profiles/r5_overlap/``).  Enabled with ``TOA_ZERO_AG=sdma`` for a ZeRO-1
job whose ranks share one node (``LOCAL_WORLD_SIZE`` == world, the
operator's node-local layout); RCCL's all-gather stays the default until
an 8-GPU run measures it.  Transports:

* ``GpuIpcTransport``: the flat weight buffers exported with torch's CUDA
  IPC (DMA-BUF on MI355X), fine-grained flag arrays from csrc/hip/comm.hip
  (``toa_ipc_alloc``), ``toa_flag_publish`` / ``toa_flags_wait`` /
  ``toa_copy_nocu``.  tests/test_comm_gpu.py runs two processes on one GPU.
* ``ShmTransport``: the same protocol on the CPU over file-backed shared
  memory (/dev/shm), so gloo tests check the pulled bytes against
  ``dist.all_gather_into_tensor`` bit for bit (tests/test_pull_gather.py).

Failure semantics.  A peer that never publishes costs its waiting ranks one
bounded spin (``timeout_ms``, once per run: a peer already marked lost is
not waited for again, csrc/hip/comm.hip ``flags_wait_kernel``).  The wait
only sets the peer's error bit; the copies behind it still run, so from
that bucket on the pulled weights (or gradient slices) are STALE and the
model is poisoned until the job restarts.  ``poll()`` surfaces the bit one
step later as a RuntimeError (the replica exits non-zero, the operator
restarts it), and ``check()`` -- run by every checkpoint save, train/llm.py
``trainer_state`` -- refuses to persist a poisoned state, so a restart
resumes from the last good checkpoint.  Teardown: ``LlamaTrainer.close``
(registered at exit) drains this rank's pulls, synchronises, barriers the
group and only then unmaps / frees, so no rank frees exported memory a
slower peer is still pulling.

Reference parity: the payloads' gradient exchange
(``examples/v1/distribution_strategy/keras-API/multi_worker_strategy-with-keras.py:76-77``;
SURVEY P3 / K16) -- the sharded step's weight half, moved without CUs.
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np
import torch
import torch.distributed as dist


def mode_from_env() -> str:
    m = os.environ.get("TOA_ZERO_AG", "rccl")
    if m not in ("rccl", "sdma"):
        raise ValueError(f"TOA_ZERO_AG={m!r}: expected rccl or sdma")
    return m


def rs_mode_from_env() -> str:
    m = os.environ.get("TOA_ZERO_RS", "rccl")
    if m not in ("rccl", "sdma"):
        raise ValueError(f"TOA_ZERO_RS={m!r}: expected rccl or sdma")
    return m


def timeout_ms_from_env() -> int:
    """How long a puller waits for a peer's epoch before marking it lost
    (``TOA_PULL_TIMEOUT_MS``, default 60 s: a peer writing a checkpoint or
    compiling on its first step is slow, not lost)."""
    v = int(os.environ.get("TOA_PULL_TIMEOUT_MS", "60000"))
    if v <= 0:
        raise ValueError(f"TOA_PULL_TIMEOUT_MS={v}: must be > 0")
    return v


class _Event:
    """Work-like handle: ``wait()`` makes the current stream wait (GPU) or
    is a no-op (CPU: the pull already ran synchronously)."""

    def __init__(self, ev=None):
        self.ev = ev

    def wait(self):
        if self.ev is not None:
            torch.cuda.current_stream().wait_event(self.ev)
        return True


class ShmTransport:
    """CPU transport over /dev/shm files: each rank's flat buffer (``buf``,
    file-backed) and flag array live in files its peers map read-only;
    waits poll the flag words."""

    def __init__(self, tag: str, rank: int, world: int, numel: int, dtype, nflags: int, timeout_s: float = 60.0):
        self.rank, self.world, self.timeout = rank, world, timeout_s
        self.tag = tag
        itemsize = torch.empty(0, dtype=dtype).element_size()
        self.dtype = dtype
        self.paths = [f"/dev/shm/toa_pull_{tag}_{r}" for r in range(world)]
        self.fpaths = [p + "_flags" for p in self.paths]
        self._np_dtype = {2: np.uint16, 4: np.uint32}[itemsize]
        mine = np.memmap(self.paths[rank], dtype=self._np_dtype, mode="w+", shape=(numel,))
        flags = np.memmap(self.fpaths[rank], dtype=np.uint32, mode="w+", shape=(nflags,))
        flags[:] = 0
        flags.flush()
        self.buf = torch.from_numpy(mine).view(dtype)
        self.my_flags = flags
        self.numel, self.nflags = numel, nflags
        dist.barrier()
        self.peer_bufs = [None if r == rank else torch.from_numpy(
            np.memmap(self.paths[r], dtype=self._np_dtype, mode="r", shape=(numel,))).view(dtype)
            for r in range(world)]
        self.peer_flags = [None if r == rank else np.memmap(self.fpaths[r], dtype=np.uint32, mode="r",
                                                           shape=(nflags,)) for r in range(world)]

    def publish(self, idx: int, epoch: int):
        self.my_flags[idx] = epoch
        self.my_flags.flush()

    def pull(self, idx: int, epoch: int, pieces, dst=None):
        """pieces: [(peer, lo, hi)] element ranges of the flat buffer, copied
        to the same range of this rank's buffer -- or [(peer, lo, hi, off)]
        copied to dst[off:off + hi - lo] (the reduce-scatter's staging)."""
        t0 = time.monotonic()
        for r in range(self.world):
            if r == self.rank:
                continue
            while int(self.peer_flags[r][idx]) < epoch:
                if time.monotonic() - t0 > self.timeout:
                    raise RuntimeError(f"pull all-gather: rank {r} never published bucket {idx} epoch {epoch}")
                time.sleep(0.0005)
        for r, lo, hi, *off in pieces:
            o = off[0] if off else lo
            (self.buf if dst is None else dst)[o:o + hi - lo].copy_(self.peer_bufs[r][lo:hi])
        return _Event()

    def close(self):
        dist.barrier()
        for p in (self.paths[self.rank], self.fpaths[self.rank]):
            try:
                os.unlink(p)
            except FileNotFoundError:
                pass


class GpuIpcTransport:
    """GPU transport: peers' flat buffers through torch's CUDA IPC, flag
    arrays through toa_ipc_alloc handles, waits / publishes / copies by the
    HIP entry points of csrc/hip/comm.hip on a high-priority copy stream."""

    def __init__(self, buf: torch.Tensor, rank: int, world: int, nflags: int, group=None, timeout_ms: int = 60000,
                 what: str = "all-gather"):
        from torch.multiprocessing.reductions import reduce_tensor

        from ..ops import _lib

        if world > 8:
            raise ValueError(f"the copy-engine {what} is for one node (<= 8 ranks)")
        self.what = what
        self._lib = _lib
        self.rank, self.world, self.group = rank, world, group
        self.buf, self.nflags, self.timeout_ms = buf, nflags, int(timeout_ms)
        L = _lib.lib()
        for name, argt in (("toa_ipc_alloc", [ctypes.c_int64, ctypes.c_void_p]),
                           ("toa_ipc_get_handle", [ctypes.c_void_p, ctypes.c_void_p]),
                           ("toa_ipc_open_handle", [ctypes.c_void_p, ctypes.c_void_p]),
                           ("toa_ipc_close_handle", [ctypes.c_void_p]), ("toa_ipc_free", [ctypes.c_void_p]),
                           ("toa_ipc_handle_size", [])):
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = ctypes.c_int
        self._L = L
        hsz = L.toa_ipc_handle_size()
        err = None
        own = ctypes.c_void_p()
        h = (ctypes.c_char * hsz)()
        try:
            if L.toa_ipc_alloc(4 * max(1, nflags), ctypes.byref(own)) != 0:
                raise RuntimeError("flag alloc failed")
            if L.toa_ipc_get_handle(own, h) != 0:
                raise RuntimeError("flag handle failed")
            shared = reduce_tensor(buf)
        except Exception as e:  # noqa: BLE001 -- exchanged below, every rank raises together
            err, shared = f"rank {rank}: {e}", None
        self._own = own if own.value else None
        infos = [None] * world
        dist.all_gather_object(infos, {"err": err, "flags": bytes(h), "buf": shared}, group=group)
        errs = [i["err"] for i in infos if i["err"]]
        self.flags = (ctypes.c_void_p * world)()
        self._opened, self.peer_bufs = [], [None] * world
        if not errs:
            try:
                for r in range(world):
                    if r == rank:
                        self.flags[r] = self._own
                        continue
                    q = ctypes.c_void_p()
                    hh = (ctypes.c_char * hsz).from_buffer_copy(infos[r]["flags"])
                    if L.toa_ipc_open_handle(hh, ctypes.byref(q)) != 0:
                        raise RuntimeError(f"open rank {r} flags")
                    self._opened.append(q)
                    self.flags[r] = q
                    fn, args = infos[r]["buf"]
                    self.peer_bufs[r] = fn(*args)
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                err = f"rank {rank}: {e}"
        ok = torch.tensor([0 if (errs or err) else 1], device=buf.device, dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        if int(ok.item()) != 1:
            self.close()
            raise RuntimeError(f"copy-engine {what} setup failed: " + "; ".join(errs + ([err] if err else [])
                                                                            or ["on a peer rank"]))
        self.err = torch.zeros(1, device=buf.device, dtype=torch.int32)
        self.stream = torch.cuda.Stream(device=buf.device, priority=-1)

    def publish(self, idx: int, epoch: int):
        L = self._lib
        L.call("toa_flag_publish", ctypes.c_void_p(self._own.value + 4 * idx), epoch, L.stream(self.buf))

    def pull(self, idx: int, epoch: int, pieces, dst=None):
        """As ShmTransport.pull, on the copy stream (SDMA copies)."""
        L = self._lib
        cur = torch.cuda.current_stream(self.buf.device)
        self.stream.wait_stream(cur)   # this rank's readers of the old weights are done
        st = ctypes.c_void_p(self.stream.cuda_stream)
        L.call("toa_flags_wait", self.flags, idx, self.rank, self.world, epoch, L.ptr(self.err), self.timeout_ms, st)
        es = self.buf.element_size()
        out = self.buf if dst is None else dst
        for r, lo, hi, *off in pieces:
            src = self.peer_bufs[r].data_ptr() + es * lo
            o = off[0] if off else lo
            L.call("toa_copy_nocu", ctypes.c_void_p(src), ctypes.c_void_p(out.data_ptr() + es * o),
                   es * (hi - lo), st)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return _Event(ev)

    def poll(self):
        """Non-blocking error check once per step: the device error word is
        copied to pinned host memory behind this step's pulls and the copy
        queued a step earlier is read (an event query, no host sync)."""
        if not hasattr(self, "_host_err"):
            self._host_err = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._err_ev = None
        if self._err_ev is not None and self._err_ev.query():
            e = int(self._host_err[0])
            self._err_ev = None
            if e:
                self._raise(e)
        if self._err_ev is None:
            with torch.cuda.stream(self.stream):
                self._host_err.copy_(self.err, non_blocking=True)
                self._err_ev = torch.cuda.Event()
                self._err_ev.record(self.stream)

    def _raise(self, e: int):
        raise RuntimeError(f"copy-engine {self.what}: ranks {[r for r in range(8) if e >> r & 1]} never "
                           "published their shards (peer lost or stalled); the result is stale")

    def check(self):
        e = int(self.err.item())
        if e:
            self._raise(e)

    def close(self):
        torch.cuda.synchronize()
        self.peer_bufs = [None] * self.world
        for q in self._opened:
            self._L.toa_ipc_close_handle(q)
        if self._own is not None:
            self._L.toa_ipc_free(self._own)
        self._opened, self._own = [], None


class PullGather:
    """The ZeRO-1 weight all-gather by peer pulls: drop-in for
    :func:`zero.all_gather_` per bucket (:class:`zero.ParamGather` with
    ``TOA_ZERO_AG=sdma``).  ``ranges``: the buckets' flat [lo, hi); each is
    split into `world` equal shards, shard r owned by rank r."""

    def __init__(self, transport, ranges, rank: int, world: int):
        self.t = transport
        self.ranges = [tuple(r) for r in ranges]
        self.rank, self.world = rank, world
        self.epoch = 0
        for lo, hi in self.ranges:
            if (hi - lo) % world:
                raise ValueError("bucket not divisible into world shards")

    def new_step(self):
        """Every rank calls this once per optimizer step (same count on all)."""
        self.epoch += 1

    def pieces(self, b):
        lo, hi = self.ranges[b]
        n = (hi - lo) // self.world
        return [(r, lo + r * n, lo + (r + 1) * n) for r in range(self.world) if r != self.rank]

    def launch_one(self, b):
        """Bucket b's own shard is updated (on the current stream): publish
        it and pull the peers'.  Returns a Work-like handle."""
        self.t.publish(b, self.epoch)
        return self.t.pull(b, self.epoch, self.pieces(b))

    def check(self):
        if hasattr(self.t, "check"):
            self.t.check()

    def poll(self):
        if hasattr(self.t, "poll"):
            self.t.poll()

    def close(self):
        self.t.close()


class PullReduceScatter:
    """The ZeRO-1 gradient reduce-scatter by peer pulls (``TOA_ZERO_RS=sdma``;
    the traffic was priced on one GPU first, ``TOA_EMULATE_RS=sdma``,
    ``profiles/r5_overlap2/``).  Per bucket, in backward order:

      every rank (compute stream):  bucket b's gradients are final ->
                                    publish the epoch in its flag word
      owner of shard r (copy stream): wait for every peer's epoch -> N-1
                                    SDMA copies of the peers' slices of
                                    shard r into a staging area -> event
      owner (compute stream, before the update):  wait the event ->
                                    shard r += the staged slices, summed in
                                    fp32 and rounded once (``reduce``)

    No reduction workgroup holds CUs while the backward runs; the sum is one
    HBM-bound pass over 1/N of the bucket per peer.  A peer cannot overwrite
    its bucket-b gradients (step t+1's backward) before the owner pulled
    them: the owner publishes its updated shard of b only after this pull,
    and the peer's next backward of b follows its forward's wait for that
    shard (the weight all-gather, by RCCL or by pulls).

    ``transport``: ShmTransport / GpuIpcTransport over the flat GRADIENT
    buffer (its own flag words); ``ranges``: the buckets' flat [lo, hi)."""

    def __init__(self, transport, ranges, rank: int, world: int):
        self.t = transport
        self.ranges = [tuple(r) for r in ranges]
        self.rank, self.world = rank, world
        self.epoch = 1
        self.stage_off, off = [], 0
        for lo, hi in self.ranges:
            if (hi - lo) % world:
                raise ValueError("bucket not divisible into world shards")
            self.stage_off.append(off)
            off += (world - 1) * ((hi - lo) // world)
        buf = transport.buf
        self.staging = torch.empty(max(off, 1), dtype=buf.dtype, device=buf.device)

    def new_step(self):
        """Every rank calls this once per optimizer step (same count on all),
        after the step's last bucket was launched."""
        self.epoch += 1

    def shard(self, b):
        lo, hi = self.ranges[b]
        n = (hi - lo) // self.world
        return lo + self.rank * n, lo + (self.rank + 1) * n

    def pieces(self, b):
        """The peers' slices of this rank's shard -> consecutive staging slots
        (peers in rank order)."""
        lo, hi = self.ranges[b]
        n = (hi - lo) // self.world
        s = lo + self.rank * n
        peers = [r for r in range(self.world) if r != self.rank]
        return [(r, s, s + n, self.stage_off[b] + k * n) for k, r in enumerate(peers)]

    def launch_one(self, b):
        """Bucket b's gradients are final on the current stream: publish
        them and pull the peers' slices of this rank's shard.  Returns a
        Work-like handle (the current stream waits the pulls)."""
        self.t.publish(b, self.epoch)
        return self.t.pull(b, self.epoch, self.pieces(b), dst=self.staging)

    def reduce(self, b):
        """Shard b += the staged slices (after the handle's wait)."""
        s, e = self.shard(b)
        n, k = e - s, self.world - 1
        if n == 0 or k == 0:
            return
        buf = self.t.buf
        st = self.staging[self.stage_off[b]:self.stage_off[b] + k * n]
        if buf.is_cuda:
            from ..ops import _lib

            if buf.dtype != torch.bfloat16:
                raise ValueError("the copy-engine reduce-scatter sums bf16 gradients")
            _lib.call("toa_sum_slices_bf16", ctypes.c_void_p(buf.data_ptr() + 2 * s), _lib.ptr(st), k, n, n,
                      _lib.stream(buf))
            return
        acc = buf[s:e].float()
        for j in range(k):
            acc += st[j * n:(j + 1) * n].float()
        buf[s:e].copy_(acc.to(buf.dtype))

    def check(self):
        if hasattr(self.t, "check"):
            self.t.check()

    def poll(self):
        if hasattr(self.t, "poll"):
            self.t.poll()

    def close(self):
        self.t.close()
