"""Fused AdamW / SGD over flat buffers (HIP kernels in csrc/hip/optim.hip).

One streaming launch per contiguous weight-decay run of the flat buffer;
the gradient clip coefficient is computed on the device from the global
squared norm (``toa_sumsq``), so ``step()`` never synchronises with the host.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib
from .wt import transpose_into


SUMSQ_WS = 32768  # floats of toa_sumsq's partials workspace (its grid cap)


def grad_norm_sq(flat_grad: torch.Tensor, workspace=None, out=None):
    """Squared L2 norm of a flat gradient (fp32 0-d device tensor)."""
    out = torch.zeros(1, device=flat_grad.device, dtype=torch.float32) if out is None else out
    if _lib.use_hip(flat_grad):
        ws = torch.empty(SUMSQ_WS, device=flat_grad.device, dtype=torch.float32) if workspace is None else workspace
        _lib.call("toa_sumsq", _lib.ptr(flat_grad), flat_grad.numel(), int(flat_grad.dtype == torch.bfloat16),
                  _lib.ptr(ws), _lib.ptr(out), 0, _lib.stream(flat_grad))
    else:
        out.copy_(flat_grad.float().pow(2).sum().reshape(1))
    return out


def adamw_reference(master, grad, m, v, *, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0,
                    norm_sq=None, max_norm=0.0):
    g = grad.float() * grad_scale
    if norm_sq is not None and max_norm > 0:
        nrm = float(norm_sq.sqrt()) * grad_scale
        g = g * min(1.0, max_norm / (nrm + 1e-6))
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = v.sqrt() / math.sqrt(bc2) + eps
    master.add_(-lr * (m / bc1) / denom - lr * weight_decay * master)


_MASKED = []   # (ExternalStream, handle): kept for the process's life


def masked_stream(n: int, mode: int = 1, device=None):
    """A torch stream over a HIP stream whose kernels may use only `n` CUs
    (csrc/hip/optim.hip toa_stream_create_cu_mask; mode 1 spreads them over
    the mask, mode 0 takes the first n)."""
    h = ctypes.c_void_p()
    _lib.call("toa_stream_create_cu_mask", int(mode), int(n), ctypes.byref(h))
    st = torch.cuda.ExternalStream(h.value, device=device)
    _MASKED.append((st, h))
    return st


class FlatAdamW:
    """AdamW over a :class:`tf_operator_amd.parallel.flat.FlatParams`.

    overlap=True (GPU): after the global grad norm, the update runs on a side
    stream bucket by bucket in FORWARD order (zeroing each gradient slice as
    it reads it when fuse_zero_grad; with fresh gradients nothing needs
    zeroing), and records one event per bucket.  The next step's forward waits per bucket (wait_bucket, called
    from module pre-hooks), so the memory-bound update of late layers runs
    under the compute-bound GEMMs of early ones; backward waits for all of it
    (wait_all) before writing gradients.  Measured on Llama-3-8B it gains
    nothing (round 2: 1100 vs 1098 ms/step; round 6 with the assembly GEMMs:
    -1.6 +- 0.6 and +5.2 +- 4.5 ms in two A/Bs, and slower on a CU-masked
    stream, TOA_OPT_CUS; docs/kernels.md): the GEMMs hold every CU, so the
    update only slots in between them; it stays opt-in (TOA_OPT_OVERLAP=1).

    fuse_zero_grad=True: the update zeroes the gradient as it reads it
    (``grads_zeroed`` tells the caller to skip its own zero_grad pass).

    post_update(lo, hi): called on the update's stream after the bf16
    weights of flat range [lo, hi) are written (per bucket in overlap mode,
    once for the whole buffer otherwise) -- derived weight copies (ops.wt)
    refresh there.

    owned=[(lo, hi), ...] (sharded data parallelism, parallel/zero.py): only
    those flat ranges are updated; the clipping norm is the all-reduced sum
    (over `group`) of the owned ranges' squared norms.  The caller zeroes
    the gradients (the not-owned ranges hold this rank's unreduced ones)."""

    def __init__(self, flat, lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0,
                 overlap=False, buckets=None, fuse_zero_grad=False, post_update=None, owned=None, group=None,
                 device_step=False):
        self.post_update = post_update
        self.sumsq = None   # an ops.gemm.SumsqSession (set by the trainer): the clipping norm from kernel partials
        # fused_wt: an ops.wt.TransposedWeights whose 2-D weights (R, C multiples of 128) the update writes
        # together with their W^T copies (toa_adamw_wt) instead of refreshing them afterwards (set by the
        # trainer for an unsharded update; post_update then refreshes only the others)
        self.fused_wt = None
        # device_step: the step count lives in device memory and is advanced
        # by a kernel, so a captured HIP graph of the whole training step
        # replays with fresh bias corrections (train/simple.py graph mode)
        self.device_step = (bool(device_step) and flat.device.type == "cuda" and _lib.available()
                            and _lib.has("toa_adamw_flat_dstep"))
        self._dstep = torch.zeros(1, device=flat.device, dtype=torch.int32) if self.device_step else None
        self.owned = None if owned is None else [tuple(r) for r in owned]
        self.group = group
        if self.owned is not None and overlap:
            raise ValueError("overlap mode and a sharded update are exclusive")
        self.flat = flat
        self.lr = lr
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        if flat.exp_avg is None:  # sized to the fp32 state this rank holds (all, or its ZeRO shards)
            flat.exp_avg = torch.zeros(flat.state_numel, device=flat.device, dtype=torch.float32)
            flat.exp_avg_sq = torch.zeros(flat.state_numel, device=flat.device, dtype=torch.float32)
        # without weight decay the decay split is moot: one launch over the whole buffer
        self.runs = flat.decay_runs() if weight_decay else [[0, flat.numel, False]]
        self._norm = torch.zeros(1, device=flat.device, dtype=torch.float32)
        self._ws = torch.empty(SUMSQ_WS, device=flat.device, dtype=torch.float32)
        self.last_norm_sq = self._norm
        self.overlap = bool(overlap) and flat.device.type == "cuda" and _lib.available()
        # zero each gradient slice as the update reads it (the caller then skips zero_grad)
        self.fuse_zero_grad = bool(fuse_zero_grad)
        self.grads_zeroed = False  # the last step() zeroed the gradients itself
        if self.overlap:
            # TOA_OPT_CUS=n[:mode]: the update's stream may use only n CUs
            # (masked_stream), so it runs beside the GEMMs instead of taking
            # every CU a finished GEMM workgroup frees
            cus = os.environ.get("TOA_OPT_CUS", "")
            self.side = (masked_stream(*[int(x) for x in cus.split(":")], device=flat.device) if cus
                         else torch.cuda.Stream(device=flat.device))
            ranges = [(b[0], b[1]) for b in buckets] if buckets else [(0, flat.numel)]
            # flat order is backward order: the forward needs the last bucket first
            self.order = list(range(len(ranges)))[::-1]
            self.ranges = ranges
            self.events = [None] * len(ranges)
            self.waited = [True] * len(ranges)
            self.done = None

    def _launch(self, a, b, decay, lr, grad_scale, clip, zero, stream):
        f = self.flat
        gflags = int(f.grad.dtype == torch.bfloat16) | (2 if zero else 0)
        pp = f.param.data_ptr() + 2 * a if f.param.dtype == torch.bfloat16 else None
        fn, step = ("toa_adamw_flat_dstep", _lib.ptr(self._dstep)) if self.device_step else ("toa_adamw_flat",
                                                                                             self.step_count)
        si = f.state_index(a)  # compact fp32 state (ZeRO shards) or == a
        if f.state_index(b - 1) != si + (b - a - 1):
            raise ValueError(f"update run [{a}, {b}) crosses fp32 state ranges")
        _lib.call(fn, f.master.data_ptr() + 4 * si, pp, f.grad.data_ptr() + f.grad.element_size() * a,
                  gflags, f.exp_avg.data_ptr() + 4 * si, f.exp_avg_sq.data_ptr() + 4 * si, b - a, float(lr),
                  float(self.beta1), float(self.beta2), float(self.eps),
                  float(self.weight_decay if decay else 0.0), step, float(grad_scale),
                  _lib.ptr(self._norm) if clip else None, float(self.max_grad_norm or 0.0), stream)

    def _fused_items(self) -> dict:
        """{(lo, hi): (lo, hi, param, view)} of the W^T copies the update can
        write itself: unsharded, HIP, bf16 gradient, no device step count, R
        and C multiples of 128, the weight in one state range."""
        wt = self.fused_wt
        f = self.flat
        if (wt is None or self.owned is not None or self.device_step or f.grad.dtype != torch.bfloat16
                or not _lib.has("toa_adamw_wt")):
            return {}
        out = {}
        for a, b, p, view in wt.items:
            R, C = p.shape
            if R % 128 == 0 and C % 128 == 0 and f.state_index(b - 1) == f.state_index(a) + (b - a - 1):
                out[(a, b)] = (a, b, p, view)
        return out

    def _launch_wt(self, item, decay, lr, grad_scale, clip, stream):
        a, b, p, view = item
        f = self.flat
        si = f.state_index(a)
        R, C = p.shape
        _lib.call("toa_adamw_wt", f.master.data_ptr() + 4 * si, f.param.data_ptr() + 2 * a,
                  f.grad.data_ptr() + 2 * a, int(bool(self.fuse_zero_grad)), f.exp_avg.data_ptr() + 4 * si,
                  f.exp_avg_sq.data_ptr() + 4 * si, _lib.ptr(view), view.stride(0), R, C, float(lr),
                  float(self.beta1), float(self.beta2), float(self.eps), float(self.weight_decay if decay else 0.0),
                  self.step_count, float(grad_scale), _lib.ptr(self._norm) if clip else None,
                  float(self.max_grad_norm or 0.0), stream)

    def _work_runs(self):
        """(a, b, decay) runs this rank updates."""
        if self.owned is None:
            yield from self.runs
            return
        for lo, hi in self.owned:
            for a, b, decay in self.runs:
                a2, b2 = max(a, lo), min(b, hi)
                if a2 < b2:
                    yield a2, b2, decay

    def _norm_sq(self):
        f = self.flat
        if self.owned is None:
            if self.sumsq is not None:   # partials from the weight-gradient kernels (ops/gemm.SumsqSession)
                self.sumsq.norm_sq(self._norm, self._ws)
                return
            grad_norm_sq(f.grad, self._ws, self._norm)
            return
        import torch.distributed as dist

        if _lib.use_hip(f.grad):
            for i, (lo, hi) in enumerate(self.owned):
                g = f.grad[lo:hi]
                _lib.call("toa_sumsq", _lib.ptr(g), g.numel(), int(g.dtype == torch.bfloat16), _lib.ptr(self._ws),
                          _lib.ptr(self._norm), int(i > 0), _lib.stream(g))
        else:
            self._norm.copy_(sum(f.grad[lo:hi].float().pow(2).sum() for lo, hi in self.owned).reshape(1))
        if dist.is_initialized():
            dist.all_reduce(self._norm, op=dist.ReduceOp.SUM, group=self.group)

    def wait_bucket(self, b):
        """Make the current stream wait until bucket b's parameters are updated."""
        if self.overlap and not self.waited[b]:
            torch.cuda.current_stream(self.flat.device).wait_event(self.events[b])
            self.waited[b] = True

    def wait_all(self):
        """Current stream waits for the whole update (and the gradient zeroing)."""
        if self.overlap and self.done is not None:
            torch.cuda.current_stream(self.flat.device).wait_event(self.done)
            self.waited = [True] * len(self.waited)
            self.done = None

    @torch.no_grad()
    def step(self, grad_scale=1.0, lr=None, bucket_order=None, after_bucket=None, before_bucket=None):
        """One update.  With a sharded update (``owned``: one range per
        gradient bucket) and ``bucket_order`` / ``after_bucket``, the owned
        shards are updated bucket by bucket in that order and
        ``after_bucket(b)`` runs right after bucket b's update is enqueued --
        the ZeRO-1 all-gather of b then starts as soon as ITS shard is done
        instead of after the whole update (parallel/zero.ParamGather.launch_one);
        ``before_bucket(b)`` runs right before it (the traffic emulator's
        fused-reduce cost, parallel/emulate.py).
        Every element is updated exactly once either way: bit-identical."""
        f = self.flat
        self.step_count += 1
        lr = self.lr if lr is None else lr
        clip = self.max_grad_norm and self.max_grad_norm > 0
        if clip:
            self._norm_sq()
        if bucket_order is not None and self.owned is not None and not self.overlap:
            self._step_pipelined(lr, grad_scale, clip, bucket_order, after_bucket, before_bucket)
            return
        if self.overlap and f.param.dtype == torch.bfloat16:
            main = torch.cuda.current_stream(f.device)
            self.side.wait_stream(main)
            s = ctypes.c_void_p(self.side.cuda_stream)
            for bi in self.order:
                lo, hi = self.ranges[bi]
                for (a, b, decay) in self.runs:
                    a2, b2 = max(a, lo), min(b, hi)
                    if a2 < b2:
                        self._launch(a2, b2, decay, lr, grad_scale, clip, self.fuse_zero_grad, s)
                if self.post_update is not None:
                    with torch.cuda.stream(self.side):
                        self.post_update(lo, hi)
                ev = torch.cuda.Event()
                ev.record(self.side)
                self.events[bi] = ev
                self.waited[bi] = False
            self.done = torch.cuda.Event()
            self.done.record(self.side)
            # tensors used on the side stream must not be recycled by the main stream's allocator
            for t in (f.grad, f.param, f.master, f.exp_avg, f.exp_avg_sq, self._norm):
                t.record_stream(self.side)
            self.grads_zeroed = self.fuse_zero_grad
            return
        self.grads_zeroed = False
        if _lib.use_hip(f.grad):
            s = _lib.stream(f.grad)
            pbf = f.param.dtype == torch.bfloat16
            if self.device_step:
                _lib.call("toa_step_inc", _lib.ptr(self._dstep), s)
            fused = self._fused_items() if pbf else {}
            for (a, b, decay) in self._work_runs():
                pos = a
                for ia, ib in sorted(k for k in fused if a <= k[0] and k[1] <= b):
                    if pos < ia:
                        self._launch(pos, ia, decay, lr, grad_scale, clip, self.fuse_zero_grad, s)
                    self._launch_wt(fused[(ia, ib)], decay, lr, grad_scale, clip, s)
                    pos = ib
                if pos < b:
                    self._launch(pos, b, decay, lr, grad_scale, clip, self.fuse_zero_grad, s)
            self.grads_zeroed = self.fuse_zero_grad and self.owned is None
            if not pbf:
                f.param_from_master()
            if fused:
                done = {id(it[2]) for it in fused.values()}
                for _, _, p, view in self.fused_wt.items:   # the copies the fused update did not write
                    if id(p) not in done:
                        transpose_into(view, p.data)
            elif self.post_update is not None:
                self.post_update(0, f.numel)
        else:
            for (a, b, decay) in self._work_runs():
                adamw_reference(f.state_view(f.master, a, b), f.grad[a:b], f.state_view(f.exp_avg, a, b),
                                f.state_view(f.exp_avg_sq, a, b), lr=lr,
                                beta1=self.beta1, beta2=self.beta2, eps=self.eps,
                                weight_decay=self.weight_decay if decay else 0.0, step=self.step_count,
                                grad_scale=grad_scale, norm_sq=self._norm if clip else None,
                                max_norm=self.max_grad_norm or 0.0)
            for lo, hi in (self.owned or [(0, f.numel)]):
                f.param[lo:hi].copy_(f.state_view(f.master, lo, hi).to(f.param.dtype))
            if self.post_update is not None:
                self.post_update(0, f.numel)

    def _step_pipelined(self, lr, grad_scale, clip, order, after, before=None):
        f = self.flat
        self.grads_zeroed = False
        hip = _lib.use_hip(f.grad)
        if hip and self.device_step:
            _lib.call("toa_step_inc", _lib.ptr(self._dstep), _lib.stream(f.grad))
        for b in order:
            lo, hi = self.owned[b]
            if before is not None:
                before(b)
            for a, e, decay in self.runs:
                a2, b2 = max(a, lo), min(e, hi)
                if a2 >= b2:
                    continue
                if hip:
                    self._launch(a2, b2, decay, lr, grad_scale, clip, self.fuse_zero_grad, _lib.stream(f.grad))
                else:
                    adamw_reference(f.state_view(f.master, a2, b2), f.grad[a2:b2], f.state_view(f.exp_avg, a2, b2),
                                    f.state_view(f.exp_avg_sq, a2, b2), lr=lr, beta1=self.beta1,
                                    beta2=self.beta2, eps=self.eps,
                                    weight_decay=self.weight_decay if decay else 0.0, step=self.step_count,
                                    grad_scale=grad_scale, norm_sq=self._norm if clip else None,
                                    max_norm=self.max_grad_norm or 0.0)
            if not hip or f.param.dtype != torch.bfloat16:
                f.param[lo:hi].copy_(f.state_view(f.master, lo, hi).to(f.param.dtype))
            if after is not None:
                after(b)

    def sync_step_count(self):
        """Host copy of the device step count (after graph replays)."""
        if self.device_step:
            self.step_count = int(self._dstep.item())
        return self.step_count

    def state_dict(self):
        return {"step": self.sync_step_count(), "lr": self.lr}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        if self.device_step:
            self._dstep.fill_(self.step_count)
        self.lr = sd.get("lr", self.lr)


class FlatSGD:
    """SGD(+momentum) over fp32 flat buffers (estimator example)."""

    def __init__(self, flat, lr=0.2, momentum=0.0, weight_decay=0.0):
        self.flat, self.lr, self.momentum, self.weight_decay = flat, lr, momentum, weight_decay
        self.buf = torch.zeros_like(flat.master) if momentum else None

    @torch.no_grad()
    def step(self, grad_scale=1.0):
        f = self.flat
        g = f.grad if grad_scale == 1.0 else f.grad * grad_scale
        if g.dtype != torch.float32:
            g = g.float()
        if _lib.use_hip(f.master):
            _lib.call("toa_sgd_flat", _lib.ptr(f.master), _lib.ptr(g), _lib.ptr(self.buf), f.numel, float(self.lr),
                      float(self.momentum), float(self.weight_decay), _lib.stream(f.master))
        else:
            gg = g + self.weight_decay * f.master
            if self.buf is not None:
                self.buf.mul_(self.momentum).add_(gg)
                gg = self.buf
            f.master.add_(gg, alpha=-self.lr)
        if f.param.data_ptr() != f.master.data_ptr():
            f.param.copy_(f.master.to(f.param.dtype))
