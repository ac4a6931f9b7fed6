"""Data-parallel trainer for the small bundled models (MNIST MLP, Keras CNN,
estimator DNN, ResNet-50): flat parameters, backward-overlapped bucketed
RCCL/gloo all-reduce, fused HIP Adam/SGD, checkpoint/resume, first-step
reporting.  The Llama path has its own trainer (:mod:`.llm`)."""
from __future__ import annotations

import os
import time

import torch

from ..ops.grad import take_fresh
from ..ops.optim import FlatAdamW, FlatSGD
from ..parallel.ddp import GradBucketer, broadcast_params
from ..parallel.flat import FlatParams
from . import checkpoint as ckpt


def attach_autograd_hooks(flat: FlatParams):
    """Params whose gradients come from plain autograd ops (convs, BN) get a
    post-accumulate hook that folds .grad into the flat buffer and fires the
    bucket hook, so their all-reduce also overlaps backward."""
    for s in flat.segments:
        p = s.param

        def hook(param):
            if param.grad is None:
                return
            if take_fresh(param):
                param.main_grad.copy_(param.grad.view_as(param.main_grad))
            else:
                param.main_grad.add_(param.grad.view_as(param.main_grad))
            param.grad = None
            h = getattr(param, "_toa_ready", None)
            if h is not None:
                h(param)

        p.register_post_accumulate_grad_hook(hook)


class DPTrainer:
    """graph=True (default on a GPU, ``TOA_HIP_GRAPH=0`` turns it off): after
    GRAPH_WARMUP eager steps (run on a side stream, so every library handle
    and workspace exists before capture) the whole training step -- zero
    grad, forward, loss, backward, optimizer -- is captured once as a HIP
    graph and each later step is two input copies plus one graph launch.
    The bundled payloads' models are tiny (79K-400K parameters), so their
    eager step is bound by kernel-launch overhead, not by the GPU.  Single
    replica only (world size 1): multi-replica steps keep the eager path
    with the bucketed all-reduce."""

    GRAPH_WARMUP = 3

    def __init__(self, model, loss_fn, runtime, lr=1e-3, optimizer="adam", weight_decay=0.0, bucket_mb=None,
                 max_grad_norm=0.0, grad_dtype=torch.float32, graph=None):
        self.model = model
        self.loss_fn = loss_fn
        self.rt = runtime
        params = [p for p in model.parameters() if p.requires_grad]
        names = {id(p): n for n, p in model.named_parameters()}
        # backward order ~ reverse registration order
        self.flat = FlatParams(list(reversed(params)), names=names, grad_dtype=grad_dtype)
        attach_autograd_hooks(self.flat)
        broadcast_params(self.flat)
        self.bucketer = GradBucketer(self.flat, bucket_bytes=None if bucket_mb is None else int(bucket_mb * 2**20))
        if graph is None:
            graph = os.environ.get("TOA_HIP_GRAPH", "1") == "1"
        self.use_graph = (bool(graph) and self.flat.device.type == "cuda" and not self.bucketer.enabled
                          and getattr(model, "graph_safe", True))
        if optimizer == "adam":
            self.opt = FlatAdamW(self.flat, lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay,
                                 max_grad_norm=max_grad_norm, device_step=self.use_graph)
        else:
            self.opt = FlatSGD(self.flat, lr=lr, weight_decay=weight_decay)
        self.step_idx = 0
        self._graph = None
        self._side = torch.cuda.Stream(self.flat.device) if self.use_graph else None

    def _body(self, x, y):
        self.flat.zero_grad()
        out = self.model(x)
        loss = self.loss_fn(out, y)
        loss.backward()
        self.bucketer.finish()
        self.opt.step(grad_scale=self.bucketer.grad_scale)
        return loss.detach(), out.detach()

    def _graph_key(self, x, y):
        # host scalars a capture freezes: a new learning rate (per-epoch
        # decay) or new input shapes re-capture
        return (float(self.opt.lr), tuple(x.shape), tuple(y.shape), x.dtype, y.dtype)

    def _capture(self, x, y):
        self._sx, self._sy = x.detach().clone(), y.detach().clone()
        torch.cuda.synchronize(self.flat.device)
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                self._sloss, self._sout = self._body(self._sx, self._sy)
        except RuntimeError as e:  # an op that cannot be captured: stay eager
            self.rt.log(f"HIP graph capture failed ({e}); continuing eagerly")
            self.use_graph = False
            self._graph = None
            torch.cuda.synchronize(self.flat.device)
            return
        self._graph = g
        self._key = self._graph_key(x, y)

    def step(self, x, y):
        if self._graph is not None and self._graph_key(x, y) != self._key:
            self._graph = None
        if self.use_graph and self._graph is None and self.step_idx >= self.GRAPH_WARMUP:
            self._capture(x, y)  # records only: the replay below takes this step
        if self._graph is not None:
            self._sx.copy_(x, non_blocking=True)
            self._sy.copy_(y, non_blocking=True)
            self._graph.replay()
            self.step_idx += 1
            return self._sloss, self._sout
        if self.use_graph:  # warm-up steps on a side stream (CUDA/HIP graph capture rules)
            self._side.wait_stream(torch.cuda.current_stream(self.flat.device))
            with torch.cuda.stream(self._side):
                loss, out = self._body(x, y)
            torch.cuda.current_stream(self.flat.device).wait_stream(self._side)
        else:
            loss, out = self._body(x, y)
        self.step_idx += 1
        if self.step_idx == 1:
            if torch.cuda.is_available() and x.is_cuda:
                torch.cuda.synchronize()
            self.rt.first_step_done()
        return loss, out

    # ------------------------------------------------------------------ checkpoint
    def state(self):
        self.bucketer.verify()  # never persist an update built from a failed one-shot all-reduce
        st = {"flat": self.flat.state_dict(), "step": self.step_idx}
        if isinstance(self.opt, FlatAdamW):
            st["opt"] = self.opt.state_dict()
        buffers = {n: b for n, b in self.model.named_buffers()}
        if buffers:
            st["buffers"] = buffers
        return st

    def save(self, ckpt_dir, keep=2):
        if ckpt_dir and self.rt.is_chief:
            ckpt.save(ckpt_dir, self.step_idx, self.state(), keep)

    def maybe_resume(self, ckpt_dir):
        payload = ckpt.load_latest(ckpt_dir)
        if payload is None:
            return 0
        st = payload["state"]
        dev = self.flat.device
        self.flat.load_state_dict({k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in st["flat"].items()})
        if "opt" in st and isinstance(self.opt, FlatAdamW):
            self.opt.load_state_dict(st["opt"])
        for n, b in (st.get("buffers") or {}).items():
            dict(self.model.named_buffers())[n].copy_(b.to(dev))
        self.step_idx = int(payload["step"])
        return self.step_idx


class PSTrainer:
    """Worker side of parameter-server training (TFJob with PS replicas;
    :mod:`tf_operator_amd.parallel.ps_collective`): forward + backward on
    this GPU, gradients reduced onto / pushed to the servers during (sync)
    or after (async) backward, fresh parameters received from them.  The
    worker keeps no optimizer state -- the servers own it."""

    def __init__(self, model, loss_fn, runtime, workers, servers, mode="sync", lr=1e-3, bucket_mb=64.0,
                 grad_dtype=torch.float32):
        from ..parallel.ps_collective import CollectivePS

        self.model, self.loss_fn, self.rt = model, loss_fn, runtime
        params = [p for p in model.parameters() if p.requires_grad]
        names = {id(p): n for n, p in model.named_parameters()}
        self.flat = FlatParams(list(reversed(params)), names=names, grad_dtype=grad_dtype, master=False)
        attach_autograd_hooks(self.flat)
        self.ps = CollectivePS(self.flat, workers, servers, mode=mode, lr=lr, bucket_mb=bucket_mb)
        self.step_idx = 0
        # the next forward waits, module by module, only for the buckets holding
        # its own parameters (the asynchronous parameter pull of sync mode)
        def waiter(buckets):
            def hook(mod, args):
                for b in buckets:
                    self.ps.wait_bucket(b)
            return hook

        self._hooks = []
        for mod in model.modules():
            bs = sorted({p._toa_bucket for p in mod.parameters(recurse=False) if hasattr(p, "_toa_bucket")})
            if bs:
                self._hooks.append(mod.register_forward_pre_hook(waiter(bs)))

    def sync_params(self):
        """Every parameter current (before reading ``flat.param`` directly:
        checkpoints, comparisons)."""
        self.ps.wait_params()

    def step(self, x, y):
        self.flat.zero_grad()
        out = self.model(x)
        loss = self.loss_fn(out, y)
        loss.backward()
        self.ps.worker_step()
        self.step_idx += 1
        if self.step_idx == 1:
            if torch.cuda.is_available() and x.is_cuda:
                torch.cuda.synchronize()
            self.rt.first_step_done()
        return loss.detach(), out.detach()


def parameter_server(model, workers, servers, mode="sync", lr=1e-3, bucket_mb=64.0, grad_dtype=torch.float32):
    """Server side: the same model (for the flat layout; its activations are
    never computed), the fp32 master / Adam state of this server's shard."""
    from ..parallel.ps_collective import CollectivePS

    params = [p for p in model.parameters() if p.requires_grad]
    names = {id(p): n for n, p in model.named_parameters()}
    flat = FlatParams(list(reversed(params)), names=names, grad_dtype=grad_dtype)
    return CollectivePS(flat, workers, servers, mode=mode, lr=lr, bucket_mb=bucket_mb)


def run(trainer: DPTrainer, data, steps, log_every=50, ckpt_dir=None, ckpt_every=0, metric_fn=None,
        samples_per_step=None):
    rt = trainer.rt
    start = trainer.maybe_resume(ckpt_dir)
    if start:
        rt.log(f"resumed from checkpoint at step {start}")
    t0 = time.perf_counter()
    n0 = trainer.step_idx
    last = None
    while trainer.step_idx < steps:
        x, y = data.next()
        loss, out = trainer.step(x, y)
        last = (loss, out, y)
        s = trainer.step_idx
        if log_every and (s % log_every == 0 or s == steps):
            msg = f"step {s} loss {float(loss):.4f}"
            if metric_fn is not None:
                msg += f" acc {float(metric_fn(out, y)):.3f}"
            rt.log(msg)
        if ckpt_dir and ckpt_every and s % ckpt_every == 0:
            trainer.save(ckpt_dir)
        if rt.preempted.is_set():
            trainer.save(ckpt_dir)
            rt.log(f"preempted at step {s}; checkpoint written")
            raise SystemExit(143)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    done = trainer.step_idx - n0
    if samples_per_step and done:
        sps = samples_per_step * done / max(dt, 1e-9)
        rt.report(samples_per_sec=sps)
        rt.log(f"throughput {sps:.1f} samples/s over {done} steps")
    if ckpt_dir:
        trainer.save(ckpt_dir)
    return last
