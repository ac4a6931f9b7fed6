"""Fused AdamW / SGD over flat buffers (HIP kernels in csrc/hip/optim.hip).

One streaming launch per contiguous weight-decay run of the flat buffer;
the gradient clip coefficient is computed on the device from the global
squared norm (``toa_sumsq``), so ``step()`` never synchronises with the host.
"""
from __future__ import annotations

import math

import torch

from . import _lib


def grad_norm_sq(flat_grad: torch.Tensor, workspace=None, out=None):
    """Squared L2 norm of a flat gradient (fp32 0-d device tensor)."""
    out = torch.zeros(1, device=flat_grad.device, dtype=torch.float32) if out is None else out
    if _lib.use_hip(flat_grad):
        ws = torch.empty(2048, device=flat_grad.device, dtype=torch.float32) if workspace is None else workspace
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


class FlatAdamW:
    """AdamW over a :class:`tf_operator_amd.parallel.flat.FlatParams`."""

    def __init__(self, flat, lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0):
        self.flat = flat
        self.lr = lr
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        if flat.exp_avg is None:
            flat.exp_avg = torch.zeros(flat.numel, device=flat.device, dtype=torch.float32)
            flat.exp_avg_sq = torch.zeros(flat.numel, device=flat.device, dtype=torch.float32)
        self.runs = flat.decay_runs()
        self._norm = torch.zeros(1, device=flat.device, dtype=torch.float32)
        self._ws = torch.empty(2048, device=flat.device, dtype=torch.float32)
        self.last_norm_sq = self._norm

    @torch.no_grad()
    def step(self, grad_scale=1.0, lr=None):
        f = self.flat
        self.step_count += 1
        lr = self.lr if lr is None else lr
        clip = self.max_grad_norm and self.max_grad_norm > 0
        if clip:
            grad_norm_sq(f.grad, self._ws, self._norm)
        if _lib.use_hip(f.grad):
            s = _lib.stream(f.grad)
            gbf = int(f.grad.dtype == torch.bfloat16)
            pbf = f.param.dtype == torch.bfloat16
            esz_p, esz_g = f.param.element_size(), f.grad.element_size()
            for (a, b, decay) in self.runs:
                n = b - a
                wd = self.weight_decay if decay else 0.0
                pp = _lib.ptr(f.param) if pbf else None
                _lib.call("toa_adamw_flat", f.master.data_ptr() + 4 * a,
                          (f.param.data_ptr() + esz_p * a) if pp is not None else None,
                          f.grad.data_ptr() + esz_g * a, gbf, f.exp_avg.data_ptr() + 4 * a,
                          f.exp_avg_sq.data_ptr() + 4 * a, n, float(lr), float(self.beta1), float(self.beta2),
                          float(self.eps), float(wd), self.step_count, float(grad_scale),
                          _lib.ptr(self._norm) if clip else None, float(self.max_grad_norm or 0.0), s)
            if not pbf:
                f.param.copy_(f.master)
        else:
            for (a, b, decay) in self.runs:
                adamw_reference(f.master[a:b], f.grad[a:b], f.exp_avg[a:b], f.exp_avg_sq[a:b], lr=lr,
                                beta1=self.beta1, beta2=self.beta2, eps=self.eps,
                                weight_decay=self.weight_decay if decay else 0.0, step=self.step_count,
                                grad_scale=grad_scale, norm_sq=self._norm if clip else None,
                                max_norm=self.max_grad_norm or 0.0)
            f.param.copy_(f.master.to(f.param.dtype))

    def state_dict(self):
        return {"step": self.step_count, "lr": self.lr}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
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
