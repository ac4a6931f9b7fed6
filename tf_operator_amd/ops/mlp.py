"""Fused dense layer: y = dropout(act(x W^T + b)) on the gfx950 MFMA kernel
(csrc/hip/mlp.hip), plus accuracy / dropout helpers.

Reference call sites: dist_mnist.py:188-192 (xw_plus_b + ReLU + softmax),
mnist_with_summaries.py:92-106 (+dropout), :130-132 (accuracy) -- SURVEY
K1/K2/K3/K8/K9/K12.  The forward GEMM with its bias/activation/dropout
epilogue is the hand-written MFMA kernel; the backward's two plain GEMMs go
to hipBLASLt and the activation/dropout/bias-gradient part is the fused
``toa_bias_act_dropout_bwd`` kernel.
"""
from __future__ import annotations

import itertools

import torch
import torch.nn.functional as F

from . import _lib
from .grad import accumulate_mm, deliver_weight_grad

ACTS = {"none": 0, "relu": 1, "gelu": 2}
_seed_counter = itertools.count(0x5EED)


def _hash_keep(seed, shape, keep_prob, device):
    """CPU reference of the kernel's counter hash (splitmix64)."""
    M, N = shape
    idx = torch.arange(M * N, dtype=torch.int64).to(torch.uint64) if hasattr(torch, "uint64") else None
    import numpy as np

    i = np.arange(M * N, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * (i + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    h = (z >> np.uint64(32)).astype(np.uint64)
    thresh = np.uint64(min(int(keep_prob * 4294967296.0), 4294967295))
    del idx
    return torch.from_numpy((h < thresh).reshape(M, N)).to(device)


class _LinearBiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, keep_prob, seed):
        a = ACTS[act]
        M, K = x.shape
        N = w.shape[0]
        if _lib.use_hip(x):
            xb = x.contiguous() if x.dtype == torch.bfloat16 else x.to(torch.bfloat16).contiguous()
            wb = w.contiguous() if w.dtype == torch.bfloat16 else w.to(torch.bfloat16).contiguous()
            y = torch.empty(M, N, device=x.device, dtype=x.dtype)
            out_bf16 = int(y.dtype == torch.bfloat16)
            bb = b.contiguous() if b is not None else None
            if act == "gelu":  # GELU backward needs the pre-activation
                z = torch.empty_like(y)
                _lib.call("toa_gemm_bias_act", out_bf16, _lib.ptr(xb), _lib.ptr(wb), _lib.ptr(bb), _lib.ptr(z),
                          M, N, K, 0, int(bb is not None and bb.dtype == torch.bfloat16), 0, 0, _lib.stream(x))
                y = F.gelu(z.float()).to(z.dtype)
                if keep_prob < 1.0:
                    _lib.call("toa_dropout_fwd", _lib.dtype_code(y), _lib.ptr(y), _lib.ptr(y), None, y.numel(),
                              float(keep_prob), seed, 0, _lib.stream(x))
            else:
                z = None
                _lib.call("toa_gemm_bias_act_dropout", out_bf16, _lib.ptr(xb), _lib.ptr(wb), _lib.ptr(bb),
                          _lib.ptr(y), M, N, K, a, int(bb is not None and bb.dtype == torch.bfloat16),
                          float(keep_prob), seed, _lib.stream(x))
        else:
            z = x.float() @ w.float().t() + (b.float() if b is not None else 0.0)
            y = {"none": z, "relu": torch.relu(z), "gelu": F.gelu(z)}[act]
            if keep_prob < 1.0:
                y = y * _hash_keep(seed, (M, N), keep_prob, x.device) / keep_prob
            y = y.to(x.dtype)
            z = z.to(x.dtype) if act == "gelu" else None
        ctx.save_for_backward(x, w, y, z)
        ctx.act, ctx.keep, ctx.seed, ctx.has_b = act, keep_prob, seed, b is not None
        ctx.b = b
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y, z = ctx.saved_tensors
        M, N = y.shape
        dy = dy.contiguous()
        if _lib.use_hip(dy):
            dz = torch.empty_like(dy)
            db = torch.empty(N, device=dy.device, dtype=torch.float32) if ctx.has_b else None
            _lib.call("toa_bias_act_dropout_bwd", _lib.dtype_code(dy), _lib.ptr(dy), _lib.ptr(y), _lib.ptr(z),
                      _lib.ptr(dz), _lib.ptr(db), M, N, ACTS[ctx.act], float(ctx.keep), ctx.seed, _lib.stream(dy))
        else:
            g = dy.float()
            if ctx.keep < 1.0:
                g = g * _hash_keep(ctx.seed, (M, N), ctx.keep, dy.device) / ctx.keep
            if ctx.act == "relu":
                g = g * (y.float() > 0)
            elif ctx.act == "gelu":
                zz = z.float()
                cdf = 0.5 * (1 + torch.erf(zz * 0.7071067811865476))
                pdf = 0.3989422804014327 * torch.exp(-0.5 * zz * zz)
                g = g * (cdf + zz * pdf)
            dz = g.to(dy.dtype)
            db = g.sum(0) if ctx.has_b else None
        dx = (dz @ w.to(dz.dtype)).to(x.dtype) if ctx.needs_input_grad[0] else None
        dw = accumulate_mm(w, dz.t().to(w.dtype), x.to(w.dtype))
        dbias = deliver_weight_grad(ctx.b, db) if ctx.has_b else None
        return dx, dw, dbias, None, None, None


def linear_bias_act(x, w, b=None, act="relu", keep_prob=1.0, seed=None):
    if keep_prob < 1.0 and seed is None:
        seed = next(_seed_counter)
    return _LinearBiasAct.apply(x, w, b, act, float(keep_prob), int(seed or 0))


class DenseAct(torch.nn.Module):
    """Linear + bias + activation (+ dropout) in one MFMA launch."""

    def __init__(self, din, dout, act="relu", dtype=torch.bfloat16, device=None, keep_prob=1.0):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.empty(dout, din, dtype=dtype, device=device))
        self.bias = torch.nn.Parameter(torch.zeros(dout, dtype=dtype, device=device))
        self.act = act
        self.keep_prob = keep_prob
        torch.nn.init.trunc_normal_(self.weight, std=1.0 / (din ** 0.5))

    def forward(self, x):
        kp = self.keep_prob if self.training else 1.0
        return linear_bias_act(x, self.weight, self.bias, self.act, kp)


def accuracy(logits, labels):
    """fraction of rows whose argmax == label (HIP: one wave per row + atomic count)."""
    if _lib.use_hip(logits):
        correct = torch.zeros(1, device=logits.device, dtype=torch.int32)
        lg = logits.contiguous()
        _lib.call("toa_accuracy", _lib.dtype_code(lg), _lib.ptr(lg), _lib.ptr(labels.to(torch.int64).contiguous()),
                  _lib.ptr(correct), lg.shape[0], lg.shape[1], _lib.stream(lg))
        return correct.float() / lg.shape[0]
    return (logits.argmax(-1) == labels).float().mean().reshape(1)
