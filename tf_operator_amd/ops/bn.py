"""Fused BatchNorm (+ residual add) (+ ReLU) for channels-last activations
(HIP kernels in csrc/hip/bn.hip) -- the ResNet-50 payload's normalisation
(BASELINE config #2).

    y = relu(batch_norm(x) [+ res])

Training mode normalises with the batch statistics and updates the running
ones (momentum, unbiased variance: torch.nn.BatchNorm2d semantics); eval
mode uses the running statistics.  The backward re-derives the ReLU mask
from x and the saved per-channel scale / shift (bit-identical to the
forward's sign), or from the saved output when a residual was added before
the ReLU, so nothing extra is stored.  dgamma / dbeta go straight into the flat gradient buffer
(``param.main_grad``) when the parameters are managed by FlatParams.

On a GPU tensor this is the HIP path only (channels-last bf16/fp32, C % 8 ==
0, C <= 2048; anything else raises); CPU tensors take the PyTorch reference.
``TOA_BN=torch`` is an explicit A/B switch that runs PyTorch's batch_norm
(+ add + relu) on the GPU too (profiles/r2_resnet compares the two).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _lib
from .grad import deliver_weight_grad, take_fresh


_MODE = os.environ.get("TOA_BN", "hip")


def _rows(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels-last (or [R, C]) -> the [R, C] row-major view."""
    if x.dim() == 2:
        return x if x.is_contiguous() else x.contiguous()
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("fused BatchNorm needs a channels-last 4D (or [rows, C]) tensor")
    return x.permute(0, 2, 3, 1).reshape(-1, x.shape[1])


def _like(t: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """[R, C] buffer -> the logical shape / memory format of x."""
    if x.dim() == 2:
        return t
    n, c, h, w = x.shape
    return t.view(n, h, w, c).permute(0, 3, 1, 2)


def _ws(R: int, C: int, device) -> torch.Tensor:
    n = int(_lib.call_ret("toa_bn_ws_floats", R, C))
    return torch.empty(n, device=device, dtype=torch.float32)


def _check_hip(x, weight):
    if not (_lib.has("toa_bn_fwd_train") and x.dtype in (torch.bfloat16, torch.float32)):
        raise RuntimeError(f"HIP BatchNorm unavailable for {x.dtype}: {_lib.load_error() or 'unsupported dtype'}")
    C = x.shape[1]
    if C % 8 or C > 2048:
        raise RuntimeError(f"HIP BatchNorm needs C % 8 == 0 and C <= 2048 (got {C})")
    if weight is not None and weight.dtype not in (torch.bfloat16, torch.float32):
        raise RuntimeError(f"HIP BatchNorm parameters must be bf16/fp32 (got {weight.dtype})")


class _BatchNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, weight, bias, running_mean, running_var, training, momentum, eps, relu):
        _check_hip(x, weight)
        x2 = _rows(x)
        R, C = x2.shape
        r2 = _rows(res) if res is not None else None
        y2 = torch.empty_like(x2)
        ws = _ws(R, C, x.device)
        pd = weight if weight is not None else running_mean
        pdt = _lib.dtype_code(pd) if pd is not None else 1
        st = _lib.stream(x)
        if training:
            stats = torch.empty(4 * C, device=x.device, dtype=torch.float32)  # mean, invstd, scale, shift
            _lib.call("toa_bn_fwd_train", _lib.dtype_code(x2), pdt, _lib.ptr(x2), _lib.ptr(r2), _lib.ptr(y2),
                      R, C, _lib.ptr(weight), _lib.ptr(bias), _lib.ptr(running_mean),
                      _lib.ptr(running_var), float(momentum), float(eps), int(relu), _lib.ptr(stats), _lib.ptr(ws), st)
        else:
            stats = None
            _lib.call("toa_bn_fwd_eval", _lib.dtype_code(x2), pdt, _lib.ptr(x2), _lib.ptr(r2), _lib.ptr(y2),
                      R, C, _lib.ptr(weight), _lib.ptr(bias), _lib.ptr(running_mean),
                      _lib.ptr(running_var), float(eps), int(relu), _lib.ptr(ws), st)
        y = _like(y2, x)
        ctx.training, ctx.relu, ctx.has_res = training, relu, res is not None
        # ReLU mask in backward: from x and the saved scale / shift unless a
        # residual was added before the ReLU (then from the saved output)
        ctx.mask = 0 if not relu else (1 if res is not None else 2)
        ctx.save_for_backward(x, y if ctx.mask == 1 else None, stats, weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, stats, weight, bias = ctx.saved_tensors
        if not ctx.training:
            raise RuntimeError("backward through an eval-mode fused BatchNorm is not supported")
        x2 = _rows(x)
        R, C = x2.shape
        dy2 = _rows(dy.contiguous(memory_format=torch.channels_last) if dy.dim() == 4 else dy.contiguous())
        y2 = _rows(y) if y is not None else None
        dx2 = torch.empty_like(x2)
        dres2 = torch.empty_like(x2) if ctx.has_res else None
        pdt = _lib.dtype_code(weight) if weight is not None else 1
        # dgamma / dbeta straight into the flat gradient buffer (main_grad,
        # accumulated by the finalize kernel) when the parameters are managed
        # by FlatParams: no per-layer temporary, cast and add
        mg = getattr(weight, "main_grad", None) if weight is not None else None
        mb = getattr(bias, "main_grad", None) if bias is not None else None
        into_flat = mg is not None and (bias is None or mb is not None) and mg.dtype in (torch.float32,
                                                                                          torch.bfloat16)
        if into_flat:
            dg, db, gdt, acc = mg, mb, _lib.dtype_code(mg), 1
            if db is not None and db.dtype != dg.dtype:
                into_flat = False
            else:  # the step's first producer overwrites (grad.take_fresh)
                fw = take_fresh(weight)
                fb = take_fresh(bias) if bias is not None else fw
                if fw and fb:
                    acc = 0
                else:
                    for p_, f_ in ((weight, fw), (bias, fb if bias is not None else False)):
                        if f_:
                            p_.main_grad.zero_()
        if not into_flat:
            dg = torch.empty(C, device=x.device, dtype=weight.dtype) if weight is not None else None
            db = torch.empty(C, device=x.device, dtype=bias.dtype) if bias is not None else None
            gdt = _lib.dtype_code(dg if dg is not None else (db if db is not None else x2))
            acc = 0
        ws = _ws(R, C, x.device)
        _lib.call("toa_bn_bwd", _lib.dtype_code(x2), pdt, _lib.ptr(dy2), _lib.ptr(x2), _lib.ptr(y2), ctx.mask,
                  _lib.ptr(stats),
                  _lib.ptr(weight), R, C, _lib.ptr(dx2), _lib.ptr(dres2), _lib.ptr(dg), _lib.ptr(db), gdt, acc,
                  _lib.ptr(ws), _lib.stream(x))
        if into_flat:
            gw = deliver_weight_grad(weight, None)
            gb = deliver_weight_grad(bias, None) if bias is not None else None
        else:
            gw = deliver_weight_grad(weight, dg) if weight is not None else None
            gb = deliver_weight_grad(bias, db) if bias is not None else None
        dres = _like(dres2, x) if dres2 is not None else None
        return _like(dx2, x), dres, gw, gb, None, None, None, None, None, None


def batch_norm_act(x, weight, bias, running_mean, running_var, training=True, momentum=0.1, eps=1e-5, relu=True,
                   residual=None):
    """y = relu(batch_norm(x) + residual) (residual / relu optional)."""
    if x.is_cuda and _MODE != "torch":
        return _BatchNormAct.apply(x, residual, weight, bias, running_mean, running_var, training, momentum, eps, relu)
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class FusedBatchNorm2d(torch.nn.BatchNorm2d):
    """``BatchNorm2d`` (same parameters, buffers and state_dict) whose forward
    is one fused HIP pass with an optional ReLU and residual add:
    ``bn(x, residual=r)`` = relu(BN(x) + r) when ``relu=True``."""

    def __init__(self, num_features, relu=False, **kw):
        super().__init__(num_features, **kw)
        self.relu = relu

    def forward(self, x, residual=None):
        training = self.training or self.running_mean is None
        momentum = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
            if self.momentum is None:  # torch: cumulative moving average, factor 1 / batches seen
                momentum = 1.0 / float(self.num_batches_tracked)
        return batch_norm_act(x, self.weight, self.bias, self.running_mean if not self.training or
                              self.track_running_stats else None,
                              self.running_var if not self.training or self.track_running_stats else None,
                              training, momentum, self.eps, self.relu, residual)
