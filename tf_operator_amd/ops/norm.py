"""RMSNorm / LayerNorm with fused residual add (HIP kernels in csrc/hip/norm.hip).

``rms_norm(x, w, eps)`` -> y
``add_rms_norm(x, residual, w, eps)`` -> (h = x + residual, y = rmsnorm(h))

Weight gradients go straight into ``weight.main_grad`` (the flat gradient
buffer of :class:`tf_operator_amd.parallel.flat.FlatParams`) when present,
and the parameter's ready-hook fires so the gradient bucketer can launch its
all-reduce while the rest of backward is still running.
"""
from __future__ import annotations

import torch

from . import _lib
from .grad import deliver_weight_grad, take_fresh


def _ref_norm(h, w, b, eps, rms):
    hf = h.float()
    if rms:
        rstd = torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps)
        mean = torch.zeros_like(rstd)
    else:
        mean = hf.mean(-1, keepdim=True)
        rstd = torch.rsqrt((hf - mean).pow(2).mean(-1, keepdim=True) + eps)
    y = (hf - mean) * rstd * w.float()
    if b is not None:
        y = y + b.float()
    return y.to(h.dtype), mean.squeeze(-1), rstd.squeeze(-1)


def _ref_norm_bwd(dy, h, w, mean, rstd, rms):
    hf, dyf, wf = h.float(), dy.float(), w.float()
    xh = (hf - mean.unsqueeze(-1)) * rstd.unsqueeze(-1)
    g = dyf * wf
    c1 = (g * xh).mean(-1, keepdim=True)
    if rms:
        dx = (g - xh * c1) * rstd.unsqueeze(-1)
    else:
        dx = (g - g.mean(-1, keepdim=True) - xh * c1) * rstd.unsqueeze(-1)
    dw = (dyf * xh).sum(0)
    db = dyf.sum(0)
    return dx, dw, db


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, rms):
        shape = x.shape
        cols = shape[-1]
        x2 = x.reshape(-1, cols)
        rows = x2.shape[0]
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        # residual == "presummed": x already holds the residual sum (the output
        # projection's GEMM added it, ops/llm._AttnOutProj): no add, h is x
        presum = isinstance(residual, str)
        r2 = residual.reshape(-1, cols).contiguous() if residual is not None and not presum else None
        if _lib.use_hip(x2):
            y = torch.empty_like(x2)
            h = torch.empty_like(x2) if r2 is not None else x2
            rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
            mean = torch.empty(rows, device=x.device, dtype=torch.float32) if not rms else None
            s = _lib.stream(x2)
            dt = _lib.dtype_code(x2)
            if rms:
                _lib.call("toa_rmsnorm_fwd", dt, _lib.ptr(x2), _lib.ptr(r2), _lib.ptr(h if r2 is not None else None),
                          _lib.ptr(weight), _lib.ptr(y), _lib.ptr(rstd), rows, cols, float(eps), s)
            else:
                _lib.call("toa_layernorm_fwd", dt, _lib.ptr(x2), _lib.ptr(r2),
                          _lib.ptr(h if r2 is not None else None), _lib.ptr(weight), _lib.ptr(bias), _lib.ptr(y),
                          _lib.ptr(mean), _lib.ptr(rstd), rows, cols, float(eps), s)
        else:
            h = x2 + r2 if r2 is not None else x2
            y, mean, rstd = _ref_norm(h, weight, bias, eps, rms)
        ctx.save_for_backward(h, weight, mean, rstd)
        ctx.rms = rms
        ctx.has_res = residual is not None
        ctx.presum = presum
        ctx.has_bias = bias is not None
        ctx.bias = bias
        ctx.shape = shape
        if residual is not None:
            return h.view(shape), y.view(shape)
        return y.view(shape)

    @staticmethod
    def backward(ctx, *grads):
        h, weight, mean, rstd = ctx.saved_tensors
        rms = ctx.rms
        cols = h.shape[-1]
        rows = h.shape[0]
        if ctx.has_res:
            dh, dy = grads
        else:
            dh, dy = None, grads[0]
        dy2 = dy.reshape(-1, cols).contiguous()
        dh2 = dh.reshape(-1, cols).contiguous() if dh is not None else None
        bias = ctx.bias
        dw = db = None
        if _lib.use_hip(dy2):
            dx = torch.empty_like(dy2)
            nb = _lib.lib().toa_norm_bwd_blocks(rows, cols)
            partial = torch.empty(nb * cols * (1 if rms else 2), device=dy.device, dtype=torch.float32)
            w_main = getattr(weight, "main_grad", None)
            dw_t = w_main if w_main is not None else torch.empty(cols, device=dy.device, dtype=torch.float32)
            b_main = getattr(bias, "main_grad", None) if bias is not None else None
            db_t = None
            if ctx.has_bias:
                db_t = b_main if b_main is not None else torch.empty(cols, device=dy.device, dtype=torch.float32)
            s = _lib.stream(dy2)
            dt = _lib.dtype_code(dy2)
            acc = 1 if w_main is not None else 0
            if acc:  # the step's first producer overwrites (grad.take_fresh)
                fw = take_fresh(weight)
                fb = take_fresh(bias) if b_main is not None else fw
                if fw and fb:
                    acc = 0
                else:
                    for p_, f_ in ((weight, fw), (bias, fb if b_main is not None else False)):
                        if f_:
                            p_.main_grad.zero_()
            if rms:
                _lib.call("toa_rmsnorm_bwd", dt, _lib.ptr(dy2), _lib.ptr(h), _lib.ptr(weight), _lib.ptr(rstd),
                          _lib.ptr(dh2), _lib.ptr(dx), _lib.ptr(partial), _lib.ptr(dw_t),
                          int(dw_t.dtype == torch.bfloat16), acc, rows, cols, s)
            else:
                _lib.call("toa_layernorm_bwd", dt, _lib.ptr(dy2), _lib.ptr(h), _lib.ptr(weight), _lib.ptr(mean),
                          _lib.ptr(rstd), _lib.ptr(dh2), _lib.ptr(dx), _lib.ptr(partial), _lib.ptr(dw_t),
                          int(dw_t.dtype == torch.bfloat16), _lib.ptr(db_t),
                          int(db_t is not None and db_t.dtype == torch.bfloat16), acc, rows, cols, s)
            if w_main is None:
                dw = dw_t.to(weight.dtype)
            else:
                deliver_weight_grad(weight, None)
            if ctx.has_bias:
                if b_main is None:
                    db = db_t.to(bias.dtype)
                else:
                    deliver_weight_grad(bias, None)
        else:
            dxf, dwf, dbf = _ref_norm_bwd(dy2, h, weight, mean if mean is not None else torch.zeros_like(rstd), rstd,
                                          rms)
            if dh2 is not None:
                dxf = dxf + dh2.float()
            dx = dxf.to(dy2.dtype)
            dw = deliver_weight_grad(weight, dwf)
            if ctx.has_bias:
                db = deliver_weight_grad(bias, dbf)
        dx = dx.view(ctx.shape)
        return dx, (dx if ctx.has_res and not ctx.presum else None), dw, db, None, None


def rms_norm(x, weight, eps=1e-5):
    return _NormFn.apply(x, None, weight, None, eps, True)


def add_rms_norm(x, residual, weight, eps=1e-5):
    """h = x + residual; return (h, rms_norm(h))."""
    return _NormFn.apply(x, residual, weight, None, eps, True)


def layer_norm(x, weight, bias=None, eps=1e-5):
    return _NormFn.apply(x, None, weight, bias, eps, False)


def add_layer_norm(x, residual, weight, bias=None, eps=1e-5):
    return _NormFn.apply(x, residual, weight, bias, eps, False)


class RMSNorm(torch.nn.Module):
    def __init__(self, dim, eps=1e-5, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(dim, dtype=dtype, device=device))

    def forward(self, x, residual=None):
        if residual is None:
            return rms_norm(x, self.weight, self.eps)
        return add_rms_norm(x, residual, self.weight, self.eps)

    def presummed(self, h):
        """(h, rmsnorm(h)) for an h that already holds the residual sum: one
        read of h, and the backward returns dh + the norm's gradient fused,
        as the residual form does.  Goes through the module call so its
        forward pre-hooks run: ZeRO-1's per-bucket all-gather wait
        (train/llm._install_param_waits) hangs on this module -- calling
        _NormFn directly read the weight before its gather had landed."""
        return self(h, "presummed")


class LayerNorm(torch.nn.Module):
    def __init__(self, dim, eps=1e-5, dtype=torch.float32, device=None):
        super().__init__()
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(dim, dtype=dtype, device=device))
        self.bias = torch.nn.Parameter(torch.zeros(dim, dtype=dtype, device=device))

    def forward(self, x, residual=None):
        if residual is None:
            return layer_norm(x, self.weight, self.bias, self.eps)
        return add_layer_norm(x, residual, self.weight, self.bias, self.eps)
