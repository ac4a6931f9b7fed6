"""Linear layers whose weight gradient lands directly in the flat gradient buffer.

Plain GEMMs go to hipBLASLt with per-shape tuned solutions
(:mod:`tf_operator_amd.ops.gemm`; the CDNA guide's rule: library GEMMs for
plain GEMMs, hand-written MFMA kernels for fused hot ops -- see
:mod:`tf_operator_amd.ops.mlp` for the fused bias+activation GEMM).
The backward computes ``dW += dY^T X`` with beta=1 straight into
``weight.main_grad`` (no per-step weight-gradient temporaries, no extra
copy into an all-reduce bucket) and fires the bucket hook.
"""
from __future__ import annotations

import torch

from . import gemm
from .grad import accumulate_mm


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        ctx.save_for_backward(x, weight)
        y = gemm.linear_fwd(x.reshape(-1, x.shape[-1]), weight)
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = gemm.linear_dgrad(dy2, weight).view_as(x) if ctx.needs_input_grad[0] else None
        x2 = x.reshape(-1, x.shape[-1])
        dw = accumulate_mm(weight, dy2.t(), x2)
        return dx, dw


def linear(x, weight):
    return _LinearFn.apply(x, weight)


class Linear(torch.nn.Module):
    """bias-free linear, weight [out, in]."""

    def __init__(self, in_features, out_features, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = torch.nn.Parameter(torch.empty(out_features, in_features, dtype=dtype, device=device))

    def forward(self, x):
        return linear(x, self.weight)
