"""Token embedding whose backward scatters straight into ``weight.main_grad``."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from .grad import deliver_weight_grad, take_fresh


def _scatter_rows(grad, idx, dy2):
    """grad[idx[i]] += dy2[i].  On the GPU: sort the ids, then one fp32 sum
    per distinct id (csrc/hip/llm.hip embed_bwd_kernel) -- deterministic, no
    float atomics (index_add_ is neither on ROCm)."""
    if (_lib.use_hip(dy2) and dy2.dtype == torch.bfloat16 and grad.dtype in (torch.bfloat16, torch.float32)
            and dy2.shape[1] % 8 == 0 and grad.is_contiguous() and idx.numel() > 0):
        srt, perm = torch.sort(idx.long(), stable=True)
        dy2 = dy2.contiguous()
        _lib.call("toa_embed_bwd", _lib.ptr(srt), _lib.ptr(perm), _lib.ptr(dy2), _lib.ptr(grad),
                  int(grad.dtype == torch.float32), idx.numel(), dy2.shape[1], _lib.stream(dy2))
    else:
        grad.index_add_(0, idx, dy2.to(grad.dtype))


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tokens, weight):
        ctx.save_for_backward(tokens)
        ctx.wshape = weight.shape
        ctx.weight = weight
        return F.embedding(tokens, weight)

    @staticmethod
    def backward(ctx, dy):
        (tokens,) = ctx.saved_tensors
        weight = ctx.weight
        dy2 = dy.reshape(-1, dy.shape[-1])
        idx = tokens.reshape(-1)
        mg = getattr(weight, "main_grad", None)
        if mg is not None:
            if take_fresh(weight):  # a scatter-add needs zeros under it
                mg.zero_()
            _scatter_rows(mg, idx, dy2)
            return None, deliver_weight_grad(weight, None)
        g = torch.zeros(ctx.wshape, device=dy.device, dtype=torch.float32)
        _scatter_rows(g, idx, dy2)
        return None, g.to(weight.dtype)


def embedding(tokens, weight):
    return _EmbeddingFn.apply(tokens, weight)


class Embedding(torch.nn.Module):
    def __init__(self, num, dim, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.empty(num, dim, dtype=dtype, device=device))

    def forward(self, tokens):
        return embedding(tokens, self.weight)
