"""Token embedding whose backward scatters straight into ``weight.main_grad``."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .grad import deliver_weight_grad


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
            if mg.dtype == dy2.dtype:
                mg.index_add_(0, idx, dy2)
            else:
                mg.index_add_(0, idx, dy2.to(mg.dtype))
            return None, deliver_weight_grad(weight, None)
        g = torch.zeros(ctx.wshape, device=dy.device, dtype=torch.float32)
        g.index_add_(0, idx, dy2.float())
        return None, g.to(weight.dtype)


def embedding(tokens, weight):
    return _EmbeddingFn.apply(tokens, weight)


class Embedding(torch.nn.Module):
    def __init__(self, num, dim, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.empty(num, dim, dtype=dtype, device=device))

    def forward(self, tokens):
        return embedding(tokens, self.weight)
