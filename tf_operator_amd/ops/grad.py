"""Weight-gradient delivery shared by every fused op.

A parameter managed by :class:`tf_operator_amd.parallel.flat.FlatParams` has
``param.main_grad`` -- a view into the model's single flat gradient buffer --
and optionally ``param._toa_ready`` (the gradient bucketer's hook).  Fused ops
write/accumulate weight gradients directly into ``main_grad`` (zero-copy:
the RCCL bucket all-reduce then runs on the flat buffer itself) and return
``None`` to autograd, so no per-parameter ``.grad`` tensors are materialised.
Parameters without ``main_grad`` get an ordinary autograd gradient.
"""
from __future__ import annotations

import torch


def take_fresh(param) -> bool:
    """True (once per step) when param.main_grad still holds the previous
    step's data (FlatParams.mark_fresh): its first gradient producer then
    overwrites instead of accumulating.  Producers whose kernel accumulates
    call this BEFORE launching it, to pick beta = 0 / accumulate = 0."""
    if param is not None and getattr(param, "_toa_fresh", False):
        param._toa_fresh = False
        return True
    return False


def deliver_weight_grad(param: torch.Tensor, grad: torch.Tensor | None):
    """Accumulate `grad` into param.main_grad if present (then return None),
    else return it (cast to the param dtype) for autograd.

    grad=None means the kernel already accumulated into main_grad.
    """
    mg = getattr(param, "main_grad", None)
    if mg is None:
        return None if grad is None else grad.to(param.dtype).view_as(param)
    if grad is not None:
        if take_fresh(param):
            mg.copy_(grad.view_as(mg))
        else:
            mg.add_(grad.view_as(mg).to(mg.dtype))
    hook = getattr(param, "_toa_ready", None)
    if hook is not None:
        hook(param)
    return None


def accumulate_mm(param: torch.Tensor, a: torch.Tensor, b: torch.Tensor):
    """param.main_grad += a @ b  (beta = 1, no temporary; = a @ b for the
    step's first producer, see take_fresh);
    falls back to returning a @ b when the param has no main_grad."""
    mg = getattr(param, "main_grad", None)
    if mg is None:
        return torch.mm(a, b).to(param.dtype).view_as(param)
    mg2 = mg.view(a.shape[0], b.shape[1])
    fresh = take_fresh(param)
    if a.dim() == 2 and a.stride(0) == 1 and a.t().is_contiguous():
        from . import gemm  # a = dy^T view: the tuned wgrad form

        gemm.wgrad_acc_(mg2, a.t(), b, beta=0.0 if fresh else 1.0)
    elif fresh:
        mg2.copy_(torch.mm(a, b))
    elif mg2.dtype == a.dtype:
        mg2.addmm_(a, b)
    else:
        mg2.add_(torch.mm(a, b).to(mg2.dtype))
    hook = getattr(param, "_toa_ready", None)
    if hook is not None:
        hook(param)
    return None
