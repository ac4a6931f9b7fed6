"""Transposed copies of the linear weights for the data-gradient GEMM.

The backward's data gradient of ``y = x W^T`` is ``dX = dY W``.  As a
row-major GEMM that is the "NN" form, which hipBLASLt runs at 1.1-1.4 PF/s
on gfx950 at the Llama-3-8B shapes, against 1.44-1.58 PF/s for the
forward's ``x W^T`` form (profiles/r1_gemm_tuning_coldcache.log).  Keeping
``W^T`` next to ``W`` turns the data gradient into that faster form:
``dX = dY (W^T)^T``.

The copies live in ONE flat bf16 buffer (15 GB at Llama-3-8B: 288 GB of
HBM leaves room for it) and are refreshed right after the optimizer writes
the bf16 weights -- per gradient bucket, on the optimizer's stream -- by the
HBM-bound ``toa_transpose_bf16`` kernel (csrc/hip/transpose.hip, ~7 ms per
step at 8B).  ``param._toa_wt`` is the [in, out] view that
:func:`tf_operator_amd.ops.gemm.linear_dgrad` picks up.

Anything that rewrites the weights outside the optimizer (checkpoint load,
rank-0 broadcast) must call :meth:`refresh`; :class:`FlatParams` does it
through its ``on_param_change`` listeners.
"""
from __future__ import annotations

import os

import torch

from . import _lib


def transpose_into(dst: torch.Tensor, src: torch.Tensor):
    """dst[C, R] = src[R, C]^T (bf16; HIP kernel on the GPU)."""
    R, C = src.shape
    if (src.is_cuda and src.dtype == torch.bfloat16 and R % 64 == 0 and C % 64 == 0 and src.stride(1) == 1
            and dst.stride(1) == 1 and src.stride(0) % 8 == 0 and dst.stride(0) % 8 == 0
            and src.data_ptr() % 16 == 0 and dst.data_ptr() % 16 == 0):
        _lib.use_hip(src)
        _lib.call("toa_transpose_bf16", _lib.ptr(src), src.stride(0), _lib.ptr(dst), dst.stride(0), R, C,
                  _lib.stream(src))
    else:
        dst.copy_(src.t())
    return dst


def enabled_default(device) -> bool:
    return torch.device(device).type == "cuda" and os.environ.get("TOA_DGRAD_WT", "1") != "0"


class TransposedWeights:
    """Keeps ``param._toa_wt = param.t().contiguous()`` fresh for `params`
    (2-D weights managed by `flat`)."""

    def __init__(self, flat, params):
        self.flat = flat
        want = {id(p) for p in params}
        self.items = []  # (flat_offset, flat_end, param, wt_view)
        total = 0
        segs = [s for s in flat.segments if id(s.param) in want and s.param.dim() == 2]
        for s in segs:
            total += (s.numel + 63) // 64 * 64
        self.buf = torch.empty(max(total, 64), device=flat.device, dtype=flat.dtype)
        off = 0
        for s in segs:
            R, C = s.param.shape
            view = self.buf[off:off + s.numel].view(C, R)
            s.param._toa_wt = view
            self.items.append((s.offset, s.offset + s.numel, s.param, view))
            off += (s.numel + 63) // 64 * 64
        flat.on_param_change.append(self.refresh)
        self.refresh()

    @property
    def nbytes(self) -> int:
        return self.buf.numel() * self.buf.element_size()

    @torch.no_grad()
    def refresh(self, lo: int = 0, hi: int | None = None):
        """Re-transpose every weight overlapping flat range [lo, hi) on the
        current stream."""
        hi = self.flat.numel if hi is None else hi
        for a, b, p, view in self.items:
            if a < hi and b > lo:
                transpose_into(view, p.data)

    def detach(self):
        for _, _, p, _ in self.items:
            if hasattr(p, "_toa_wt"):
                del p._toa_wt
        if self.refresh in self.flat.on_param_change:
            self.flat.on_param_change.remove(self.refresh)
        self.items = []
