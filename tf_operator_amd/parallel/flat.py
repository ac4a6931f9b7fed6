"""Flat parameter / gradient / optimizer-state storage.

MI355X-first memory layout: with 288 GB of HBM per GPU a Llama-3-8B replica
(bf16 weights 16 GB + fp32 master 32 GB + Adam m/v 64 GB + bf16 grads 16 GB
= 128 GB) fits whole on every rank, so the framework keeps each of those
states as ONE contiguous buffer:

* every parameter's ``.data`` becomes a view into ``self.param`` (bf16),
* ``param.main_grad`` is a view into ``self.grad`` (the fused ops write
  weight gradients there directly),
* the optimizer streams ``self.master`` / ``self.exp_avg`` /
  ``self.exp_avg_sq`` with one kernel per contiguous weight-decay run.

Parameters are laid out in *backward order* (first gradient produced =
lowest offset) so gradient buckets become ready front-to-back and their
RCCL all-reduces overlap the rest of backward.
"""
from __future__ import annotations

import dataclasses

import torch

ALIGN = 64  # elements; keeps every view 128-B aligned for 16-B vector access


def _round_up(n, a=ALIGN):
    return (n + a - 1) // a * a


@dataclasses.dataclass
class Segment:
    name: str
    param: torch.nn.Parameter
    offset: int
    numel: int
    decay: bool


class FlatParams:
    def __init__(self, params, names=None, no_decay=None, grad_dtype=None, master=True):
        params = list(params)
        seen = {}
        uniq = []
        for p in params:
            if id(p) in seen:
                seen[id(p)] += 1
                continue
            seen[id(p)] = 1
            uniq.append(p)
        names = names or {}
        dev = uniq[0].device
        dtype = uniq[0].dtype
        self.dtype = dtype
        self.device = dev
        self.segments: list[Segment] = []
        off = 0
        for p in uniq:
            n = p.numel()
            decay = not (no_decay(p) if no_decay else p.dim() == 1)
            self.segments.append(Segment(names.get(id(p), f"p{len(self.segments)}"), p, off, n, decay))
            off += _round_up(n)
        self.numel = max(off, ALIGN)
        gdt = grad_dtype or dtype
        self.param = torch.zeros(self.numel, device=dev, dtype=dtype)
        self.grad = torch.zeros(self.numel, device=dev, dtype=gdt)
        for s in self.segments:
            view = self.param[s.offset:s.offset + s.numel].view_as(s.param)
            view.copy_(s.param.data)
            s.param.data = view
            s.param.main_grad = self.grad[s.offset:s.offset + s.numel].view_as(s.param)
            s.param._toa_uses = seen[id(s.param)]
        self.master = None
        if master:
            self.master = self.param.float() if dtype != torch.float32 else self.param.clone()
        self.exp_avg = None
        self.exp_avg_sq = None
        # callbacks run after the bf16 weights are rewritten outside the
        # optimizer (checkpoint load, broadcast): derived copies such as
        # ops.wt.TransposedWeights re-derive themselves
        self.on_param_change = []

    def params_changed(self):
        for fn in list(self.on_param_change):
            fn()

    def decay_runs(self):
        """Contiguous [start, end, decay] runs (for per-run optimizer launches)."""
        runs = []
        for s in self.segments:
            end = s.offset + _round_up(s.numel)
            if runs and runs[-1][2] == s.decay and runs[-1][1] == s.offset:
                runs[-1][1] = end
            else:
                runs.append([s.offset, end, s.decay])
        if runs:
            runs[-1][1] = self.numel
        return runs

    def zero_grad(self):
        self.grad.zero_()

    def state_dict(self):
        return {
            "master": self.master,
            "exp_avg": self.exp_avg,
            "exp_avg_sq": self.exp_avg_sq,
            "layout": [(s.name, s.offset, s.numel) for s in self.segments],
        }

    def load_state_dict(self, sd):
        layout = [(s.name, s.offset, s.numel) for s in self.segments]
        if [tuple(x) for x in sd["layout"]] != layout:
            raise ValueError("flat layout mismatch between checkpoint and model")
        if sd.get("master") is not None and self.master is not None:
            self.master.copy_(sd["master"])
            self.param.copy_(self.master.to(self.param.dtype))
        for k in ("exp_avg", "exp_avg_sq"):
            if sd.get(k) is not None:
                if getattr(self, k) is None:
                    setattr(self, k, torch.zeros_like(sd[k], device=self.device))
                getattr(self, k).copy_(sd[k])
        self.params_changed()
