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

The fp32 state need not cover the whole flat buffer: :meth:`shard_state`
keeps master / m / v only for the flat ranges this rank updates (ZeRO-1,
parallel/zero.py), packed back to back ("compact" storage), which frees
12 B/param x (1 - 1/world) of HBM.  ``state_ranges`` lists the covered
flat ranges and :meth:`state_index` maps a flat offset into the compact
buffers.

Parameters are laid out in *backward order* (first gradient produced =
lowest offset) so gradient buckets become ready front-to-back and their
RCCL all-reduces overlap the rest of backward.
"""
from __future__ import annotations

import bisect
import dataclasses
import os

import torch

ALIGN = 64  # elements; keeps every view 128-B aligned for 16-B vector access


def _uncovered(x: int, y: int, covered) -> list:
    """Sub-ranges of [x, y) not in any of the (disjoint) `covered` ranges."""
    out = [(x, y)]
    for a, b in covered:
        nxt = []
        for p, q in out:
            if b <= p or a >= q:
                nxt.append((p, q))
                continue
            if p < a:
                nxt.append((p, a))
            if b < q:
                nxt.append((b, q))
        out = nxt
    return out


def _as_tensor(x):
    """numpy (incl. read-only checkpoint memmaps) or torch -> torch, no copy."""
    if torch.is_tensor(x):
        return x
    import warnings

    import numpy as np

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # read-only memmap: only ever read
        return torch.from_numpy(np.ascontiguousarray(x))


def _round_up(n, a=ALIGN):
    return (n + a - 1) // a * a


@dataclasses.dataclass
class Segment:
    name: str
    param: torch.nn.Parameter
    offset: int
    numel: int
    decay: bool
    nhwc: bool = False  # a channels-last 4D weight: stored N,H,W,C in the flat buffer


def _channels_last(p: torch.Tensor) -> bool:
    if os.environ.get("TOA_FLAT_NHWC") == "0":  # A/B switch: NCHW views, as before
        return False
    return p.dim() == 4 and not p.is_contiguous() and p.is_contiguous(memory_format=torch.channels_last)


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
            self.segments.append(Segment(names.get(id(p), f"p{len(self.segments)}"), p, off, n, decay,
                                         _channels_last(p)))
            off += _round_up(n)
        self.numel = max(off, ALIGN)
        gdt = grad_dtype or dtype
        self.param = torch.zeros(self.numel, device=dev, dtype=dtype)
        self.grad = torch.zeros(self.numel, device=dev, dtype=gdt)
        for s in self.segments:
            # channels-last conv weights keep their memory format in the flat
            # buffers: no per-forward layout copy of the weight, and the
            # channels-last gradient adds into main_grad without a permute
            view = self._view(self.param, s)
            view.copy_(s.param.data)
            s.param.data = view
            s.param.main_grad = self._view(self.grad, s)
            s.param._toa_uses = seen[id(s.param)]
        self.master = None
        if master:
            self.master = self.param.float() if dtype != torch.float32 else self.param.clone()
        # flat ranges covered by master / exp_avg / exp_avg_sq, and where each
        # starts in those (compact) buffers
        self.state_ranges = [(0, self.numel)]
        self._state_lo = [0]
        self._state_off = [0]
        self.state_numel = self.numel
        self.exp_avg = None
        self.exp_avg_sq = None
        # callbacks run after the bf16 weights are rewritten outside the
        # optimizer (checkpoint load, broadcast): derived copies such as
        # ops.wt.TransposedWeights re-derive themselves
        self.on_param_change = []

    # ------------------------------------------------------------------ sharded state
    @property
    def state_sharded(self) -> bool:
        return self.state_ranges != [(0, self.numel)]

    @torch.no_grad()
    def shard_state(self, ranges):
        """Keep the fp32 state only for flat `ranges` (sorted, disjoint),
        packed in that order.  Existing master / moments are carried over."""
        ranges = [(int(lo), int(hi)) for lo, hi in ranges]
        offs, tot = [], 0
        for lo, hi in ranges:
            offs.append(tot)
            tot += hi - lo
        new = {}
        for k in ("master", "exp_avg", "exp_avg_sq"):
            old = getattr(self, k)
            if old is None:
                continue
            t = torch.empty(tot, device=old.device, dtype=old.dtype)
            for (lo, hi), o in zip(ranges, offs):
                t[o:o + hi - lo].copy_(old[self.state_index(lo):self.state_index(lo) + hi - lo])
            new[k] = t
        for k in ("master", "exp_avg", "exp_avg_sq"):
            setattr(self, k, None)
        for k, t in new.items():
            setattr(self, k, t)
        self.state_ranges = ranges
        self._state_lo = [lo for lo, _ in ranges]
        self._state_off = offs
        self.state_numel = tot

    def state_index(self, a: int) -> int:
        """Offset in the compact state buffers of flat element `a`."""
        i = bisect.bisect_right(self._state_lo, a) - 1
        if i < 0 or a >= self.state_ranges[i][1]:
            raise IndexError(f"flat offset {a} has no fp32 state on this rank")
        return self._state_off[i] + a - self.state_ranges[i][0]

    def state_view(self, t, lo: int, hi: int):
        """View of compact state tensor `t` for flat range [lo, hi) (inside one state range)."""
        i = self.state_index(lo)
        return t[i:i + hi - lo]

    @torch.no_grad()
    def master_from_param(self):
        """Re-derive the fp32 master of every held range from the bf16 weights."""
        if self.master is None:
            return
        for lo, hi in self.state_ranges:
            self.state_view(self.master, lo, hi).copy_(self.param[lo:hi].float())

    @torch.no_grad()
    def param_from_master(self):
        for lo, hi in self.state_ranges:
            self.param[lo:hi].copy_(self.state_view(self.master, lo, hi).to(self.param.dtype))

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

    def mark_fresh(self):
        """Start a step WITHOUT zeroing the gradient buffer: every parameter's
        first gradient producer of the step overwrites its main_grad slice
        instead of accumulating (ops/grad.py take_fresh).  Saves the 2 B /
        parameter zeroing pass (16 GB at Llama-3-8B)."""
        for s in self.segments:
            s.param._toa_fresh = True

    def zero_stale(self):
        """After backward: zero the main_grad of parameters no producer wrote
        since mark_fresh() (unused parameters), so they hold no stale data."""
        for s in self.segments:
            if getattr(s.param, "_toa_fresh", False):
                s.param.main_grad.zero_()
                s.param._toa_fresh = False

    def state_dict(self):
        """This rank's fp32 state (compact) and where it belongs in the flat
        buffer.  World-size independent when combined with the other ranks'
        (see :func:`load_state_shards`)."""
        return {
            "master": self.master,
            "exp_avg": self.exp_avg,
            "exp_avg_sq": self.exp_avg_sq,
            "state_ranges": [tuple(r) for r in self.state_ranges],
            "numel": self.numel,
            "layout": self.layout(),
        }

    @staticmethod
    def _view(buf: torch.Tensor, s: Segment) -> torch.Tensor:
        seg = buf[s.offset:s.offset + s.numel]
        if s.nhwc:
            n, c, h, w = s.param.shape
            return seg.view(n, h, w, c).permute(0, 3, 1, 2)
        return seg.view(s.param.shape)

    def layout(self):
        # a channels-last segment's element order differs: name it, so a
        # checkpoint of the other order is refused instead of permuted
        return [(s.name + ("@nhwc" if s.nhwc else ""), s.offset, s.numel) for s in self.segments]

    def check_layout(self, layout):
        if [tuple(x) for x in layout] != self.layout():
            raise ValueError("flat layout mismatch between checkpoint and model")

    @torch.no_grad()
    def load_state_shards(self, shards, set_params="held"):
        """Fill this rank's state ranges from any set of saved shards
        (``state_dict()`` outputs of ANY world size; tensors may be CPU,
        device or numpy memmaps) that together cover them.  ``set_params``:
        "held" re-derives the bf16 weights of the held ranges, "all" of every
        range the shards cover (then no weight all-gather is needed)."""
        covered, pcovered = [], []  # ranges already restored (state / bf16 weights)
        for sh in shards:
            if "layout" in sh:
                self.check_layout(sh["layout"])
            src_off = 0
            for lo, hi in sh["state_ranges"]:
                lo, hi = int(lo), int(hi)
                for (a, b) in self.state_ranges:
                    x, y = max(a, lo), min(b, hi)
                    # replicated (non-ZeRO) ranks each saved the whole state:
                    # copy every range once, from the first share that has it
                    for p, q in (_uncovered(x, y, covered) if x < y and sh.get("master") is not None else []):
                        for k in ("master", "exp_avg", "exp_avg_sq"):
                            src = sh.get(k)
                            if src is None:
                                continue
                            if getattr(self, k) is None:
                                setattr(self, k, torch.zeros(self.state_numel, device=self.device,
                                                             dtype=torch.float32))
                            piece = _as_tensor(src[src_off + p - lo:src_off + q - lo])
                            self.state_view(getattr(self, k), p, q).copy_(piece, non_blocking=False)
                        covered.append((p, q))
                if set_params == "all" and sh.get("master") is not None:
                    for p, q in _uncovered(lo, hi, pcovered):
                        piece = _as_tensor(sh["master"][src_off + p - lo:src_off + q - lo])
                        self.param[p:q].copy_(piece.to(self.device).to(self.param.dtype))
                        pcovered.append((p, q))
                src_off += hi - lo
        need = sum(b - a for a, b in self.state_ranges)
        if self.master is not None and sum(b - a for a, b in covered) != need:
            raise ValueError("checkpoint shards do not cover this rank's optimizer state")
        if set_params == "held":
            self.param_from_master()

    def load_state_dict(self, sd):
        self.load_state_shards([sd], set_params="all")
        self.params_changed()
