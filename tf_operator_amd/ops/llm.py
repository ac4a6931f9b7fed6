"""Transformer ops for the Llama trainer: RoPE+relayout, SwiGLU(+down proj),
fused cross-entropy and causal attention.

HIP kernels: csrc/hip/llm.hip (RoPE, SwiGLU, cross-entropy) and
csrc/hip/attention.hip (flash attention, when built); CPU tensors take the
PyTorch reference path (used by the numerics tests).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from . import _lib
from . import gemm
from .grad import accumulate_mm


# ---------------------------------------------------------------------------
# RoPE
# ---------------------------------------------------------------------------
def rope_tables(seq_len, head_dim, theta=500000.0, device=None, scaling=None):
    """cos/sin [S, D/2] fp32 (Llama-3 frequencies; optional llama3 rope scaling dict)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling:
        factor = scaling.get("factor", 8.0)
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        wl = 2 * math.pi / inv
        lo_wl, hi_wl = old / lo, old / hi
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(seq_len, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def _rope_ref(x, cos, sin):
    # x [B, H, S, D]
    d2 = x.shape[-1] // 2
    x1, x2 = x[..., :d2].float(), x[..., d2:].float()
    c, s = cos[None, None], sin[None, None]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)


class _RopeQKV(torch.autograd.Function):
    """qkv [B*S, (Hq+2Hkv)*D] -> q [B,Hq,S,D], k/v [B,Hkv*rep,S,D]."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, B, S, Hq, Hkv, D, rep):
        ctx.dims = (B, S, Hq, Hkv, D, rep)
        ctx.dtype = qkv.dtype
        ctx.save_for_backward(cos, sin)
        Hk = Hkv * rep
        if _lib.use_hip(qkv):
            qkv = qkv.contiguous()
            q = torch.empty(B, Hq, S, D, device=qkv.device, dtype=qkv.dtype)
            k = torch.empty(B, Hk, S, D, device=qkv.device, dtype=qkv.dtype)
            v = torch.empty(B, Hk, S, D, device=qkv.device, dtype=qkv.dtype)
            _lib.call("toa_rope_fwd", _lib.ptr(qkv), _lib.ptr(cos), _lib.ptr(sin), _lib.ptr(q), _lib.ptr(k),
                      _lib.ptr(v), B, S, Hq, Hkv, D, rep, _lib.stream(qkv))
            return q, k, v
        x = qkv.view(B, S, Hq + 2 * Hkv, D).transpose(1, 2)
        q = _rope_ref(x[:, :Hq], cos, sin).to(qkv.dtype)
        k = _rope_ref(x[:, Hq:Hq + Hkv], cos, sin).to(qkv.dtype)
        v = x[:, Hq + Hkv:]
        k = k.repeat_interleave(rep, dim=1).contiguous()
        v = v.repeat_interleave(rep, dim=1).contiguous()
        return q.contiguous(), k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin = ctx.saved_tensors
        B, S, Hq, Hkv, D, rep = ctx.dims
        if _lib.use_hip(dq):
            dq, dk, dv = dq.contiguous(), dk.contiguous(), dv.contiguous()
            dqkv = torch.empty(B * S, (Hq + 2 * Hkv) * D, device=dq.device, dtype=dq.dtype)
            _lib.call("toa_rope_bwd", _lib.ptr(dq), _lib.ptr(dk), _lib.ptr(dv), _lib.ptr(cos), _lib.ptr(sin),
                      _lib.ptr(dqkv), B, S, Hq, Hkv, D, rep, _lib.stream(dq))
            return dqkv, None, None, None, None, None, None, None, None
        dk = dk.float().view(B, Hkv, rep, S, D).sum(2)
        dv = dv.float().view(B, Hkv, rep, S, D).sum(2)
        # inverse rotation = rotation by -theta
        dq = _rope_ref(dq.float(), cos, -sin)
        dk = _rope_ref(dk, cos, -sin)
        out = torch.cat([dq, dk, dv], 1).transpose(1, 2).reshape(B * S, (Hq + 2 * Hkv) * D)
        return out.to(ctx.dtype), None, None, None, None, None, None, None, None


def rope_qkv(qkv, cos, sin, B, S, Hq, Hkv, D, rep=None):
    rep = Hq // Hkv if rep is None else rep
    return _RopeQKV.apply(qkv, cos, sin, B, S, Hq, Hkv, D, rep)


# ---------------------------------------------------------------------------
# SwiGLU (+ down projection, recomputing the activation in backward)
# ---------------------------------------------------------------------------
def swiglu(gu):
    F_ = gu.shape[-1] // 2
    if _lib.use_hip(gu):
        gu = gu.contiguous()
        T = gu.numel() // (2 * F_)
        out = torch.empty(*gu.shape[:-1], F_, device=gu.device, dtype=gu.dtype)
        _lib.call("toa_swiglu_fwd", _lib.ptr(gu), _lib.ptr(out), T, F_, _lib.stream(gu))
        return out
    g, u = gu[..., :F_].float(), gu[..., F_:].float()
    return (F.silu(g) * u).to(gu.dtype)


def swiglu_bwd(dout, gu):
    F_ = gu.shape[-1] // 2
    if _lib.use_hip(gu):
        dout = dout.contiguous()
        T = gu.numel() // (2 * F_)
        dgu = torch.empty_like(gu)
        _lib.call("toa_swiglu_bwd", _lib.ptr(dout), _lib.ptr(gu), _lib.ptr(dgu), T, F_, _lib.stream(gu))
        return dgu
    g, u, d = gu[..., :F_].float(), gu[..., F_:].float(), dout.float()
    sg = torch.sigmoid(g)
    du = d * g * sg
    dg = d * u * sg * (1 + g * (1 - sg))
    return torch.cat([dg, du], -1).to(gu.dtype)


_SWIGLU_RECOMPUTE = os.environ.get("TOA_SWIGLU_RECOMPUTE", "0") == "1"


class _SwiGLUDown(torch.autograd.Function):
    """out = swiglu(gu) @ Wd^T.  Saves gu and the [T, F] activation s for the
    down-projection's weight gradient (470 MB/layer at Llama-3-8B x 16k
    tokens, ~15 GB for 32 layers -- HBM has room at 288 GB); with
    TOA_SWIGLU_RECOMPUTE=1 s is recomputed in backward instead (one extra
    SwiGLU pass per layer, ~8 ms/step)."""

    @staticmethod
    def forward(ctx, gu, wd):
        s = swiglu(gu)
        ctx.save_for_backward(gu, wd, None if _SWIGLU_RECOMPUTE else s)
        return gemm.linear_fwd(s.reshape(-1, s.shape[-1]), wd).view(*s.shape[:-1], wd.shape[0])

    @staticmethod
    def backward(ctx, dout):
        gu, wd, s = ctx.saved_tensors
        if s is None:
            s = swiglu(gu)
        d2 = dout.reshape(-1, dout.shape[-1])
        dw = accumulate_mm(wd, d2.t(), s.reshape(-1, s.shape[-1]))
        ds = gemm.linear_dgrad(d2, wd).view(*dout.shape[:-1], wd.shape[1])
        del s
        dgu = swiglu_bwd(ds, gu)
        return dgu, dw


def swiglu_down(gu, wd):
    return _SwiGLUDown.apply(gu, wd)


class _SwiGLUMLP(torch.autograd.Function):
    """out = swiglu(x Wgu^T) Wd^T with the SwiGLU fused into the GEMMs
    (ops/gemm.py ``swiglu_gate_up`` / ``swiglu_down_dgrad``,
    csrc/asm/gemm_gen.py): the gate|up GEMM writes gu and s = silu(gate) *
    up, and the down projection's data gradient emits dgu directly -- no
    separate SwiGLU pass over the [T, 2F] activations in either direction.
    Weight gradients land in the flat buffer as in ``ops.linear``."""

    @staticmethod
    def forward(ctx, x, wgu, wd, residual=None):
        x2 = x.reshape(-1, x.shape[-1])
        r = gemm.swiglu_gate_up(x2, wgu)
        gu, s = r if r is not None else (None, None)
        if gu is None:
            gu = gemm.linear_fwd(x2, wgu)
            s = swiglu(gu)
        ctx.save_for_backward(x, wgu, wd, gu, s)
        ctx.has_res = residual is not None
        if residual is not None:   # + residual in the down projection's epilogue (toa_gemm_asm_resadd)
            r2 = residual.reshape(s.shape[0], -1)
            out = torch.empty_like(r2)
            _lib.call("toa_gemm_asm_resadd", _lib.ptr(s), s.stride(0), _lib.ptr(wd), wd.stride(0), _lib.ptr(out),
                      out.stride(0), _lib.ptr(r2), s.shape[0], wd.shape[0], s.shape[1], _lib.stream(s))
            return out.view_as(residual)
        return gemm.linear_fwd(s, wd).view(*x.shape[:-1], wd.shape[0])

    @staticmethod
    def backward(ctx, dout):
        x, wgu, wd, gu, s = ctx.saved_tensors
        d2 = dout.reshape(-1, dout.shape[-1])
        dwd = accumulate_mm(wd, d2.t(), s)
        del s
        dgu = gemm.swiglu_down_dgrad(d2, wd, gu)
        if dgu is None:
            dgu = swiglu_bwd(gemm.linear_dgrad(d2, wd), gu)
        del gu
        x2 = x.reshape(-1, x.shape[-1])
        dx = gemm.linear_dgrad(dgu, wgu).view_as(x) if ctx.needs_input_grad[0] else None
        dwgu = accumulate_mm(wgu, dgu.t(), x2)
        return dx, dwgu, dwd, (dout if ctx.has_res else None)


def swiglu_mlp(x, wgu, wd, residual=None):
    """The Llama MLP, x -> swiglu(x Wgu^T) Wd^T (+ residual, added in the
    down projection's epilogue: see swiglu_mlp_resadd_ok), fused where the
    assembly GEMM takes the shapes (policy ``asm``: the default since round
    5, see ops.gemm.resolve_auto), else the two-GEMM + SwiGLU path (``nosk``)."""
    if gemm.mode() == "asm":
        return _SwiGLUMLP.apply(x, wgu, wd, residual)
    from .linear import linear

    out = swiglu_down(linear(x, wgu), wd)
    return out if residual is None else out + residual


def resadd_fused_enabled() -> bool:
    """Residual add in the GEMM epilogues (TOA_RESADD_FUSED=0 turns it off):
    -2.75 +- 0.49 ms/step (profiles/r6_ra3).  The next norm runs presummed,
    through its module call so ZeRO-1's gather waits still fire (ops/norm)."""
    return os.environ.get("TOA_RESADD_FUSED", "1") != "0"


def swiglu_mlp_resadd_ok(x, wd, residual) -> bool:
    """The residual add fits the fused MLP's down-projection epilogue."""
    T = x.reshape(-1, x.shape[-1]).shape[0]
    return (x.is_cuda and residual.dtype == wd.dtype == torch.bfloat16 and gemm.mode() == "asm"
            and wd.is_contiguous() and residual.is_contiguous() and T % 256 == 0 and wd.shape[0] % 256 == 0
            and wd.shape[1] % 64 == 0 and residual.numel() == T * wd.shape[0]
            and _lib.has("toa_gemm_asm_resadd") and resadd_fused_enabled())


# ---------------------------------------------------------------------------
# Cross entropy (mean over non-ignored tokens)
# ---------------------------------------------------------------------------
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, inplace_grad):
        V = logits.shape[-1]
        x = logits.reshape(-1, V)
        t = target.reshape(-1).to(torch.int64).contiguous()
        rows = x.shape[0]
        if _lib.use_hip(x):
            if x.stride(-1) != 1:
                x = x.contiguous()
            loss = torch.empty(rows, device=x.device, dtype=torch.float32)
            lse = torch.empty(rows, device=x.device, dtype=torch.float32)
            _lib.call("toa_xent_fwd", _lib.dtype_code(x), _lib.ptr(x), _lib.ptr(t), _lib.ptr(loss), _lib.ptr(lse),
                      rows, V, x.stride(0), int(ignore_index), _lib.stream(x))
        else:
            xf = x.float()
            lse = torch.logsumexp(xf, -1)
            valid = t != ignore_index
            tt = t.clamp(0, V - 1)
            loss = torch.where(valid, lse - xf.gather(1, tt[:, None]).squeeze(1), torch.zeros_like(lse))
        n_valid = (t != ignore_index).sum().float()
        ctx.save_for_backward(x, t, lse, n_valid)
        ctx.ignore_index = ignore_index
        ctx.inplace = inplace_grad
        ctx.shape = logits.shape
        return loss.sum() / n_valid.clamp(min=1.0)

    @staticmethod
    def backward(ctx, g):
        x, t, lse, n_valid = ctx.saved_tensors
        V = x.shape[-1]
        if _lib.use_hip(x):
            dx = x if ctx.inplace else torch.empty_like(x)
            go = g.reshape(1).float().contiguous()
            nv = n_valid.reshape(1).contiguous()
            _lib.call("toa_xent_bwd", _lib.dtype_code(x), _lib.ptr(x), _lib.ptr(t), _lib.ptr(lse), _lib.ptr(go),
                      _lib.ptr(nv), _lib.ptr(dx), x.shape[0], V, x.stride(0), int(ctx.ignore_index), _lib.stream(x))
        else:
            p = torch.softmax(x.float(), -1)
            valid = t != ctx.ignore_index
            p[torch.arange(x.shape[0]), t.clamp(0, V - 1)] -= 1.0
            p = p * valid[:, None].float() * (g / n_valid.clamp(min=1.0))
            dx = p.to(x.dtype)
        return dx.view(ctx.shape), None, None, None


def cross_entropy(logits, target, ignore_index=-100, inplace_grad=False):
    """Mean token cross entropy.  ``inplace_grad=True`` writes the logits
    gradient over the logits buffer (saves one [tokens, vocab] tensor)."""
    return _CrossEntropy.apply(logits, target, ignore_index, inplace_grad)


# ---------------------------------------------------------------------------
# Causal attention
# ---------------------------------------------------------------------------
ATTN_HEAD_DIMS = (64, 128)  # the HIP kernel's head-dim instantiations (csrc/hip/attention.hip)


def _attn_hip_ok(q):
    return (q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in ATTN_HEAD_DIMS and _lib.has("toa_attn_fwd")
            and _lib.has("toa_attn_bwd"))


class _FlashAttn(torch.autograd.Function):
    """HIP flash attention.  bshd=True returns O as [B, S, H, D] (what the
    output projection reads) and takes dO in that layout: no transpose copies."""

    @staticmethod
    def forward(ctx, q, k, v, scale, bshd=False):
        B, H, S, D = q.shape
        Hk = k.shape[1]
        o = torch.empty(B, S, H, D, device=q.device, dtype=q.dtype) if bshd else torch.empty_like(q)
        lse = torch.empty(B, H, S, device=q.device, dtype=torch.float32)
        _lib.call("toa_attn_fwd", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(o), _lib.ptr(lse), B, H, Hk, S, D,
                  1 | (2 if bshd else 0), float(scale), _lib.stream(q))
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.scale = scale
        ctx.bshd = bshd
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        return (*_attn_bwd(q, k, v, o, lse, do.contiguous(), ctx.scale, ctx.bshd), None, None)


def _attn_ws(B, H, S, D, device):
    """Workspace of the dS-through-HBM backward form (attention.hip, the
    default where S % 256 == 0): the lower-triangular dS blocks, 3.2 GB at the
    Llama-3-8B bench shape.  None when the form in force needs none."""
    nws = _lib.call_ret("toa_attn_bwd_ws_bytes", B, H, S, D) if _lib.has("toa_attn_bwd_ws_bytes") else 0
    return torch.empty(nws, device=device, dtype=torch.uint8) if nws > 0 else None


def _attn_bwd(q, k, v, o, lse, do, scale, bshd):
    B, H, S, D = q.shape
    Hk = k.shape[1]
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    delta = torch.empty(B, H, S, device=q.device, dtype=torch.float32)
    ws = _attn_ws(B, H, S, D, q.device)
    _lib.call("toa_attn_bwd", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(o), _lib.ptr(do), _lib.ptr(lse),
              _lib.ptr(delta), _lib.ptr(ws), _lib.ptr(dq), _lib.ptr(dk), _lib.ptr(dv), B, H, Hk, S, D,
              1 | (2 if bshd else 0), float(scale), _lib.stream(q))
    return dq, dk, dv


# TOA_ATTN_ROPE_FUSED=0: RoPE backward as its own pass even where the fused
# epilogues could take it (A/B)
_ROPE_FUSED_BWD = os.environ.get("TOA_ATTN_ROPE_FUSED", "1") != "0"


class _RopeAttn(torch.autograd.Function):
    """RoPE + causal attention as one autograd node (packed K/V, one copy
    per kv head).  Forward: toa_rope_fwd, then the flash-attention forward.
    Backward: d(qkv) straight from the attention backward's epilogues,
    rotated back there (toa_attn_bwd_rope: no dq / dk / dv tensors, no RoPE
    backward pass); where that form is off (ragged S, TOA_ATTN_BWD=split)
    the attention backward + toa_rope_bwd."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, B, S, Hq, Hkv, D, scale, bshd):
        qkv = qkv.contiguous()
        q = torch.empty(B, Hq, S, D, device=qkv.device, dtype=qkv.dtype)
        k = torch.empty(B, Hkv, S, D, device=qkv.device, dtype=qkv.dtype)
        v = torch.empty(B, Hkv, S, D, device=qkv.device, dtype=qkv.dtype)
        _lib.call("toa_rope_fwd", _lib.ptr(qkv), _lib.ptr(cos), _lib.ptr(sin), _lib.ptr(q), _lib.ptr(k), _lib.ptr(v),
                  B, S, Hq, Hkv, D, 1, _lib.stream(qkv))
        o = torch.empty(B, S, Hq, D, device=q.device, dtype=q.dtype) if bshd else torch.empty_like(q)
        lse = torch.empty(B, Hq, S, device=q.device, dtype=torch.float32)
        _lib.call("toa_attn_fwd", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(o), _lib.ptr(lse), B, Hq, Hkv, S, D,
                  1 | (2 if bshd else 0), float(scale), _lib.stream(q))
        ctx.save_for_backward(q, k, v, o, lse, cos, sin)
        ctx.scale, ctx.bshd = scale, bshd
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, cos, sin = ctx.saved_tensors
        dqkv = _rope_attn_dqkv(q, k, v, o, lse, cos, sin, do, ctx.scale, ctx.bshd)
        return dqkv, None, None, None, None, None, None, None, None, None


# (dO data_ptr, numel, -delta rows) left by the output projection's backward
# (_AttnOutProj: toa_gemm_asm_delta) for the attention backward that follows
_PENDING_DELTA = None


def _rope_attn_dqkv(q, k, v, o, lse, cos, sin, do, scale, bshd):
    """d(qkv) [B S, (Hq + 2 Hkv) D] of RoPE + causal attention from dO."""
    global _PENDING_DELTA
    B, Hq, S, D = q.shape
    Hkv = k.shape[1]
    do = do.contiguous()
    pend, _PENDING_DELTA = _PENDING_DELTA, None
    dqkv = torch.empty(B * S, (Hq + 2 * Hkv) * D, device=q.device, dtype=q.dtype)
    flags = 1 | (2 if bshd else 0)
    ws = _attn_ws(B, Hq, S, D, q.device)
    if ws is not None and _ROPE_FUSED_BWD and _lib.has("toa_attn_bwd_rope"):
        if pend is not None and bshd and pend[0] == do.data_ptr() and pend[1] == do.numel():
            delta = pend[2].view(B, Hq, S)   # the -delta rows from the projection's GEMM: no delta pass
            flags |= 4
        else:
            delta = torch.empty(B, Hq, S, device=q.device, dtype=torch.float32)
        rc = _lib.call_ret("toa_attn_bwd_rope", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(o), _lib.ptr(do),
                           _lib.ptr(lse), _lib.ptr(delta), _lib.ptr(ws), _lib.ptr(cos), _lib.ptr(sin),
                           _lib.ptr(dqkv), B, Hq, Hkv, S, D, flags, float(scale), _lib.stream(q))
        if rc == 0:
            return dqkv
        if rc != 801:  # hipErrorNotSupported: take the two-pass path below
            raise RuntimeError(f"toa_attn_bwd_rope failed with hipError {rc}")
    del ws
    dq, dk, dv = _attn_bwd(q, k, v, o, lse, do, scale, bshd)
    _lib.call("toa_rope_bwd", _lib.ptr(dq), _lib.ptr(dk), _lib.ptr(dv), _lib.ptr(cos), _lib.ptr(sin),
              _lib.ptr(dqkv), B, S, Hq, Hkv, D, 1, _lib.stream(q))
    return dqkv


class _AttnOutProj(torch.autograd.Function):
    """The attention output projection linear(o, wo) whose backward also
    writes the attention backward's -delta rows: its data-gradient GEMM
    (toa_gemm_asm_delta) dots each stored dO row with O per head in its
    epilogue, so the attention backward (_rope_attn_dqkv) skips its pass over
    dO and O.  Elsewhere (no W^T copy, other shapes) the plain linear."""

    @staticmethod
    def forward(ctx, o2, wo, B, S, H, residual=None):
        ctx.save_for_backward(o2, wo)
        ctx.dims = (B, S, H)
        ctx.has_res = residual is not None
        if residual is None:
            return gemm.linear_fwd(o2, wo)
        # the residual add in the GEMM's epilogue (toa_gemm_asm_resadd): out = o2 wo^T + residual
        r2 = residual.reshape(o2.shape[0], -1)
        out = torch.empty_like(r2)
        _lib.call("toa_gemm_asm_resadd", _lib.ptr(o2), o2.stride(0), _lib.ptr(wo), wo.stride(0), _lib.ptr(out),
                  out.stride(0), _lib.ptr(r2), o2.shape[0], wo.shape[0], o2.shape[1], _lib.stream(o2))
        return out.view_as(residual)

    @staticmethod
    def backward(ctx, dy):
        global _PENDING_DELTA
        from .grad import accumulate_mm

        o2, wo = ctx.saved_tensors
        B, S, H = ctx.dims
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = None
        wt = getattr(wo, "_toa_wt", None)
        if (ctx.needs_input_grad[0] and wt is not None and dy2.stride(-1) == 1 and wt.stride(-1) == 1
                and o2.is_contiguous() and os.environ.get("TOA_ATTN_DELTA_FUSED", "1") != "0"
                and _lib.has("toa_gemm_asm_delta") and gemm.mode() == "asm"):
            T, N = o2.shape
            dx = torch.empty_like(o2)
            nd = torch.empty(B * H * S, device=o2.device, dtype=torch.float32)
            rc = _lib.call_ret("toa_gemm_asm_delta", _lib.ptr(dy2), dy2.stride(0), _lib.ptr(wt), wt.stride(0),
                               _lib.ptr(dx), dx.stride(0), _lib.ptr(o2), _lib.ptr(nd), T, N, dy2.shape[1], S, H,
                               _lib.stream(dy2))
            if rc == 0:
                _PENDING_DELTA = (dx.data_ptr(), dx.numel(), nd)
            elif rc == 1:   # hipErrorInvalidValue: a shape it does not take
                dx = None
            else:
                raise RuntimeError(f"toa_gemm_asm_delta failed with hipError {rc}")
        if dx is None and ctx.needs_input_grad[0]:
            dx = gemm.linear_dgrad(dy2, wo)
        dw = accumulate_mm(wo, dy2.t(), o2)
        return dx, dw, None, None, None, (dy if ctx.has_res else None)


def attn_out_proj(o2, wo, B, S, H, residual=None):
    """linear(o2, wo) (+ residual, added in the GEMM's epilogue) for the
    attention output o2 [B S, H 128]; its backward hands the attention
    backward its delta rows."""
    return _AttnOutProj.apply(o2, wo, B, S, H, residual)


def attn_out_proj_resadd_ok(o2, wo, residual) -> bool:
    """The residual add fits the output projection's epilogue (TOA_RESADD_FUSED)."""
    return (o2.is_cuda and o2.dtype == wo.dtype == residual.dtype == torch.bfloat16 and gemm.mode() == "asm"
            and o2.is_contiguous() and wo.is_contiguous() and residual.is_contiguous()
            and o2.shape[0] % 256 == 0 and wo.shape[0] % 256 == 0 and o2.shape[1] % 64 == 0
            and residual.numel() == o2.shape[0] * wo.shape[0] and _lib.has("toa_gemm_asm_resadd")
            and resadd_fused_enabled())


_COSSIN: dict = {}   # (cos ptr, sin ptr, S) -> cos | sin [2][S][64] fp32 (toa_gemm_asm_rope's table)


def _cossin(cos, sin):
    key = (cos.data_ptr(), sin.data_ptr(), cos.shape[0])
    t = _COSSIN.get(key)
    if t is None:
        if len(_COSSIN) > 16:
            _COSSIN.clear()
        t = _COSSIN[key] = torch.stack([cos.float(), sin.float()]).contiguous()
    return t


class _QKVRopeAttn(torch.autograd.Function):
    """The fused-QKV projection, RoPE and causal attention as one node: the
    projection's assembly GEMM writes rotated, head-major q | k | v straight
    from its accumulators (toa_gemm_asm_rope: no [T, (Hq + 2 Hkv) D] qkv
    tensor, no toa_rope_fwd pass); backward: d(qkv) from the attention
    backward (rotated back there), then the projection's data and weight
    gradients (ops/linear.py)."""

    @staticmethod
    def forward(ctx, x, wqkv, cos, sin, B, S, Hq, Hkv, D, scale, bshd):
        x2 = x.reshape(-1, x.shape[-1])
        T, K = x2.shape
        out = torch.empty(T * (Hq + 2 * Hkv) * D, device=x.device, dtype=x.dtype)
        cs = _cossin(cos, sin)
        _lib.call("toa_gemm_asm_rope", _lib.ptr(x2), x2.stride(0), _lib.ptr(wqkv), wqkv.stride(0), _lib.ptr(out),
                  _lib.ptr(cs), T, K, S, Hq, Hkv, _lib.stream(x2))
        nq, nk = B * Hq * S * D, B * Hkv * S * D
        q = out[:nq].view(B, Hq, S, D)
        k = out[nq:nq + nk].view(B, Hkv, S, D)
        v = out[nq + nk:].view(B, Hkv, S, D)
        o = torch.empty(B, S, Hq, D, device=x.device, dtype=x.dtype) if bshd else torch.empty_like(q)
        lse = torch.empty(B, Hq, S, device=x.device, dtype=torch.float32)
        _lib.call("toa_attn_fwd", _lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(o), _lib.ptr(lse), B, Hq, Hkv, S, D,
                  1 | (2 if bshd else 0), float(scale), _lib.stream(q))
        ctx.save_for_backward(x, wqkv, q, k, v, o, lse, cos, sin)
        ctx.scale, ctx.bshd = scale, bshd
        return o

    @staticmethod
    def backward(ctx, do):
        from .grad import accumulate_mm

        x, wqkv, q, k, v, o, lse, cos, sin = ctx.saved_tensors
        dqkv = _rope_attn_dqkv(q, k, v, o, lse, cos, sin, do, ctx.scale, ctx.bshd)
        x2 = x.reshape(-1, x.shape[-1])
        dx = gemm.linear_dgrad(dqkv, wqkv).view_as(x) if ctx.needs_input_grad[0] else None
        dw = accumulate_mm(wqkv, dqkv.t(), x2)
        return dx, dw, None, None, None, None, None, None, None, None, None


def qkv_rope_attention_ok(x, wqkv, S, Hq, Hkv, D) -> bool:
    """The fused projection + RoPE path applies: the assembly GEMM policy,
    bf16, head dim 128, S and the projection width multiples of 256."""
    return (x.is_cuda and x.dtype == wqkv.dtype == torch.bfloat16 and D == 128 and S % 256 == 0
            and ((Hq + 2 * Hkv) * D) % 256 == 0 and Hq % Hkv == 0 and gemm.mode() == "asm"
            and os.environ.get("TOA_QKV_ROPE", "1") != "0" and _lib.has("toa_gemm_asm_rope")
            and x.reshape(-1, x.shape[-1]).stride(-1) == 1 and wqkv.stride(-1) == 1
            and (x.reshape(-1, x.shape[-1]).shape[0]) % S == 0 and x.shape[-1] % 64 == 0)


def qkv_rope_attention(x, wqkv, cos, sin, B, S, Hq, Hkv, D, scale=None, out_layout="bshd"):
    """linear(x, wqkv) -> rope_attention, fused where qkv_rope_attention_ok."""
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    return _QKVRopeAttn.apply(x, wqkv, cos, sin, B, S, Hq, Hkv, D, scale, out_layout == "bshd")


def rope_attention(qkv, cos, sin, B, S, Hq, Hkv, D, scale=None, out_layout="bshd"):
    """RoPE (Llama rotate-half, cos / sin [S, D/2]) on the fused QKV
    projection [B*S, (Hq + 2 Hkv) D], then causal attention with packed GQA:
    O as [B, S, Hq, D] (out_layout="bshd") or [B, Hq, S, D].  On the GPU one
    autograd node (_RopeAttn) whose backward writes d(qkv) directly; on the
    CPU rope_qkv + causal_attention."""
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if qkv.is_cuda:
        if not (qkv.dtype == torch.bfloat16 and D in ATTN_HEAD_DIMS and _lib.has("toa_attn_fwd")
                and _lib.has("toa_rope_fwd")):
            raise RuntimeError(f"HIP rope + flash attention needs bf16 and head_dim in {ATTN_HEAD_DIMS} "
                               f"(got {qkv.dtype}, head_dim {D}; library: {_lib.load_error() or 'ok'})")
        if Hq % Hkv:
            raise ValueError(f"query heads {Hq} not a multiple of kv heads {Hkv}")
        return _RopeAttn.apply(qkv, cos, sin, B, S, Hq, Hkv, D, scale, out_layout == "bshd")
    q, k, v = rope_qkv(qkv, cos, sin, B, S, Hq, Hkv, D, 1)
    return causal_attention(q, k, v, scale, out_layout)


def _attention_reference(q, k, v, scale):
    """Plain PyTorch causal attention (fp32 math, packed GQA expanded): the
    CPU path and the numerics reference of the HIP kernel."""
    rep = q.shape[1] // k.shape[1]
    if rep > 1:
        k = k.repeat_interleave(rep, 1)
        v = v.repeat_interleave(rep, 1)
    S = q.shape[2]
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return torch.matmul(torch.softmax(s, -1), v.float()).to(q.dtype)


def causal_attention(q, k, v, scale=None, out_layout="bhsd"):
    """q [B,H,S,D], k/v [B,Hk,S,D] (packed GQA, H % Hk == 0), any S.
    Returns O as [B,H,S,D], or as [B,S,H,D] with out_layout="bshd".

    On a GPU tensor this is ALWAYS the HIP flash-attention kernel (bf16,
    head_dim 64 or 128); anything else raises -- there is no library
    fallback.  CPU tensors take the plain PyTorch reference."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    if q.is_cuda:
        if not _attn_hip_ok(q):
            raise RuntimeError(f"HIP flash attention needs bf16 and head_dim in {ATTN_HEAD_DIMS} "
                               f"(got {q.dtype}, head_dim {q.shape[-1]}; library: {_lib.load_error() or 'ok'})")
        if q.shape[1] % k.shape[1]:
            raise ValueError(f"query heads {q.shape[1]} not a multiple of kv heads {k.shape[1]}")
        return _FlashAttn.apply(q.contiguous(), k.contiguous(), v.contiguous(), scale, out_layout == "bshd")
    o = _attention_reference(q, k, v, scale)
    return o.transpose(1, 2) if out_layout == "bshd" else o