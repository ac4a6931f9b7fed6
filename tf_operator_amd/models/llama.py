"""Llama-3 family decoder (random init, bf16) built on the fused HIP ops.

This is the BASELINE.json config-#3 model (TFJob Worker=8 all-reduce
Llama-3-8B bf16).  Per layer the forward is:

    (h, x) = add_rms_norm(h_prev, delta_prev)      HIP, residual add fused
    qkv    = x @ Wqkv^T                             hipBLASLt (fused Q|K|V weight)
    o      = rope_attention(qkv)                    HIP RoPE + head-major relayout, flash attention
                                                    (packed GQA); backward writes d(qkv) directly
    a      = o^T @ Wo^T                             hipBLASLt
    (h, x) = add_rms_norm(h, a)                     HIP
    gu     = x @ Wgu^T                              hipBLASLt (fused gate|up weight)
    delta  = swiglu(gu) @ Wd^T                      HIP SwiGLU, recomputed in bwd
final norm -> lm_head -> fused cross entropy (HIP, in-place logit gradient).

Every weight gradient is accumulated by the op straight into the flat
gradient buffer (``main_grad``), in backward order, so bucket all-reduces
start during backward.
"""
from __future__ import annotations

import dataclasses
import math

import torch

from ..ops.embedding import Embedding
from ..ops.linear import linear
from ..ops.llm import (attn_out_proj, attn_out_proj_resadd_ok, causal_attention, cross_entropy, qkv_rope_attention,
                       qkv_rope_attention_ok, rope_attention, rope_qkv, rope_tables, swiglu_mlp,
                       swiglu_mlp_resadd_ok)
from ..ops.norm import RMSNorm, add_rms_norm


@dataclasses.dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    ffn: int = 14336
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq: int = 8192
    tie_embeddings: bool = False
    init_std: float = 0.02
    # "expand" materialises K/V per query head (kept for A/B runs); the HIP
    # flash-attention kernel (and the CPU reference) read packed GQA K/V directly.
    kv_layout: str = "auto"

    @property
    def head_dim(self):
        return self.hidden // self.heads

    def num_params(self):
        h, f, v, L = self.hidden, self.ffn, self.vocab_size, self.layers
        d = self.head_dim
        per_layer = h * (self.heads + 2 * self.kv_heads) * d + self.heads * d * h + 2 * f * h + f * h + 2 * h
        emb = v * h * (1 if self.tie_embeddings else 2)
        return L * per_layer + emb + h

    def flops_per_token(self, seq):
        """Training FLOPs/token (6N + causal attention 6*L*S*H... per Megatron)."""
        n = self.num_params() - self.vocab_size * self.hidden  # embedding lookup is not a GEMM
        attn = 6 * self.layers * seq * self.hidden  # 12*L*S*H/2 (causal)
        return 6 * n + attn


PRESETS = {
    "llama3-8b": LlamaConfig(),
    "llama3-1b": LlamaConfig(vocab_size=128256, hidden=2048, layers=16, heads=32, kv_heads=8, ffn=8192,
                             tie_embeddings=True),
    "llama-tiny": LlamaConfig(vocab_size=512, hidden=256, layers=2, heads=4, kv_heads=2, ffn=512, max_seq=512),
    # head_dim 128 like Llama-3-8B: the smoke model runs the same attention kernel as the flagship
    "llama-tiny128": LlamaConfig(vocab_size=1024, hidden=512, layers=2, heads=4, kv_heads=2, ffn=1024, max_seq=1024),
}


# a block's second output when its down projection already added the residual (the next norm is presummed)
PRESUMMED = object()


class LlamaBlock(torch.nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        d = cfg.head_dim
        qkv_out = (cfg.heads + 2 * cfg.kv_heads) * d
        self.attn_norm = RMSNorm(cfg.hidden, cfg.norm_eps, dtype=dtype, device=device)
        self.wqkv = torch.nn.Parameter(torch.empty(qkv_out, cfg.hidden, dtype=dtype, device=device))
        self.wo = torch.nn.Parameter(torch.empty(cfg.hidden, cfg.heads * d, dtype=dtype, device=device))
        self.mlp_norm = RMSNorm(cfg.hidden, cfg.norm_eps, dtype=dtype, device=device)
        self.wgu = torch.nn.Parameter(torch.empty(2 * cfg.ffn, cfg.hidden, dtype=dtype, device=device))
        self.wd = torch.nn.Parameter(torch.empty(cfg.hidden, cfg.ffn, dtype=dtype, device=device))

    def params_backward_order(self):
        return [self.wd, self.wgu, self.mlp_norm.weight, self.wo, self.wqkv, self.attn_norm.weight]

    def forward(self, h, delta, cos, sin, B, S):
        cfg = self.cfg
        if delta is None:
            x = self.attn_norm(h)
        elif delta is PRESUMMED:   # the previous block's down projection added the residual already
            h, x = self.attn_norm.presummed(h)
        else:
            h, x = self.attn_norm(h, delta)
        if cfg.kv_layout in ("packed", "auto") and qkv_rope_attention_ok(x, self.wqkv, S, cfg.heads, cfg.kv_heads,
                                                                         cfg.head_dim):
            # the projection's GEMM writes rotated head-major q | k | v (no qkv tensor, no RoPE pass)
            o = qkv_rope_attention(x, self.wqkv, cos, sin, B, S, cfg.heads, cfg.kv_heads, cfg.head_dim)
        elif cfg.kv_layout in ("packed", "auto"):
            # the attention kernel reads packed GQA K/V natively; RoPE and
            # attention are one autograd node whose backward writes d(qkv)
            qkv = linear(x, self.wqkv)
            o = rope_attention(qkv, cos, sin, B, S, cfg.heads, cfg.kv_heads, cfg.head_dim)  # [B, S, H, D]
        else:
            qkv = linear(x, self.wqkv)
            rep = cfg.heads // cfg.kv_heads
            q, k, v = rope_qkv(qkv, cos, sin, B, S, cfg.heads, cfg.kv_heads, cfg.head_dim, rep)
            o = causal_attention(q, k, v, out_layout="bshd")  # [B, S, H, D]: no transpose copy
        o = o.reshape(B * S, cfg.heads * cfg.head_dim)
        # the RoPE-attention nodes consume the delta rows the projection's backward leaves; the other
        # attention path does not, so it keeps the plain linear
        packed = cfg.kv_layout in ("packed", "auto")
        if o.is_cuda and packed and attn_out_proj_resadd_ok(o, self.wo, h):
            # the residual add in the projection's epilogue; the norm then reads the sum once
            h, x = self.mlp_norm.presummed(attn_out_proj(o, self.wo, B, S, cfg.heads, residual=h))
        else:
            a = attn_out_proj(o, self.wo, B, S, cfg.heads) if (o.is_cuda and packed) else linear(o, self.wo)
            h, x = self.mlp_norm(h, a)
        if swiglu_mlp_resadd_ok(x, self.wd, h):
            # + the residual in the down projection's epilogue: the next norm reads the sum once
            return swiglu_mlp(x, self.wgu, self.wd, residual=h), PRESUMMED
        delta = swiglu_mlp(x, self.wgu, self.wd)  # SwiGLU fused into the GEMMs under TOA_GEMM=hip
        return h, delta


class Llama(torch.nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        self.embed = Embedding(cfg.vocab_size, cfg.hidden, dtype=dtype, device=device)
        self.blocks = torch.nn.ModuleList([LlamaBlock(cfg, device, dtype) for _ in range(cfg.layers)])
        self.norm = RMSNorm(cfg.hidden, cfg.norm_eps, dtype=dtype, device=device)
        if not cfg.tie_embeddings:
            self.lm_head = torch.nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden, dtype=dtype, device=device))
        self._rope_cache = {}

    @torch.no_grad()
    def init_weights(self, seed=0):
        g = torch.Generator(device=self.embed.weight.device)
        g.manual_seed(seed)
        std = self.cfg.init_std
        out_std = std / math.sqrt(2 * self.cfg.layers)
        for name, p in self.named_parameters():
            if p.dim() == 1:
                p.fill_(1.0)
            elif name.endswith("wo") or name.endswith("wd"):
                p.normal_(0.0, out_std, generator=g)
            else:
                p.normal_(0.0, std, generator=g)

    def head_weight(self):
        return self.embed.weight if self.cfg.tie_embeddings else self.lm_head

    def params_backward_order(self):
        ps = []
        if not self.cfg.tie_embeddings:
            ps.append(self.lm_head)
        ps.append(self.norm.weight)
        for b in reversed(self.blocks):
            ps.extend(b.params_backward_order())
        ps.append(self.embed.weight)
        return ps

    def no_decay(self, p):
        return p.dim() == 1

    def rope(self, S, device):
        key = (S, str(device))
        if key not in self._rope_cache:
            self._rope_cache[key] = rope_tables(S, self.cfg.head_dim, self.cfg.rope_theta, device=device)
        return self._rope_cache[key]

    def forward(self, tokens, targets=None):
        B, S = tokens.shape
        cos, sin = self.rope(S, tokens.device)
        h = self.embed(tokens).view(B * S, self.cfg.hidden)
        delta = None
        for blk in self.blocks:
            h, delta = blk(h, delta, cos, sin, B, S)
        _, x = self.norm.presummed(h) if delta is PRESUMMED else self.norm(h, delta)
        logits = linear(x, self.head_weight())
        if targets is None:
            return logits.view(B, S, -1)
        return cross_entropy(logits, targets.reshape(-1), inplace_grad=True)
