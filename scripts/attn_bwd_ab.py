"""In-process A/B of the attention-backward kernel forms at the Llama-3-8B
bench shape (B=6, H=32, Hkv=8, S=4096, D=128, O/dO in [B,S,H,D]):
dQ + dK/dV with the 8-wave dK/dV kernel (K/V re-read from LDS) vs the
4-wave one (K/V fragments in registers), interleaved rounds on random
data (guide §5.4 rules 24/25).  Also checks the two forms agree.

    python scripts/attn_bwd_ab.py [--rounds 6] [--reps 5]
"""
import argparse
import json
import math
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=6)
    a = ap.parse_args()
    B, H, Hk, S, D = a.batch, 32, 8, 4096, 128
    dev = "cuda"
    torch.manual_seed(0)
    q = torch.randn(B, H, S, D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device=dev).to(torch.bfloat16)
    o = torch.empty(B, S, H, D, device=dev, dtype=torch.bfloat16)
    do = torch.randn(B, S, H, D, device=dev).to(torch.bfloat16)
    lse = torch.empty(B, H, S, device=dev, dtype=torch.float32)
    delta = torch.empty_like(lse)
    scale = 1.0 / math.sqrt(D)
    flags = 1 | 2  # causal, O/dO in [B,S,H,D]
    P = _lib.ptr
    _lib.call("toa_attn_fwd", P(q), P(k), P(v), P(o), P(lse), B, H, Hk, S, D, flags, scale, _lib.stream(q))
    outs = {}

    def run(variant):
        _lib.call("toa_attn_set_dkdv_variant", variant)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _lib.call("toa_attn_bwd", P(q), P(k), P(v), P(o), P(do), P(lse), P(delta), None, P(dq), P(dk), P(dv), B, H,
                  Hk, S, D, flags, scale, _lib.stream(q))
        return dq, dk, dv

    for var in (8, 4):
        outs[var] = run(var)
    torch.cuda.synchronize()
    agree = {n: float((outs[4][i].float() - outs[8][i].float()).norm() / outs[8][i].float().norm())
             for i, n in enumerate(("dq", "dk", "dv"))}
    flops_fwd = 4 * B * H * S * S * D / 2  # causal: two matmuls over half the scores
    times = {8: [], 4: []}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(a.rounds):
        for var in (8, 4):
            run(var)
            ev[0].record()
            for _ in range(a.reps):
                run(var)
            ev[1].record()
            torch.cuda.synchronize()
            times[var].append(ev[0].elapsed_time(ev[1]) / a.reps)
    res = {"shape": [B, H, Hk, S, D], "rel_diff_4_vs_8": agree}
    for var, t in times.items():
        med = statistics.median(t)
        res[f"dkdv{var}"] = {"median_ms": round(med, 3), "min_ms": round(min(t), 3),
                             "useful_PFps": round(2.5 * flops_fwd / med / 1e12, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
