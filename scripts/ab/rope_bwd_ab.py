"""In-process A/B of the RoPE-fused attention backward (toa_attn_bwd_rope:
delta pass + dK/dV storing dS + dQ GEMM writing d(qkv)) at the Llama-3-8B
bench shape, A/B of one switch (--switch):

    prefetch  the dQ GEMM's cos / sin rows loaded before its main loop (1) or
              in its epilogue (0)           toa_attn_set_rope_prefetch
    stagger   (rejected, removed) the dK/dV kernel's two query-half wave rows
              staggered by one segment: profiles/r3_attn_pmc/ab_dkdv_stagger_rejected.log

Interleaved rounds on random data; checks the two arms agree bit for bit.

    python scripts/ab/rope_bwd_ab.py [--switch prefetch] [--rounds 8] [--reps 5]
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
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--switch", default="prefetch", choices=("prefetch",))
    a = ap.parse_args()
    setter = {"prefetch": "toa_attn_set_rope_prefetch"}[a.switch]
    B, H, Hk, S, D = 6, 32, 8, 4096, 128
    dev = "cuda"
    torch.manual_seed(0)
    P, st = _lib.ptr, None
    q = torch.randn(B, H, S, D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device=dev).to(torch.bfloat16)
    o = torch.empty(B, S, H, D, device=dev, dtype=torch.bfloat16)
    do = torch.randn(B, S, H, D, device=dev).to(torch.bfloat16)
    lse = torch.empty(B, H, S, device=dev, dtype=torch.float32)
    delta = torch.empty_like(lse)
    pos = torch.arange(S, device=dev, dtype=torch.float32)[:, None]
    inv = 500000.0 ** (-torch.arange(0, D, 2, device=dev, dtype=torch.float32) / D)
    cos, sin = torch.cos(pos * inv).contiguous(), torch.sin(pos * inv).contiguous()
    scale = 1.0 / math.sqrt(D)
    flags = 1 | 2
    st = _lib.stream(q)
    _lib.call("toa_attn_fwd", P(q), P(k), P(v), P(o), P(lse), B, H, Hk, S, D, flags, scale, st)
    ws = torch.empty(_lib.call_ret("toa_attn_bwd_ws_bytes", B, H, S, D), device=dev, dtype=torch.uint8)
    outs = {}

    def run(pre):
        _lib.call(setter, pre)
        dqkv = torch.empty(B * S, (H + 2 * Hk) * D, device=dev, dtype=torch.bfloat16)
        _lib.call("toa_attn_bwd_rope", P(q), P(k), P(v), P(o), P(do), P(lse), P(delta), P(ws), P(cos), P(sin),
                  P(dqkv), B, H, Hk, S, D, flags, scale, st)
        return dqkv

    for pre in (1, 0):
        outs[pre] = run(pre)
    torch.cuda.synchronize()
    same = bool(torch.equal(outs[0], outs[1]))
    times = {1: [], 0: []}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(a.rounds):
        for pre in (1, 0):
            run(pre)
            ev[0].record()
            for _ in range(a.reps):
                run(pre)
            ev[1].record()
            torch.cuda.synchronize()
            times[pre].append(ev[0].elapsed_time(ev[1]) / a.reps)
    _lib.call(setter, -1)
    print(json.dumps({"switch": a.switch, "bit_identical": same, "on_ms": round(statistics.median(times[1]), 4),
                      "off_ms": round(statistics.median(times[0]), 4), "on_min": round(min(times[1]), 4),
                      "off_min": round(min(times[0]), 4)}))


if __name__ == "__main__":
    main()
