"""In-process timing of the assembly dK/dV kernel (csrc/asm/attn_bwd_gen.py)
and its diagnostic arms at the Llama-3-8B bench shape (B=6, H=32, Hkv=8,
S=4096, D=128, dO in [B,S,H,D], RoPE epilogue into d(qkv) rows), interleaved
rounds on random data.  Arm v (1..) switches one mechanism off (VARIANTS in
the generator); its output is wrong by design, only its time is read.

    python scripts/attn_dkdv_arms.py [--rounds 5] [--reps 5] [--arms 0,1,2,3,4,5,6]
"""
import argparse
import json
import math
import statistics
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "csrc/asm")
from tf_operator_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=6)
    ap.add_argument("--arms", default="0,1,2,3,4,5,6")
    a = ap.parse_args()
    import attn_bwd_gen
    names = ["asm"] + [v for v, _ in attn_bwd_gen.VARIANTS]
    B, H, Hk, S, D = a.batch, 32, 8, 4096, 128
    H3 = H + 2 * Hk
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
    P = _lib.ptr
    st = _lib.stream(q)
    _lib.call("toa_attn_fwd", P(q), P(k), P(v), P(o), P(lse), B, H, Hk, S, D, 3, scale, st)
    pos = torch.arange(S, device=dev, dtype=torch.float32)[:, None]
    inv = 10000.0 ** (-torch.arange(D // 2, device=dev, dtype=torch.float32) * 2.0 / D)
    cosv, sinv = torch.cos(pos * inv).contiguous(), torch.sin(pos * inv).contiguous()
    nws = _lib.call_ret("toa_attn_bwd_ws_bytes", B, H, S, D)
    ws = torch.empty(nws, device=dev, dtype=torch.uint8)
    dqkv = torch.empty(B * S, H3 * D, device=dev, dtype=torch.bfloat16)
    # the fused backward fills the delta pass's -lse log2 e / -delta rows
    _lib.call("toa_attn_bwd_rope", P(q), P(k), P(v), P(o), P(do), P(lse), P(delta), P(ws), P(cosv), P(sinv),
              P(dqkv), B, H, Hk, S, D, 3, scale, st)
    nb = S // 32
    ds_bytes = B * H * (nb * (nb + 1) // 2) * 2048
    nlse2 = ws[ds_bytes:ds_bytes + B * H * S * 4]

    def run(arm):
        _lib.call("toa_attn_dkdv_asm_variant", arm, P(q), P(k), P(v), P(do), P(nlse2), P(delta), P(dqkv), P(dqkv),
                  P(ws), B, H, Hk, S, D, scale, 3, P(cosv), P(sinv), H3, st)

    arms = [int(x) for x in a.arms.replace("+", ",").split(",")]
    # flops of dK/dV: S, dP, dV, dK over the causal half (4 S^2 D products x 2 flop / 2)
    flops = 4 * B * H * S * S * D
    times = {x: [] for x in arms}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(a.rounds):
        for x in arms:
            run(x)
            ev[0].record()
            for _ in range(a.reps):
                run(x)
            ev[1].record()
            torch.cuda.synchronize()
            times[x].append(ev[0].elapsed_time(ev[1]) / a.reps)
    res = {"shape": [B, H, Hk, S, D]}
    for x, t in times.items():
        med = statistics.median(t)
        res[names[x]] = {"median_ms": round(med, 4), "min_ms": round(min(t), 4), "PFps": round(flops / med / 1e12, 3)}
    # the s_memtime arm: loop cycles per step (64 MFMAs = 2048 matrix-core cycles per SIMD)
    nwg = (S // 128) * B * Hk
    dbg = torch.zeros(nwg * 4 * 8, device=dev, dtype=torch.int32)
    ev[0].record()
    _lib.call("toa_attn_dkdv_asm_timing", P(dbg), P(q), P(k), P(v), P(do), P(nlse2), P(delta), P(dqkv), P(dqkv),
              P(ws), B, H, Hk, S, D, scale, 3, P(cosv), P(sinv), H3, st)
    ev[1].record()
    torch.cuda.synchronize()
    r = dbg.view(nwg, 4, 8).cpu().long()
    cyc = (r[..., 0] & 0xFFFFFFFF) + (r[..., 1] << 32)
    steps = r[..., 2].clamp(min=1)
    per = (cyc.double() / steps.double()).flatten()
    srt = per.sort().values
    by_kb = {}
    for kb in range(S // 128):
        sel = r[..., 3] == kb
        if sel.any():
            by_kb[kb] = round(float((cyc[sel].double() / steps[sel].double()).mean()), 1)
    wall = ev[0].elapsed_time(ev[1])
    res["timing"] = {"cyc_per_step_mean": round(float(per.mean()), 1), "p10": round(float(srt[len(srt) // 10]), 1),
                     "p90": round(float(srt[9 * len(srt) // 10]), 1), "mfma_cycles_per_step": 2048,
                     "by_key_block": by_kb, "wall_ms": round(wall, 4),
                     "sum_loop_cycles_per_simd_over_256_cus": round(float(cyc[:, 0].sum()) / 256, 0)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
