"""In-process A/B of the attention-backward forms at the Llama-3-8B bench
shape (B=6, H=32, Hkv=8, S=4096, D=128, O/dO in [B,S,H,D]), interleaved
rounds on random data (guide §5.4 rules 24/25):

    split   dQ kernel (recomputes S, dP) + 8-wave dK/dV (K/V re-read from LDS)
    ds      delta pass + dK/dV storing dS + dQ as a GEMM over the stored dS
            (dK/dV on the assembly kernel, csrc/asm/attn_bwd_gen.py)
    dship   the same with the HIP dK/dV kernel (attn_bwd_dkdv_ds_kernel)

(Round-4 arms measured with this script, profiles/r4_attn/: kept -- the
pipelined sub-tile, the store-aware step-end wait, P / dS overlapped with the
first half's MFMAs; removed -- static priority, pipelined or buffer-DMA dQ
GEMM, register-pair P / dS.)

--timing: one extra run of the ds form with the dK/dV kernel's s_memtime
instrumentation (issue vs step-end wait cycles per step, per wave).

Also checks every form agrees with the first.

    python scripts/attn_bwd_ab.py [--rounds 6] [--reps 5] [--variants split,ds] [--timing]
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
    ap.add_argument("--variants", default="split,ds")
    ap.add_argument("--timing", action="store_true")
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

    # backward form: 0 = split (dQ recomputes S / dP), 1 = dS through HBM + dQ GEMM
    forms = {"split": 0, "ds": 1, "dship": 1}
    dkdv = {"split": -1, "ds": 1, "dship": 0}
    variants = a.variants.replace("+", ",").split(",")

    def run(variant):
        _lib.call("toa_attn_set_bwd_variant", forms[variant])
        _lib.call("toa_attn_set_dkdv_variant", dkdv[variant])
        nws = _lib.call_ret("toa_attn_bwd_ws_bytes", B, H, S, D)
        ws = torch.empty(nws, device=dev, dtype=torch.uint8) if nws > 0 else None
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _lib.call("toa_attn_bwd", P(q), P(k), P(v), P(o), P(do), P(lse), P(delta), P(ws), P(dq), P(dk), P(dv), B, H,
                  Hk, S, D, flags, scale, _lib.stream(q))
        return dq, dk, dv

    for var in variants:
        outs[var] = run(var)
    torch.cuda.synchronize()
    base = variants[0]
    agree = {f"{var}_vs_{base}": {n: float((outs[var][i].float() - outs[base][i].float()).norm()
                                            / outs[base][i].float().norm()) for i, n in enumerate(("dq", "dk", "dv"))}
             for var in variants[1:]}
    flops_fwd = 4 * B * H * S * S * D / 2  # causal: two matmuls over half the scores
    times = {v: [] for v in variants}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(a.rounds):
        for var in variants:
            run(var)
            ev[0].record()
            for _ in range(a.reps):
                run(var)
            ev[1].record()
            torch.cuda.synchronize()
            times[var].append(ev[0].elapsed_time(ev[1]) / a.reps)
    res = {"shape": [B, H, Hk, S, D], "rel_diff": agree}
    for var, t in times.items():
        med = statistics.median(t)
        res[var] = {"median_ms": round(med, 3), "min_ms": round(min(t), 3),
                             "useful_PFps": round(2.5 * flops_fwd / med / 1e12, 3)}
    if a.timing:
        nblk = (S // 128) * B * Hk
        for var in variants:
            if forms[var] == 0:
                continue
            ts = torch.zeros(nblk * 8 * 4, device=dev, dtype=torch.int64)
            _lib.call("toa_attn_set_bwd_timing", P(ts))
            run(var)
            torch.cuda.synchronize()
            _lib.call("toa_attn_set_bwd_timing", None)
            t = ts.view(nblk, 8, 4).double().cpu()
            steps = t[..., 2].clamp(min=1)
            per = {}
            for m in (0, 1):
                w = slice(4 * m, 4 * m + 4)
                per[f"m{m}"] = {"issue_cyc_per_step": round(float((t[:, w, 0] / steps[:, w]).mean()), 1),
                                "wait_cyc_per_step": round(float((t[:, w, 1] / steps[:, w]).mean()), 1)}
            res[var]["timing"] = per
    _lib.call("toa_attn_set_bwd_variant", -1)
    _lib.call("toa_attn_set_dkdv_variant", -1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
