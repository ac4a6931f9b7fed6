"""In-process A/B of the attention-forward forms at the Llama-3-8B bench
shape (B=6, H=32, Hkv=8, S=4096, D=128, O in [B,S,H,D]), interleaved rounds
on random data (guide §5.4 rules 24/25):

    reg  K/V tiles staged through registers + ds_write (attn_fwd_kernel)
    gl   K/V tiles by LDS-DMA into two distinct LDS objects (attn_fwd_gl_kernel)
    asm  the generated gfx950 assembly kernel (csrc/asm/attn_gen.py; default
         since round 5)
    d1.. its DIAGNOSTIC arms (attn_gen.py VARIANTS: one mechanism switched
         off each; wrong outputs, timing only -- excluded from the diffs)
(Round 4 measured more arms of the LDS-DMA kernel and removed them, all
slower than gl and bit-identical to it, profiles/r4_attn/: buffer-path DMA
with fragments read one MFMA pair ahead 0.860 vs 0.798 ms, buffer-path DMA
alone 0.838 vs 0.803 ms; then against gl's 0.805 ms (r4_fwd): K fragments
one pair ahead 0.815, the same with buffer-path DMA 0.833, the first 32 keys'
PV MFMAs between the second 32's exponentials 0.838, that with buffer-path
DMA 0.894, all three 0.876.  Then the stagger, profiles/r4_fwd_stagger/:
the two waves of each SIMD half a tile apart (waves 4-7 run O += V P(t-1)
before scoring tile t, three K/V buffers) 0.846 vs 0.809 ms, that with
s_setprio 1 around every MFMA run 0.859, and three buffers without the lag
0.834 -- the third buffer's code alone costs 3 %, the lag another 1.5 %, so
the waves' shared phase is not what holds the forward at 47 % MFMA busy.
Static s_setprio 1 for waves 4-7 before the loop: 0.826 vs 0.814 ms.)

and the max |difference| of O / lse between them (same arithmetic: 0 expected).

    python scripts/attn_fwd_ab.py [--rounds 6] [--reps 10] [--forms gl,asm]
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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=6)
    ap.add_argument("--forms", default="gl,asm")
    a = ap.parse_args()
    B, H, Hk, S, D = a.batch, 32, 8, 4096, 128
    torch.manual_seed(0)
    q = torch.randn(B, H, S, D, device="cuda").to(torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device="cuda").to(torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device="cuda").to(torch.bfloat16)
    P = _lib.ptr
    arms = ("d1", "d2", "d3", "d4", "d5", "t1", "c1")   # attn_gen.py VARIANTS order
    forms = {k: v for k, v in {"reg": 0, "gl": 1, "asm": 2, **{x: -(i + 1) for i, x in enumerate(arms)}}.items()
             if k in a.forms.split(",")}
    outs = {}

    def run(form):
        o = torch.empty(B, S, H, D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
        if forms[form] < 0:   # diagnostic arm of the assembly kernel
            _lib.call("toa_attn_fwd_asm_variant", -forms[form], P(q), P(k), P(v), P(o), P(lse), B, H, Hk, S, D,
                      1 | 2, 1.0 / math.sqrt(D), _lib.stream(q))
            return o, lse
        _lib.call("toa_attn_set_fwd_variant", forms[form])
        _lib.call("toa_attn_fwd", P(q), P(k), P(v), P(o), P(lse), B, H, Hk, S, D, 1 | 2, 1.0 / math.sqrt(D),
                  _lib.stream(q))
        return o, lse

    for f in forms:
        outs[f] = run(f)
    torch.cuda.synchronize()
    base = list(forms)[0]
    diff = {f"{f}_vs_{base}": {"o": float((outs[f][0].float() - outs[base][0].float()).abs().max()),
                               "o_rel": float((outs[f][0].float() - outs[base][0].float()).norm()
                                              / outs[base][0].float().norm()),
                               "lse": float((outs[f][1] - outs[base][1]).abs().max())}
            for f in list(forms)[1:] if forms[f] >= 0}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = {f: [] for f in forms}
    for _ in range(a.rounds):
        for f in forms:
            run(f)
            ev[0].record()
            for _ in range(a.reps):
                run(f)
            ev[1].record()
            torch.cuda.synchronize()
            times[f].append(ev[0].elapsed_time(ev[1]) / a.reps)
    _lib.call("toa_attn_set_fwd_variant", -1)
    flops = 4 * B * H * S * S * D / 2
    res = {"shape": [B, H, Hk, S, D], "max_abs_diff": diff}
    for f, t in times.items():
        med = statistics.median(t)
        res[f] = {"median_ms": round(med, 4), "min_ms": round(min(t), 4), "PFps": round(flops / med / 1e12, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
