"""Where the assembly attention forward's cycles go (the s_memtime arm,
csrc/asm/attn_gen.py VARIANTS "t1", bit-identical outputs): per (workgroup,
wave) prologue / loop / epilogue shader cycles at the Llama-3-8B bench shape
(B=6, H=32, Hkv=8, S=4096, D=128, O in [B,S,H,D]).

    python scripts/attn_fwd_timing.py [--batch 6] [--seq 4096]

Prints one JSON object: loop cycles per 64-key tile (mean / by query
block), prologue and epilogue cycles, rescales per wave, the wall time of
the uninstrumented kernel and the shader clock that the cycle sum implies.
"""
import argparse
import json
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=6)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--arm", type=int, default=1, help="1: product schedule, 2: group-placed fillers (c1)")
    a = ap.parse_args()
    B, H, Hk, S, D = a.batch, 32, 8, a.seq, 128
    torch.manual_seed(0)
    q = torch.randn(B, H, S, D, device="cuda").to(torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device="cuda").to(torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device="cuda").to(torch.bfloat16)
    o = torch.empty(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    o2 = torch.empty_like(o)
    lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
    lse2 = torch.empty_like(lse)
    nwg = (S // 256) * H * B
    dbg = torch.zeros(nwg * 4 * 8, device="cuda", dtype=torch.int32)
    P, st = _lib.ptr, _lib.stream(q)
    args = (B, H, Hk, S, D, 3, 1.0 / math.sqrt(D), st)
    var = 0 if a.arm == 1 else 7   # the product kernel / its c1 arm (attn_gen.py VARIANTS index)
    for _ in range(3):
        _lib.call("toa_attn_fwd_asm_variant", var, P(q), P(k), P(v), P(o), P(lse), *args)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        _lib.call("toa_attn_fwd_asm_variant", var, P(q), P(k), P(v), P(o), P(lse), *args)
    ev[1].record()
    torch.cuda.synchronize()
    wall_us = ev[0].elapsed_time(ev[1]) / 10 * 1e3
    _lib.call("toa_attn_fwd_asm_timing", a.arm, P(dbg), P(q), P(k), P(v), P(o2), P(lse2), *args)
    torch.cuda.synchronize()
    rec = dbg.view(nwg, 4, 8).cpu().numpy().astype(np.int64)
    pro, loop, epi, tiles, qb, resc = (rec[..., i] for i in range(6))
    per_tile = loop / tiles
    by_qb = {int(b): round(float(per_tile[qb == b].mean()), 1) for b in np.unique(qb)}
    # per workgroup, the slowest wave bounds it; cycles summed over the CU's workgroups
    wg_cycles = (pro + loop + epi).max(axis=1)
    out = {
        "shape": [B, H, Hk, S, D],
        "identical_to_product": bool(torch.equal(o, o2) and torch.equal(lse, lse2)),
        "wall_us": round(wall_us, 1),
        "loop_cycles_per_tile": {"mean": round(float(per_tile.mean()), 1), "p10": round(float(np.percentile(per_tile, 10)), 1),
                                 "p90": round(float(np.percentile(per_tile, 90)), 1), "by_query_block": by_qb},
        "prologue_cycles": {"mean": round(float(pro.mean())), "p90": round(float(np.percentile(pro, 90)))},
        "epilogue_cycles": {"mean": round(float(epi.mean())), "p90": round(float(np.percentile(epi, 90)))},
        "wave_skew_in_wg_cycles": round(float(((pro + loop + epi).max(1) - (pro + loop + epi).min(1)).mean())),
        "rescales_per_wave": round(float(resc.mean()), 2),
        "cycles_per_cu": round(float(wg_cycles.sum() / 256)),
        "implied_clock_ghz": round(float(wg_cycles.sum() / 256 / (wall_us * 1e3)), 3),
        "mfma_cycles_per_tile": 72 * 32,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
