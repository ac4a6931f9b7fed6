"""Attention-forward cost model: time the assembly and HIP forwards at
shapes with different (key tiles, workgroups) counts and fit

    t = a * tiles + b * workgroups        (per CU: divide by 256)

so a = the loop's cost per 64-key tile of a 256-row block and b = the
per-workgroup prologue + epilogue.  Shapes: (B, S) with H = 32, Hkv = 8,
D = 128, O in [B, S, H, D].

    python scripts/attn_fwd_sweep.py [--forms gl,asm] [--reps 10]
"""
import argparse
import json
import math
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402

SHAPES = ((6, 4096), (24, 2048), (96, 512), (3, 8192), (48, 1024))


def counts(B, S, H=32):
    nqb = S // 256
    wgs = nqb * H * B
    tiles = H * B * sum(4 * (qb + 1) for qb in range(nqb))
    return tiles, wgs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--forms", default="gl,asm")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    H, Hk, D = 32, 8, 128
    forms = {k: v for k, v in {"gl": 1, "asm": 2}.items() if k in a.forms.split(",")}
    P = _lib.ptr
    res = {"shapes": [], "fit": {}}
    times = {f: {} for f in forms}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for B, S in SHAPES:
        torch.manual_seed(0)
        q = torch.randn(B, H, S, D, device="cuda").to(torch.bfloat16)
        k = torch.randn(B, Hk, S, D, device="cuda").to(torch.bfloat16)
        v = torch.randn(B, Hk, S, D, device="cuda").to(torch.bfloat16)
        o = torch.empty(B, S, H, D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)

        def run(f):
            _lib.call("toa_attn_set_fwd_variant", forms[f])
            _lib.call("toa_attn_fwd", P(q), P(k), P(v), P(o), P(lse), B, H, Hk, S, D, 3, 1.0 / math.sqrt(D),
                      _lib.stream(q))

        for f in forms:
            run(f)
        ts = {f: [] for f in forms}
        for _ in range(a.rounds):
            for f in forms:
                run(f)
                ev[0].record()
                for _ in range(a.reps):
                    run(f)
                ev[1].record()
                torch.cuda.synchronize()
                ts[f].append(ev[0].elapsed_time(ev[1]) / a.reps)
        tiles, wgs = counts(B, S)
        row = {"B": B, "S": S, "tiles": tiles, "wgs": wgs}
        for f in forms:
            times[f][(B, S)] = statistics.median(ts[f])
            row[f"{f}_ms"] = round(times[f][(B, S)], 4)
        res["shapes"].append(row)
        print(json.dumps(row), flush=True)
        del q, k, v, o, lse
    _lib.call("toa_attn_set_fwd_variant", -1)
    A = np.array([[counts(B, S)[0] / 256, counts(B, S)[1] / 256] for B, S in SHAPES])
    for f in forms:
        y = np.array([times[f][s] * 1e3 for s in SHAPES])  # us
        (ct, cw), *_ = np.linalg.lstsq(A, y, rcond=None)
        res["fit"][f] = {"us_per_tile_per_cu": round(float(ct), 4), "us_per_wg_per_cu": round(float(cw), 3),
                         "resid_us": [round(float(r), 2) for r in (y - A @ np.array([ct, cw]))]}
    print(json.dumps(res["fit"]))


if __name__ == "__main__":
    main()
