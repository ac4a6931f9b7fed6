"""First-call cost of the GEMM layer (part of every job's submit -> first
step): each Llama-3-8B forward / dgrad form called once, then again, under
one GEMM policy, in a fresh process.

    python scripts/gemm_first_call.py --mode nosk|torch [--tokens 24576] [--prewarm]

TOA_GEMM_TRACE=1 adds the GEMM layer's per-phase host times on stderr.
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import gemm  # noqa: E402

FORMS = {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096),
         "lm_head": (4096, 128256)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="nosk")
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--prewarm", action="store_true", help="gemm.prewarm() first (timed separately)")
    a = ap.parse_args()
    torch.cuda.init()
    torch.empty(1, device="cuda")
    torch.cuda.synchronize()
    gemm.set_mode(a.mode)
    T = a.tokens
    out = {"mode": a.mode, "prewarm": a.prewarm, "first_ms": {}, "second_ms": {}}
    if a.prewarm:
        t0 = time.perf_counter()
        gemm.prewarm(background=False)
        out["prewarm_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    t_all = time.perf_counter()
    for name, (K, N) in FORMS.items():
        for kind, (kk, nn) in (("fwd", (K, N)), ("dgrad_wt", (N, K))):
            x = torch.empty(T, kk, device="cuda", dtype=torch.bfloat16).normal_()
            w = torch.empty(nn, kk, device="cuda", dtype=torch.bfloat16).normal_()
            torch.cuda.synchronize()
            for tag in ("first_ms", "second_ms"):
                t0 = time.perf_counter()
                gemm.linear_fwd(x, w)
                torch.cuda.synchronize()
                out[tag][f"{name}.{kind}"] = round((time.perf_counter() - t0) * 1e3, 2)
            del x, w
    out["total_first_minus_second_ms"] = round(sum(out["first_ms"].values()) - sum(out["second_ms"].values()), 1)
    out["wall_s"] = round(time.perf_counter() - t_all, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
