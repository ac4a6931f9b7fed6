"""In-process A/B of attention kernel variants (build/variants/attention_*.so):
same inputs, interleaved rounds, median ms per kernel family; each variant's
outputs are checked against the first's.

    python scripts/ab/attn_ab.py base noslp [--B 6]
"""
import argparse
import ctypes
import glob
import math
import os
import statistics

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
p = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float


def load(name):
    lib = ctypes.CDLL(os.path.join(ROOT, "build", "variants", f"attention_{name}.so"))
    lib.toa_attn_fwd.argtypes = [p, p, p, p, p, I, I, I, I, I, I, F, p]
    lib.toa_attn_bwd.argtypes = [p, p, p, p, p, p, p, p, p, p, p, I, I, I, I, I, I, F, p]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--B", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    B, H, Hk, S, D = a.B, 32, 8, 4096, 128
    dev = "cuda"
    torch.manual_seed(0)
    q = torch.randn(B, H, S, D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device=dev).to(torch.bfloat16)
    do = torch.randn(B, S, H, D, device=dev).to(torch.bfloat16)
    scale = 1 / math.sqrt(D)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    libs = {n: load(n) for n in a.variants}
    outs = {}
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def mk():
        return dict(o=torch.empty(B, S, H, D, device=dev, dtype=torch.bfloat16),
                    lse=torch.empty(B, H, S, device=dev, dtype=torch.float32),
                    delta=torch.empty(B, H, S, device=dev, dtype=torch.float32),
                    dq=torch.empty_like(q), dk=torch.empty_like(k), dv=torch.empty_like(v))

    bufs = {n: mk() for n in libs}

    def fwd(n):
        b = bufs[n]
        rc = libs[n].toa_attn_fwd(P(q), P(k), P(v), P(b["o"]), P(b["lse"]), B, H, Hk, S, D, 3, scale, st)
        assert rc == 0, rc

    def bwd(n):
        b = bufs[n]
        rc = libs[n].toa_attn_bwd(P(q), P(k), P(v), P(b["o"]), P(do), P(b["lse"]), P(b["delta"]), None, P(b["dq"]),
                                  P(b["dk"]), P(b["dv"]), B, H, Hk, S, D, 3, scale, st)
        assert rc == 0, rc

    for n in libs:
        fwd(n)
        bwd(n)
    torch.cuda.synchronize()
    ref = a.variants[0]
    for n in libs:
        errs = {t: float((bufs[n][t].float() - bufs[ref][t].float()).abs().max()) for t in ("o", "dq", "dk", "dv")}
        print(n, "max|diff| vs", ref, {t: round(e, 5) for t, e in errs.items()}, flush=True)

    def timeit(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.reps

    res = {n: {"fwd": [], "bwd": []} for n in libs}
    for _ in range(a.rounds):
        for n in libs:
            res[n]["fwd"].append(timeit(lambda: fwd(n)))
            res[n]["bwd"].append(timeit(lambda: bwd(n)))
    fl = 4 * B * H * S * S * D / 2
    for n in libs:
        f, b = statistics.median(res[n]["fwd"]), statistics.median(res[n]["bwd"])
        print(f"{n:12s} fwd {f:7.3f} ms ({fl / f / 1e9:6.1f} TF)  bwd {b:7.3f} ms ({2.5 * fl / b / 1e9:6.1f} TF)",
              flush=True)


if __name__ == "__main__":
    main()
