"""Hand-written NT weight-gradient GEMM (csrc/hip/wgrad.hip) vs hipBLASLt
(torch addmm_, beta = 1) on the Llama-3-8B wgrad shapes, T = 24576 tokens
(micro-batch 6 x 4096).  Random uniform operands, interleaved rounds in one
process (guide §5.4 rules 24/25), median of the rounds.

    python scripts/wgrad_nt_bench.py [--tokens T] [--rounds R] [--only NAME]
"""
import argparse
import json
import statistics

import torch

from tf_operator_amd.ops import gemm

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    T = a.tokens
    # numerics first: small shape against an fp32 reference
    torch.manual_seed(0)
    for (n, k, t, beta) in ((256, 256, 512, 0), (512, 768, 1024, 1), (1024, 512, 4096, 1)):
        dy = (torch.rand(t, n, device=dev) * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(t, k, device=dev) * 2 - 1).to(torch.bfloat16)
        g0 = (torch.rand(n, k, device=dev) * 2 - 1).to(torch.bfloat16)
        ref = dy.float().t() @ x.float() + (g0.float() if beta else 0)
        for split in (1, 2, 4):
            if t % (128 * split):
                continue
            g = g0.clone()
            gemm.wgrad_hip_(g, dy, x, beta=beta, split=split)
            err = float((g.float() - ref).abs().max() / ref.abs().max())
            print(json.dumps({"check": [n, k, t, beta, split], "rel_err": round(err, 5)}), flush=True)
            assert err < 1e-2, err
    for name, (N, K) in SHAPES.items():
        if a.only and name != a.only:
            continue
        dy = (torch.rand(T, N, device=dev) * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(T, K, device=dev) * 2 - 1).to(torch.bfloat16)
        g_t = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
        g_h = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
        auto = gemm._lib.call_ret("toa_wgrad_split", N, K, T)
        variants = {"hipblaslt": lambda: g_t.addmm_(dy.t(), x)}
        for sp in sorted({1, 2, auto}):
            variants[f"hip_s{sp}"] = (lambda sp=sp: gemm.wgrad_hip_(g_h, dy, x, 1.0, sp))
        # one accumulation each, compared (same beta=1 from zero)
        g_t.zero_()
        g_h.zero_()
        g_t.addmm_(dy.t(), x)
        gemm.wgrad_hip_(g_h, dy, x, 1.0)
        rel = float((g_h.float() - g_t.float()).abs().max() / g_t.float().abs().max())
        for f in variants.values():
            f()
        torch.cuda.synchronize()
        res = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, f in variants.items():
                res[k].append(timeit(f, a.reps))
        flops = 2.0 * N * K * T
        out = {"name": name, "N": N, "K": K, "T": T, "auto_split": auto, "rel_vs_hipblaslt": round(rel, 5)}
        for k, v in res.items():
            ms = statistics.median(v)
            out[k] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}
        print(json.dumps(out), flush=True)
        del dy, x, g_t, g_h
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
