"""Hand-written TN GEMM (csrc/hip/gemm_tn.hip) vs hipBLASLt at the
Llama-3-8B forward / data-gradient forms (T = 24576 tokens), in-process
interleaved rounds on random operands (guide §5.4 rules 24/25):

    tn        toa_gemm_tn (plain epilogue), full-line 64-k main loop (default)
    tn32      the same with the 32-k main loop (toa_gemm_tn_set_variant(0))
    tn4w      one wave per SIMD, 128 x 128 per wave (toa_gemm_tn_set_variant(2))
    tnrot     tn with a per-tile k rotation (toa_gemm_tn_set_variant(3))
    tnpad     tn on operands with row stride K + 64 (L2-channel probe)
    tndm      tn with the LDS-DMA issued between the MFMAs (variant 4)
    tn32d3    tn32 with the DMA three 32-k stages ahead (variant 5)
    tn5       full lines in a five-slot ring (variant 6)
    blt_nosk  hipBLASLt, the non-stream-K table (ops/gemm.py ``nosk``)
    blt_heur  hipBLASLt heuristic (torch.matmul; stream-K kernels)

plus the fused MLP ends: gate|up + SwiGLU (one kernel) vs hipBLASLt +
swiglu_fwd_rows_kernel, and the down projection's dgrad + SwiGLU backward vs
hipBLASLt + swiglu_bwd_rows_kernel.

    python scripts/gemm_tn_bench.py [--tokens 24576] [--rounds 5] [--reps 5]
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib, gemm, llm  # noqa: E402

FORMS = {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096)}


def timer(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    T = a.tokens
    torch.manual_seed(0)
    out = {"tokens": T, "forms": {}}
    for name, (K, N) in FORMS.items():
        for kind, (kk, nn) in (("fwd", (K, N)), ("dgrad_wt", (N, K))):
            x = torch.randn(T, kk, device="cuda").to(torch.bfloat16)
            w = (torch.randn(nn, kk, device="cuda") / kk ** 0.5).to(torch.bfloat16)
            y = torch.empty(T, nn, device="cuda", dtype=torch.bfloat16)

            def tn():
                _lib.call("toa_gemm_tn", _lib.ptr(x), kk, _lib.ptr(w), kk, _lib.ptr(y), nn, T, nn, kk,
                          _lib.stream(x))

            def tn32():
                _lib.call("toa_gemm_tn_set_variant", 0)
                tn()
                _lib.call("toa_gemm_tn_set_variant", -1)

            def nosk():
                gemm.set_mode("nosk")
                gemm.linear_fwd(x, w)

            def heur():
                torch.matmul(x, w.t())

            def tn4w():
                _lib.call("toa_gemm_tn_set_variant", 2)
                tn()
                _lib.call("toa_gemm_tn_set_variant", -1)

            def tnrot():
                _lib.call("toa_gemm_tn_set_variant", 3)
                tn()
                _lib.call("toa_gemm_tn_set_variant", -1)

            def tndm():
                _lib.call("toa_gemm_tn_set_variant", 4)
                tn()
                _lib.call("toa_gemm_tn_set_variant", -1)

            def tn32d3():
                _lib.call("toa_gemm_tn_set_variant", 5)
                tn()
                _lib.call("toa_gemm_tn_set_variant", -1)

            def tn5():
                _lib.call("toa_gemm_tn_set_variant", 6)
                tn()
                _lib.call("toa_gemm_tn_set_variant", -1)

            xp = torch.empty(T, kk + 64, device="cuda", dtype=torch.bfloat16)[:, :kk]
            xp.copy_(x)
            wp = torch.empty(nn, kk + 64, device="cuda", dtype=torch.bfloat16)[:, :kk]
            wp.copy_(w)

            def tnpad():
                _lib.call("toa_gemm_tn", _lib.ptr(xp), kk + 64, _lib.ptr(wp), kk + 64, _lib.ptr(y), nn, T, nn, kk,
                          _lib.stream(x))

            arms = (("tn", tn), ("tn32", tn32), ("tn4w", tn4w), ("tnrot", tnrot), ("tnpad", tnpad), ("tndm", tndm), ("tn32d3", tn32d3), ("tn5", tn5),
                    ("blt_nosk", nosk), ("blt_heur", heur))
            ts = {k2: [] for k2, _ in arms}
            for _ in range(a.rounds):
                for k2, f in arms:
                    ts[k2].append(timer(f, a.reps))
            ref = (x.float() @ w.float().t())
            tn()
            torch.cuda.synchronize()
            err = float((y.float() - ref).norm() / ref.norm())
            fl = 2.0 * T * nn * kk
            out["forms"][f"{name}.{kind}"] = {k2: {"ms": round(statistics.median(v), 4),
                                                   "TFps": round(fl / statistics.median(v) / 1e9, 1)}
                                              for k2, v in ts.items()}
            out["forms"][f"{name}.{kind}"]["tn_rel_err"] = round(err, 5)
            print(json.dumps({f"{name}.{kind}": out["forms"][f"{name}.{kind}"]}), flush=True)
            del x, w, y, ref, xp, wp
    # fused MLP ends at the gate|up and down shapes
    F_, Hd = 14336, 4096
    x = torch.randn(T, Hd, device="cuda").to(torch.bfloat16)
    wgu = (torch.randn(2 * F_, Hd, device="cuda") / Hd ** 0.5).to(torch.bfloat16)
    wd = (torch.randn(Hd, F_, device="cuda") / F_ ** 0.5).to(torch.bfloat16)
    wd._toa_wt = wd.t().contiguous()
    d2 = torch.randn(T, Hd, device="cuda").to(torch.bfloat16)

    def fused_fwd():
        gemm.set_mode("hip")
        return gemm.swiglu_gate_up(x, wgu)

    def unfused_fwd():
        gemm.set_mode("nosk")
        return llm.swiglu(gemm.linear_fwd(x, wgu))

    gu, _ = fused_fwd()

    def fused_bwd():
        gemm.set_mode("hip")
        return gemm.swiglu_down_dgrad(d2, wd, gu)

    def unfused_bwd():
        gemm.set_mode("nosk")
        return llm.swiglu_bwd(gemm.linear_fwd(d2, wd._toa_wt), gu)

    ts = {k: [] for k in ("fused_fwd", "unfused_fwd", "fused_bwd", "unfused_bwd")}
    for _ in range(a.rounds):
        for k, f in (("fused_fwd", fused_fwd), ("unfused_fwd", unfused_fwd), ("fused_bwd", fused_bwd),
                     ("unfused_bwd", unfused_bwd)):
            ts[k].append(timer(f, a.reps))
    out["mlp"] = {k: round(statistics.median(v), 4) for k, v in ts.items()}
    print(json.dumps({"mlp_ms": out["mlp"]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
