"""In-process A/B of the weight-gradient kernel variants at the Llama-3-8B
shapes (T = 6 x 4096 tokens): the 8-wave kernel against the 4-wave
(one wave per SIMD, 32x32x16 MFMA) one and the 8-wave one with its DMA
three phases ahead (variant 3), switched with toa_wgrad_set_variant.  Interleaved rounds, median ms; the two results
compared.

    python scripts/wgrad_variant_ab.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tf_operator_amd.ops import _lib as L  # noqa: E402
from tf_operator_amd.ops import gemm  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}
T = 24576
VARIANTS = tuple(int(v) for v in os.environ.get("WGRAD_AB_VARIANTS", "8,3").split(","))


def main():
    res = {}
    for name, (N, K) in SHAPES.items():
        torch.manual_seed(0)
        dy = (torch.rand(T, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(T, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        outs = {}
        for v in VARIANTS:
            assert L.call_ret("toa_wgrad_set_variant", v) == 0
            g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
            gemm.wgrad_hip_(g, dy, x, beta=0.0)
            outs[v] = g
        torch.cuda.synchronize()
        diff = {v: float((outs[8].float() - outs[v].float()).abs().max()) for v in VARIANTS if v != 8}
        times = {v: [] for v in VARIANTS}
        g = outs[8]
        for _ in range(7):
            for v in VARIANTS:
                L.call_ret("toa_wgrad_set_variant", v)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(5):
                    gemm.wgrad_hip_(g, dy, x, beta=1.0)
                b.record()
                torch.cuda.synchronize()
                times[v].append(a.elapsed_time(b) / 5)
        fl = 2.0 * N * K * T
        res[name] = {f"{v}w": {"ms": round(statistics.median(t), 4), "tflops": round(fl / statistics.median(t) / 1e9, 1)}
                     for v, t in times.items()}
        res[name]["max_abs_diff"] = diff
        print(json.dumps({name: res[name]}), flush=True)
        del dy, x, outs, g
        torch.cuda.empty_cache()
    L.call_ret("toa_wgrad_set_variant", 8)
    step = {f"{v}w": round(sum(res[n][f"{v}w"]["ms"] * (1 if n == "lm_head" else 32) for n in SHAPES), 2)
            for v in VARIANTS}
    print(json.dumps({"wgrad_ms_per_step": step}))


if __name__ == "__main__":
    main()
