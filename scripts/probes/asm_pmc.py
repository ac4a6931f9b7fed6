"""Counter subject: the hand-written assembly GEMM (toa_gemm_tn_asm_plain) and
hipBLASLt's non-stream-K kernel on the same TN problem (x W^T at the
Llama-3-8B gate|up shape, T = 24576, N = 28672, K = 4096), 5 calls each after
a warm-up, random operands.

    rocprofv3 --pmc ... -- python3 scripts/probes/asm_pmc.py
    python scripts/pmc_summary.py <out> toa_gemm_tn_asm Cijk
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tf_operator_amd.ops import _lib, gemm  # noqa: E402


def main():
    # ASM_PMC_SHAPE="T,N,K" (default: the gate|up forward)
    T, N, K = (int(v) for v in os.environ.get("ASM_PMC_SHAPE", "24576,28672,4096").split(","))
    torch.manual_seed(0)
    x = (torch.rand(T, K, device="cuda") - 0.5).to(torch.bfloat16)
    w = (torch.rand(N, K, device="cuda") - 0.5).to(torch.bfloat16)
    y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    gemm.set_mode("nosk")

    def asm():
        _lib.call("toa_gemm_asm", _lib.ptr(x), K, _lib.ptr(w), K, _lib.ptr(y), N, T, N, K, _lib.stream(x))

    for _ in range(2):
        asm()
        gemm.linear_fwd(x, w)
    torch.cuda.synchronize()
    for _ in range(5):
        asm()
    for _ in range(5):
        gemm.linear_fwd(x, w)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
