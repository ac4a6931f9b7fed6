"""Counter subject: the hand-written assembly GEMM (toa_gemm_tn_asm_plain) and
hipBLASLt's non-stream-K kernel on the same TN problem (x W^T at the
Llama-3-8B gate|up shape, T = 24576, N = 28672, K = 4096), 5 calls each after
a warm-up, random operands.

    rocprofv3 --pmc ... -- python3 scripts/probes/asm_pmc.py
    python scripts/pmc_summary.py <out> toa_gemm_tn_asm Cijk

ASM_PMC_ORDER=interleave alternates the two kernels call by call (same
thermal state for both); ASM_PMC_WGRAD=1 measures the weight-gradient form
instead: the assembly NT kernel (toa_wgrad_nt_asm) against the HIP one
(wgrad_nt_kernel) at dW[N, K] = dY^T X over T tokens.
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

    def other():
        gemm.linear_fwd(x, w)

    if os.environ.get("ASM_PMC_WGRAD") == "1":
        dy = (torch.rand(T, N, device="cuda") - 0.5).to(torch.bfloat16)
        g = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        ws = torch.empty(max(int(_lib.call_ret("toa_wgrad_workspace", N, K, T, 0)), 16) // 4, device="cuda",
                         dtype=torch.float32)

        def asm():  # noqa: F811
            _lib.call("toa_wgrad_asm", _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(g), K, _lib.ptr(ws), N, K, T, 0, 0,
                      _lib.stream(dy))

        def other():  # noqa: F811
            _lib.call("toa_wgrad", _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(g), K, _lib.ptr(ws), N, K, T, 0, 0,
                      _lib.stream(dy))

    for _ in range(2):
        asm()
        other()
    torch.cuda.synchronize()
    if os.environ.get("ASM_PMC_ORDER") == "interleave":
        for _ in range(5):
            asm()
            other()
    else:
        for _ in range(5):
            asm()
        for _ in range(5):
            other()
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
