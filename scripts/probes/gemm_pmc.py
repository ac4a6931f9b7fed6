"""Counter subject for the GEMM comparison: the hand-written NT
weight-gradient kernel, the hand-written TN kernel (gemm_tn.hip: the
full-line 64-k main loop `gemm_tn64_kernel` and the 32-k one
`gemm_tn_kernel`) and hipBLASLt's TN form (the forward's x W^T) at the
Llama-3-8B gate|up shape, 5 calls each after a warm-up.

    rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES ... -- python3 scripts/probes/gemm_pmc.py
    python scripts/pmc_summary.py <out> wgrad_nt_kernel Cijk
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tf_operator_amd.ops import _lib, gemm  # noqa: E402


def main():
    T, N, K = 24576, 28672, 4096
    torch.manual_seed(0)
    dy = (torch.rand(T, N, device="cuda") - 0.5).to(torch.bfloat16)
    x = (torch.rand(T, K, device="cuda") - 0.5).to(torch.bfloat16)
    g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.rand(N, K, device="cuda") - 0.5).to(torch.bfloat16)
    assert gemm.wgrad_hip_ok(g, dy, x)
    for _ in range(2):
        gemm.wgrad_hip_(g, dy, x, beta=0.0)
        torch.matmul(x, w.t())
    torch.cuda.synchronize()
    for _ in range(5):
        gemm.wgrad_hip_(g, dy, x, beta=0.0)
    for _ in range(5):
        torch.matmul(x, w.t())
    y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    for v in (1, 0, 2):
        _lib.call("toa_gemm_tn_set_variant", v)
        for _ in range(7):
            _lib.call("toa_gemm_tn", _lib.ptr(x), K, _lib.ptr(w), K, _lib.ptr(y), N, T, N, K, _lib.stream(x))
    _lib.call("toa_gemm_tn_set_variant", -1)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
