"""Counter subject for the attention kernels at the Llama-3-8B bench shape
(B=6, H=32, Hkv=8, S=4096, D=128, causal, packed GQA): 5 forward + backward
passes (dS-form backward) with the HIP LDS-DMA forward and the HIP dK/dV,
then 5 with the assembly forward and the assembly dK/dV.  Used with
scripts/gpu_attn_pmc.sh."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tf_operator_amd.ops import _lib, llm  # noqa: E402


def main():
    B, H, Hk, S, D = 6, 32, 8, 4096, 128
    torch.manual_seed(0)
    q = torch.randn(B, H, S, D, device="cuda").to(torch.bfloat16).requires_grad_()
    k = torch.randn(B, Hk, S, D, device="cuda").to(torch.bfloat16).requires_grad_()
    v = torch.randn(B, Hk, S, D, device="cuda").to(torch.bfloat16).requires_grad_()
    do = torch.randn(B, H, S, D, device="cuda").to(torch.bfloat16)
    for form, dkdv in ((1, 0), (2, 1)):
        _lib.call("toa_attn_set_fwd_variant", form)
        _lib.call("toa_attn_set_dkdv_variant", dkdv)
        for _ in range(5):
            o = llm._FlashAttn.apply(q, k, v, 1 / math.sqrt(D))
            o.backward(do)
            q.grad = k.grad = v.grad = None
        torch.cuda.synchronize()
    _lib.call("toa_attn_set_fwd_variant", -1)
    _lib.call("toa_attn_set_dkdv_variant", -1)
    print("ok", flush=True)


if __name__ == "__main__":
    main()
