"""Micro-benchmark: HIP flash attention (packed GQA) vs torch SDPA (aotriton,
expanded K/V) at the Llama-3-8B training shape.  Prints ms and TFLOP/s."""
import math
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import llm  # noqa: E402

B, H, Hk, S, D = 4, 32, 8, 4096, 128
dev = "cuda"
torch.manual_seed(0)
XS = float(os.environ.get("XS", "1"))    # input scale (q, k, v)
GS = float(os.environ.get("GS", "1"))    # upstream-gradient scale
q = (torch.randn(B, H, S, D, device=dev) * XS).to(torch.bfloat16).requires_grad_()
k = (torch.randn(B, Hk, S, D, device=dev) * XS).to(torch.bfloat16).requires_grad_()
v = (torch.randn(B, Hk, S, D, device=dev) * XS).to(torch.bfloat16).requires_grad_()
do = (torch.randn(B, H, S, D, device=dev) * GS).to(torch.bfloat16)
scale = 1 / math.sqrt(D)
flops_fwd = 4 * B * H * S * S * D / 2


def hip_fwd():
    return llm._FlashAttn.apply(q, k, v, scale)


def sdpa_fwd():
    kk = k.repeat_interleave(H // Hk, 1)
    vv = v.repeat_interleave(H // Hk, 1)
    return torch.nn.functional.scaled_dot_product_attention(q, kk, vv, is_causal=True, scale=scale)


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


print(f"XS={XS} GS={GS}")
for name, f in (("hip", hip_fwd), ("sdpa", sdpa_fwd)):
    with torch.no_grad():
        tf = timeit(f)
    tfb = timeit(lambda: torch.autograd.backward(f(), do))
    print(f"{name:5s} fwd {tf:7.3f} ms ({flops_fwd / tf / 1e9:6.1f} TF)  fwd+bwd {tfb:7.3f} ms "
          f"({3.5 * flops_fwd / tfb / 1e9:6.1f} TF eff)", flush=True)
