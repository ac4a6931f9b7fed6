"""wgrad layouts: dW[N,K] += dY^T X as (a) NT on the natural layouts (what
the step runs), (b) TN on transposed copies dY^T [N,T], X^T [K,T] (+ the
two transposes), (c) NN on dY^T only.  Cold-ish: a 1 GB buffer is rewritten
between reps so operands come from HBM like in the step."""
import sys

import torch

T = 16384
SHAPES = {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096),
          "lm_head": (4096, 128256)}
flush = torch.empty(256 * 2**20, device="cuda", dtype=torch.float32)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    tot = 0.0
    for i in range(reps):
        flush.fill_(i)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        tot += s.elapsed_time(e)
    return tot / reps


for name, (K, N) in SHAPES.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * T * K * N
    nt = timeit(lambda: g.addmm_(dy.t(), x))
    xt = x.t().contiguous()
    dyt = dy.t().contiguous()
    tr = timeit(lambda: (x.t().contiguous(), dy.t().contiguous()))
    tn = timeit(lambda: g.addmm_(dyt, xt.t()))
    nn = timeit(lambda: g.addmm_(dyt, x))
    tr1 = timeit(lambda: dy.t().contiguous())
    print(f"{name:8s} NT {nt:7.3f} ms ({fl/nt/1e9:6.0f} TF) | TN {tn:7.3f} ({fl/tn/1e9:6.0f}) + 2 transposes {tr:6.3f}"
          f" = {tn+tr:7.3f} | NN {nn:7.3f} ({fl/nn/1e9:6.0f}) + 1 transpose {tr1:6.3f} = {nn+tr1:7.3f}", flush=True)
    del x, dy, g, xt, dyt
