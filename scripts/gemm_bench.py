"""Per-shape GEMM throughput of the Llama-3-8B training step (T = 4 x 4096
tokens): forward, dgrad and wgrad(+=) forms exactly as ops/linear.py issues
them, on hipBLASLt (and rocBLAS for comparison)."""
import sys

import torch

T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
SHAPES = {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096),
          "lm_head": (4096, 128256)}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def run(lib):
    torch.backends.cuda.preferred_blas_library(lib)
    tot = 0.0
    for name, (K, N) in SHAPES.items():
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * K * N
        for form, fn in (("fwd", lambda: torch.matmul(x, w.t())), ("dgrad", lambda: torch.matmul(dy, w)),
                         ("wgrad", lambda: g.addmm_(dy.t(), x))):
            ms = timeit(fn)
            mult = 32 if name != "lm_head" else 1
            tot += ms * mult
            print(f"{lib:9s} {name:8s} {form:6s} T={T} K={K:6d} N={N:6d}: {ms:7.3f} ms  {fl / ms / 1e9:7.1f} TF/s",
                  flush=True)
        del x, w, dy, g
    print(f"{lib}: est. GEMM time per step {tot:.1f} ms")


if __name__ == "__main__":
    for lib in sys.argv[2:] or ["cublaslt", "cublas"]:
        run(lib)
