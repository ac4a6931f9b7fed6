"""Data-gradient GEMM of the Llama-3-8B linears: dY W (NN, hipBLASLt) against
dY (W^T)^T on a transposed weight copy (the forward's TN form), plus the
cost of producing W^T with toa_transpose_bf16.  T = micro-batch x 4096."""
import json
import sys

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops.wt import transpose_into  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 24576
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


tot = {"nn": 0.0, "tn": 0.0, "tr": 0.0}
for name, (K, N) in SHAPES.items():
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    wt = torch.empty(K, N, device="cuda", dtype=torch.bfloat16)
    transpose_into(wt, w)
    assert torch.equal(wt, w.t().contiguous()), name
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    ref = torch.matmul(dy, w)
    got = torch.matmul(dy, wt.t())
    err = float((got.float() - ref.float()).abs().max() / ref.float().abs().max())
    fl = 2.0 * T * K * N
    nn = timeit(lambda: torch.matmul(dy, w))
    tn = timeit(lambda: torch.matmul(dy, wt.t()))
    tr = timeit(lambda: transpose_into(wt, w))
    mult = 32 if name != "lm_head" else 1
    tot["nn"] += nn * mult
    tot["tn"] += tn * mult
    tot["tr"] += tr * mult
    print(json.dumps({"name": name, "T": T, "K": K, "N": N, "rel_err": err, "nn_ms": round(nn, 4),
                      "nn_tflops": round(fl / nn / 1e9, 1), "tn_ms": round(tn, 4), "tn_tflops": round(fl / tn / 1e9, 1),
                      "transpose_ms": round(tr, 4), "transpose_GBps": round(4 * N * K / tr / 1e6, 1)}), flush=True)
    del w, wt, dy, ref, got
print(json.dumps({"per_step_ms": {k: round(v, 1) for k, v in tot.items()}}))
