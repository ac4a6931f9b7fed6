"""The flat AdamW at several grid sizes (toa_set_stream_variant bits 8..:
grid cap / 1024), and the W^T refresh behind it, on one Llama-3-8B layer's
linear weights (qkv, o, gate_up, down: 218M parameters), in one process,
interleaved rounds.

    python scripts/adamw_grid_bench.py [--rounds 6] [--iters 10]
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402
from tf_operator_amd.ops.optim import FlatAdamW  # noqa: E402
from tf_operator_amd.ops.wt import TransposedWeights  # noqa: E402
from tf_operator_amd.parallel.flat import FlatParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.manual_seed(0)
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    ps = [torch.nn.Parameter(torch.randn(*s, device="cuda").to(torch.bfloat16) * 0.02) for s in shapes]
    flat = FlatParams(ps)
    wt = TransposedWeights(flat, ps)
    with_wt = FlatAdamW(flat, lr=1e-4, max_grad_norm=0.0, post_update=wt.refresh)
    plain = FlatAdamW(flat, lr=1e-4, max_grad_norm=0.0)
    flat.grad.copy_(torch.randn(flat.grad.numel(), device="cuda").to(flat.grad.dtype) * 1e-3)
    nparam = sum(p.numel() for p in ps)
    arms = {f"cap{c}" + ("+refresh" if o is with_wt else ""): (c, o)
            for c in (2, 16, 64, 255) for o in (plain, with_wt)}
    times = {k: [] for k in arms}

    def run(arm):
        cap, o = arms[arm]
        _lib.call_ret("toa_set_stream_variant", 1 | 2 | (cap << 8))
        o.step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            o.step()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    for r in range(a.rounds):
        order = list(arms) if r % 2 == 0 else list(arms)[::-1]
        for arm in order:
            times[arm].append(run(arm))
    _lib.call_ret("toa_set_stream_variant", 1 | 2 | (255 << 8))
    out = {k: {"ms": round(statistics.median(v), 4), "TBps_28B": round(nparam * 28 / statistics.median(v) / 1e9, 3)}
           for k, v in times.items()}
    out["params"] = nparam
    print(json.dumps(out))


if __name__ == "__main__":
    main()
