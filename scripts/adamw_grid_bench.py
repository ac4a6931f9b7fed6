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
    ap.add_argument("--caps", default="2,16,64,255", help="grid caps / 1024")
    ap.add_argument("--two", action="store_true", help="add the two-chunks-per-thread arms (variant bit 2)")
    a = ap.parse_args()
    a.caps = [int(c) for c in a.caps.split(",")]
    torch.manual_seed(0)
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    ps = [torch.nn.Parameter(torch.randn(*s, device="cuda").to(torch.bfloat16) * 0.02) for s in shapes]
    flat = FlatParams(ps)
    wt = TransposedWeights(flat, ps)
    with_wt = FlatAdamW(flat, lr=1e-4, max_grad_norm=0.0, post_update=wt.refresh)
    plain = FlatAdamW(flat, lr=1e-4, max_grad_norm=0.0)
    flat.grad.copy_(torch.randn(flat.grad.numel(), device="cuda").to(flat.grad.dtype) * 1e-3)
    nparam = sum(p.numel() for p in ps)
    # arm -> (variant word, optimizer): bits 8.. grid cap / 1024, bit 2 two chunks per thread
    arms = {f"cap{c}" + ("x2" if two else "") + ("+refresh" if o is with_wt else ""): (1 | 2 | (4 if two else 0) | (c << 8), o)
            for c in a.caps for two in ((False, True) if a.two else (False,)) for o in (plain, with_wt)}
    times = {k: [] for k in arms}
    if a.two:   # the two-chunk kernel updates every element as the one-chunk kernel does
        state = [t.clone() for t in (flat.master, flat.exp_avg, flat.exp_avg_sq, flat.param)]
        outs = []
        for word in (1 | 2 | (255 << 8), 1 | 2 | 4 | (255 << 8)):
            for t, s0 in zip((flat.master, flat.exp_avg, flat.exp_avg_sq, flat.param), state):
                t.data.copy_(s0)
            _lib.call_ret("toa_set_stream_variant", word)
            plain.step()
            torch.cuda.synchronize()
            outs.append([t.clone() for t in (flat.master, flat.exp_avg, flat.exp_avg_sq, flat.param)])
        print(json.dumps({"two_chunk_bit_identical": all(torch.equal(x, y) for x, y in zip(*outs))}), flush=True)

    def run(arm):
        word, o = arms[arm]
        _lib.call_ret("toa_set_stream_variant", word)
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
