"""RMSNorm backward at the bench shape (24576 x 4096, bf16, with the
residual gradient added): the residual-gradient loads hoisted before the
row-sum barrier (toa_norm_set_bwd_hoist 1, default) against after it (0),
interleaved rounds, outputs compared bit for bit.

    python scripts/rms_bwd_ab.py [--rows 24576] [--cols 4096] [--rounds 8]
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=24576)
    ap.add_argument("--cols", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    R, C = a.rows, a.cols
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    dy, h, dadd = (torch.randn(R, C, device=dev).to(torch.bfloat16) for _ in range(3))
    w = torch.randn(C, device=dev).to(torch.bfloat16)
    rstd = torch.rand(R, device=dev) + 0.5
    nb = _lib.lib().toa_norm_bwd_blocks(R, C)
    partial = torch.empty(nb * C, device=dev)
    dw = torch.empty(C, device=dev, dtype=torch.bfloat16)
    outs = {v: torch.empty(R, C, device=dev, dtype=torch.bfloat16) for v in (0, 1)}

    def run(v):
        _lib.call("toa_norm_set_bwd_hoist", v)
        _lib.call("toa_rmsnorm_bwd", 0, _lib.ptr(dy), _lib.ptr(h), _lib.ptr(w), _lib.ptr(rstd), _lib.ptr(dadd),
                  _lib.ptr(outs[v]), _lib.ptr(partial), _lib.ptr(dw), 1, 0, R, C, _lib.stream(dy))

    times = {0: [], 1: []}
    for r in range(a.rounds):
        for v in ((0, 1) if r % 2 == 0 else (1, 0)):
            run(v)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run(v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.reps)
    _lib.call("toa_norm_set_bwd_hoist", 1)
    nbytes = 4 * R * C * 2
    out = {f"hoist{v}": {"ms": round(statistics.median(t), 4), "TBps": round(nbytes / statistics.median(t) / 1e9, 2)}
           for v, t in times.items()}
    out["bit_identical"] = bool(torch.equal(outs[0], outs[1]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
