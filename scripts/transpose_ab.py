"""The W^T refresh transposes at the Llama-3-8B weight shapes: the register
kernel (variant 0, 64 x 64 tiles, 128-byte runs) against the LDS-staged one
(variant 1, 128 x 128 tiles, 256-byte runs), interleaved rounds, outputs
compared bit for bit.

    python scripts/transpose_ab.py [--rounds 6]
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {}
    for name, (R, C) in SHAPES.items():
        src = torch.randn(R, C, device=dev).to(torch.bfloat16)
        dsts = {v: torch.empty(C, R, device=dev, dtype=torch.bfloat16) for v in (0, 1)}

        def run(v):
            _lib.call("toa_transpose_set_variant", v)
            _lib.call("toa_transpose_bf16", _lib.ptr(src), C, _lib.ptr(dsts[v]), R, R, C, _lib.stream(src))

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
        nbytes = 2 * R * C * 2
        out[name] = {f"v{v}": {"ms": round(statistics.median(t), 4),
                               "TBps": round(nbytes / statistics.median(t) / 1e9, 2)} for v, t in times.items()}
        out[name]["bit_identical"] = bool(torch.equal(dsts[0], dsts[1]) and torch.equal(dsts[1], src.t()))
        print(json.dumps({name: out[name]}), flush=True)
        del src, dsts
    _lib.call("toa_transpose_set_variant", 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
