"""How fast the flat AdamW runs when its stream may use only n CUs
(toa_stream_create_cu_mask, mode 0: CUs 0..n-1 of the mask; mode 1: spread):
the bandwidth curve says how many CUs the memory-bound update needs, and
mode 0 vs 1 at small n says whether the mask's bit order packs CUs into one
XCD (then mode 0 is capped by one XCD's share of the fabric).

    python scripts/cu_mask_probe.py [--params 218103808] [--reps 5]
"""
import argparse
import ctypes
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402
from tf_operator_amd.ops.optim import masked_stream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=218103808)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cus", default="8,16,32,48,64,96,128,256")
    a = ap.parse_args()
    n = a.params
    dev = torch.device("cuda", 0)
    master = torch.randn(n, device=dev)
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    g = torch.randn(n, device=dev).to(torch.bfloat16)
    p = master.to(torch.bfloat16)
    nbytes = n * (4 * 6 + 2 + 2)

    def run(stream):
        _lib.call("toa_adamw_flat", master.data_ptr(), p.data_ptr(), g.data_ptr(), 1, m.data_ptr(), v.data_ptr(), n,
                  1e-4, 0.9, 0.95, 1e-8, 0.1, 1, 1.0, None, 0.0, ctypes.c_void_p(stream.cuda_stream))

    streams = {"default": torch.cuda.current_stream(dev)}
    for c in [int(x) for x in a.cus.split(",")]:
        for mode in (0, 1):
            streams[f"n{c}_m{mode}"] = masked_stream(c, mode, dev)
    out = {}
    for name, st in streams.items():
        run(st)
        torch.cuda.synchronize()
        t = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            run(st)
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        ms = min(t) * 1e3
        out[name] = {"ms": round(ms, 3), "TBps": round(nbytes / (ms / 1e3) / 1e12, 2)}
        print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
