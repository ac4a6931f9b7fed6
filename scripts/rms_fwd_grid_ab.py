"""RMSNorm forward (+ residual add) at the Llama-3-8B bench shape
(24576 x 4096 bf16) under several grid caps of the one-row-per-workgroup
kernel (toa_norm_set_fwd_cap), interleaved rounds in one process; outputs
checked identical across caps.

    python scripts/rms_fwd_grid_ab.py
"""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib  # noqa: E402


def main():
    T, C = 24576, 4096
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(T, C, device="cuda", generator=g).to(torch.bfloat16)
    r = torch.randn(T, C, device="cuda", generator=g).to(torch.bfloat16)
    w = torch.randn(C, device="cuda", generator=g).to(torch.bfloat16)
    h, y = torch.empty_like(x), torch.empty_like(x)
    rstd = torch.empty(T, device="cuda")
    s = _lib.stream(x)
    caps = [2048, 8192, 24576]
    outs, times = {}, {c: [] for c in caps}

    def run():
        _lib.call("toa_rmsnorm_fwd", _lib.dtype_code(x), _lib.ptr(x), _lib.ptr(r), _lib.ptr(h), _lib.ptr(w),
                  _lib.ptr(y), _lib.ptr(rstd), T, C, 1e-5, s)

    for rnd in range(6):
        for c in (caps if rnd % 2 == 0 else caps[::-1]):
            _lib.call("toa_norm_set_fwd_cap", c)
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / 20)
            outs[c] = y.clone()
    _lib.call("toa_norm_set_fwd_cap", 0)
    same = all(torch.equal(outs[c], outs[caps[0]]) for c in caps)
    print(json.dumps({"ms": {c: round(statistics.median(v), 4) for c, v in times.items()}, "identical": same}))


if __name__ == "__main__":
    main()
