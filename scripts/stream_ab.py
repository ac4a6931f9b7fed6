"""In-process A/B of the HBM-streaming kernel variants (toa_set_stream_variant).

AdamW over a flat 1.5e9-parameter state (bf16 grad, fp32 master/m/v, bf16
param: 28 B per parameter, ~42 GB touched per call) and SwiGLU forward /
backward at the Llama-3-8B bench shape (T = 24576, F = 14336).  Arms are
interleaved round-robin in one process so clock and thermal drift hit every
arm alike; each arm reports the median of its reps and the effective HBM
rate.  Outputs of every arm are checked bit-identical to arm 0.

    python scripts/stream_ab.py [--reps 8] [--n 1.5e9]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tf_operator_amd.ops import _lib  # noqa: E402


def timed(fn, reps_out, stream):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    fn()
    e.record(stream)
    e.synchronize()
    reps_out.append(s.elapsed_time(e))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--n", type=float, default=1.5e9)
    ap.add_argument("--T", type=int, default=24576)
    ap.add_argument("--F", type=int, default=14336)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)

    # ---- AdamW ----
    n = int(a.n) // 64 * 64
    master0 = torch.randn(n, device=dev, generator=g) * 0.02
    grad = (torch.randn(n, device=dev, generator=g) * 1e-3).bfloat16()
    m0 = torch.randn(n, device=dev, generator=g) * 1e-4
    v0 = torch.rand(n, device=dev, generator=g) * 1e-6
    master, m, v = master0.clone(), m0.clone(), v0.clone()
    param = torch.empty(n, device=dev, dtype=torch.bfloat16)
    ref = None

    def adamw():
        _lib.call("toa_adamw_flat", master.data_ptr(), param.data_ptr(), grad.data_ptr(), 1, m.data_ptr(),
                  v.data_ptr(), n, 1e-4, 0.9, 0.95, 1e-8, 0.1, 10, 1.0, None, 0.0, sp)

    arms = {"adamw v0": 0, "adamw nt": 1, "adamw nt grid4k": 1 | (4 << 8), "adamw grid8k": 8 << 8,
            "adamw nt grid16k": 1 | (16 << 8)}
    times = {k: [] for k in arms}
    for k, var in arms.items():  # correctness: one step from the same state, bit-identical to arm 0
        master.copy_(master0), m.copy_(m0), v.copy_(v0)
        _lib.lib().toa_set_stream_variant(var)
        adamw()
        torch.cuda.synchronize()
        out = (master.clone(), m.clone(), v.clone(), param.clone())
        if ref is None:
            ref = out
        else:
            same = all(torch.equal(x, y) for x, y in zip(ref, out))
            print(f"{k}: bit-identical to arm 0: {same}", flush=True)
        del out
    del ref, master0, m0, v0
    for _ in range(a.reps):
        for k, var in arms.items():
            _lib.lib().toa_set_stream_variant(var)
            timed(adamw, times[k], st)
    nbytes = 28 * n
    for k, ts in times.items():
        med = statistics.median(ts)
        print(f"{k:22s} median {med:8.3f} ms  min {min(ts):8.3f}  {nbytes / med / 1e9:6.2f} TB/s  "
              f"(x{8.03e9 / n:.2f} -> {med * 8.03e9 / n:.1f} ms at Llama-3-8B)", flush=True)
    del master, m, v, param, grad
    torch.cuda.empty_cache()

    # ---- SwiGLU ----
    T, F = a.T, a.F
    gu = torch.randn(T, 2 * F, device=dev, generator=g).bfloat16()
    dout = torch.randn(T, F, device=dev, generator=g).bfloat16()
    out = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
    dgu = torch.empty(T, 2 * F, device=dev, dtype=torch.bfloat16)

    def fwd():
        _lib.call("toa_swiglu_fwd", gu.data_ptr(), out.data_ptr(), T, F, sp)

    def bwd():
        _lib.call("toa_swiglu_bwd", dout.data_ptr(), gu.data_ptr(), dgu.data_ptr(), T, F, sp)

    arms = {"swiglu flat": 0, "swiglu rows nt": 2}
    refs = None
    for k, var in arms.items():
        _lib.lib().toa_set_stream_variant(var)
        fwd(), bwd()
        torch.cuda.synchronize()
        o = (out.clone(), dgu.clone())
        if refs is None:
            refs = o
        else:
            print(f"{k}: bit-identical to arm 0: {all(torch.equal(x, y) for x, y in zip(refs, o))}", flush=True)
    tf = {k: [] for k in arms}
    tb = {k: [] for k in arms}
    for _ in range(a.reps * 2):
        for k, var in arms.items():
            _lib.lib().toa_set_stream_variant(var)
            timed(fwd, tf[k], st)
            timed(bwd, tb[k], st)
    bf, bb = T * F * 2 * 3, T * F * 2 * 5
    for k in arms:
        mf, mb = statistics.median(tf[k]), statistics.median(tb[k])
        print(f"{k:22s} fwd {mf:7.3f} ms {bf / mf / 1e9:5.2f} TB/s   bwd {mb:7.3f} ms {bb / mb / 1e9:5.2f} TB/s",
              flush=True)
    _lib.lib().toa_set_stream_variant(0)


if __name__ == "__main__":
    main()
