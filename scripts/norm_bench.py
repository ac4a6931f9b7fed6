"""RMSNorm kernels at the Llama-3-8B step shape (6 x 4096 tokens, 4096 wide,
bf16): time and effective HBM bandwidth of the fused add+norm forward and the
backward (dx + residual-stream gradient, weight-gradient partials + column
reduce).

    python scripts/norm_bench.py [--rows 24576] [--cols 4096] [--libs a.so,b.so]

--libs: single-source builds of norm.hip (scripts/ab/build_variants.py) timed
interleaved in one process; default: the in-tree libtoa_hip.so, with the
backward's two forms interleaved (toa_norm_set_row: "row" = one row per
workgroup, the default; "wave" = one row per wave with a second read).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tf_operator_amd.ops import _lib  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=24576)
    ap.add_argument("--cols", type=int, default=4096)
    ap.add_argument("--libs", default="")
    a = ap.parse_args()
    libs = {}
    for path in [p for p in a.libs.split(",") if p] or [_lib.LIB_PATH]:
        L = ctypes.CDLL(path)
        for n in ("toa_rmsnorm_fwd", "toa_rmsnorm_bwd", "toa_norm_bwd_blocks"):
            getattr(L, n).argtypes = _lib._SIGS[n]
            getattr(L, n).restype = ctypes.c_int
        if not a.libs and hasattr(L, "toa_norm_set_row"):
            L.toa_norm_set_row.argtypes = [ctypes.c_int]
            libs["row"] = (L, 1)
            libs["wave"] = (L, 0)
        else:
            libs[os.path.basename(path)] = (L, None)
    results = {}
    for rnd in range(3):
        for name, (L, form) in libs.items():
            if form is not None:
                L.toa_norm_set_row(form)
            r = run(a, L)
            results.setdefault(name, []).append(r)
            print(json.dumps({"lib": name, "round": rnd, **r}), flush=True)
    summ = {n: {k: min(x[k] for x in rs) for k in ("fwd_ms", "bwd_ms")} for n, rs in results.items()}
    print(json.dumps({"best_ms": summ}))


def run(a, L):
    R, C = a.rows, a.cols
    dev = "cuda"
    bf = torch.bfloat16
    x, r, dy, dh = (torch.randn(R, C, device=dev, dtype=bf) for _ in range(4))
    w = torch.rand(C, device=dev, dtype=bf) + 0.5
    h, y, dx = (torch.empty(R, C, device=dev, dtype=bf) for _ in range(3))
    rstd = torch.empty(R, device=dev, dtype=torch.float32)
    nb = L.toa_norm_bwd_blocks(R, C)
    part = torch.empty(nb * C, device=dev, dtype=torch.float32)
    dw = torch.zeros(C, device=dev, dtype=torch.float32)
    s = _lib.stream(x)

    def call(name, *args):
        rc = getattr(L, name)(*args)
        if rc:
            raise RuntimeError(f"{name} -> {rc}")

    def fwd():
        call("toa_rmsnorm_fwd", 0, _lib.ptr(x), _lib.ptr(r), _lib.ptr(h), _lib.ptr(w), _lib.ptr(y),
             _lib.ptr(rstd), R, C, 1e-5, s)

    def bwd():
        call("toa_rmsnorm_bwd", 0, _lib.ptr(dy), _lib.ptr(h), _lib.ptr(w), _lib.ptr(rstd), _lib.ptr(dh),
             _lib.ptr(dx), _lib.ptr(part), _lib.ptr(dw), 0, 1, R, C, s)

    tf = timeit(fwd)
    tb = timeit(bwd)
    # numerics of the backward against fp32 PyTorch
    hf = h.float()
    rs = torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5)
    xh = hf * rs
    g = dy.float() * w.float()
    ref = (g - xh * (g * xh).mean(-1, keepdim=True)) * rs + dh.float()
    dw.zero_()
    bwd()
    torch.cuda.synchronize()
    err = ((dx.float() - ref).abs().max() / ref.abs().max()).item()
    dw_ref = (dy.float() * xh).sum(0)
    dw_err = ((dw - dw_ref).abs().max() / dw_ref.abs().max()).item()
    eb = 2 * R * C
    out = {"rows": R, "cols": C, "bwd_blocks": nb,
           "fwd_ms": round(tf, 4), "fwd_GBps": round(4 * eb / tf / 1e6, 1),
           "bwd_ms": round(tb, 4), "bwd_GBps": round(4 * eb / tb / 1e6, 1),
           "bwd_dx_rel_err": err, "bwd_dw_rel_err": dw_err}
    assert err < 2e-2 and dw_err < 1e-2, out
    return out


if __name__ == "__main__":
    main()
