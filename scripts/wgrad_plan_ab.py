"""In-process A/B of the NT weight-gradient kernel's launch plans at the
Llama-3-8B shapes (T = 6 x 4096 tokens): a library built before the
tail-only split-K plan (uniform split of every tile, `toa_wgrad_split`)
against the current one (auto plan, split = 0).  Interleaved rounds,
median ms, and the two results compared.

    python scripts/wgrad_plan_ab.py build/variants/libtoa_hip_before_wgrad_plan.so [tf_operator_amd/lib/libtoa_hip.so]
"""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}
T = 24576
P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64


def load(path, new):
    L = ctypes.CDLL(path)
    L.toa_wgrad.argtypes = [P, I64, P, I64, P, I64, P, I, I, I, I, I, P]
    L.toa_wgrad.restype = I
    L.toa_wgrad_split.argtypes = [I, I, I]
    L.toa_wgrad_split.restype = I
    if new:
        L.toa_wgrad_workspace.argtypes = [I, I, I, I]
        L.toa_wgrad_workspace.restype = I64
    return L


def main():
    old_path = sys.argv[1]
    new_path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "tf_operator_amd", "lib", "libtoa_hip.so")
    libs = {"uniform_split": load(old_path, False), "tail_split": load(new_path, True)}
    st = P(torch.cuda.current_stream().cuda_stream)
    ptr = lambda t: P(t.data_ptr())  # noqa: E731
    res = {}
    for name, (N, K) in SHAPES.items():
        torch.manual_seed(0)
        dy = (torch.rand(T, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(T, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        outs, calls = {}, {}
        for arm, L in libs.items():
            if arm == "uniform_split":
                split = L.toa_wgrad_split(N, K, T)
                nbytes = split * N * K * 4 if split > 1 else 0
            else:
                split = 0
                nbytes = L.toa_wgrad_workspace(N, K, T, 0)
            ws = torch.empty(max(nbytes // 4, 1), device="cuda", dtype=torch.float32)
            g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)

            def call(L=L, g=g, ws=ws, split=split):
                rc = L.toa_wgrad(ptr(dy), N, ptr(x), K, ptr(g), K, ptr(ws), N, K, T, split, 0, st)
                assert rc == 0, rc

            calls[arm] = call
            call()
            outs[arm] = g
        torch.cuda.synchronize()
        diff = float((outs["uniform_split"].float() - outs["tail_split"].float()).abs().max())
        times = {a: [] for a in libs}
        for _ in range(7):
            for arm, fn in calls.items():
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(5):
                    fn()
                b.record()
                torch.cuda.synchronize()
                times[arm].append(a.elapsed_time(b) / 5)
        fl = 2.0 * N * K * T
        res[name] = {a: {"ms": round(statistics.median(v), 4), "tflops": round(fl / statistics.median(v) / 1e9, 1)}
                     for a, v in times.items()}
        res[name]["max_abs_diff"] = diff
        print(json.dumps({name: res[name]}), flush=True)
    # per training step: 32 layers of qkv/o/gate_up/down + one lm_head
    step = {a: round(sum(res[n][a]["ms"] * (1 if n == "lm_head" else 32) for n in SHAPES), 2) for a in libs}
    print(json.dumps({"wgrad_ms_per_step": step}))


if __name__ == "__main__":
    main()
