"""Do high-priority side-stream kernels (what RCCL's collectives are) get
CUs while hipBLASLt's persistent stream-K GEMMs run?  A chain of Llama-3-8B
shaped GEMMs on the main stream; 20 small copies on a high-priority stream,
queued after the GEMMs are.  The kernel trace (rocprofv3 --kernel-trace)
shows where the copies ran; this script also prints the host-timed end of
the copies relative to the GEMM chain.

    rocprofv3 --kernel-trace --output-format csv -d out -- python3 scripts/probes/sk_starvation.py
    TENSILE_STREAMK_MAX_CUS=224 python3 scripts/probes/sk_starvation.py
    python3 scripts/probes/sk_starvation.py --reserve 8 [--spread]

``--reserve K`` runs the GEMMs on a stream whose CU mask leaves K CUs out
(hipExtStreamCreateWithCUMask) and the copies on a stream masked to
exactly those K CUs: the split a training step would use to keep RCCL's
kernels off the GEMMs' CUs.  ``--spread`` leaves out K CUs spread over the
mask (every 256/K-th bit) instead of the top K bits.
"""
import argparse
import ctypes
import json
import os

import torch


def masked_stream(bits):
    """A torch ExternalStream over a HIP stream restricted to CU bits `bits`."""
    hip = ctypes.CDLL("libamdhip64.so")
    words = [0] * 8
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    arr = (ctypes.c_uint32 * 8)(*words)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(8), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(h.value)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reserve", type=int, default=0)
    ap.add_argument("--spread", action="store_true")
    args = ap.parse_args()
    dev = "cuda"
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    if args.reserve:
        step = ncu // args.reserve
        res = set(range(0, ncu, step)[:args.reserve]) if args.spread else set(range(ncu - args.reserve, ncu))
        compute = masked_stream(sorted(set(range(ncu)) - res))
        side = masked_stream(sorted(res))
        torch.cuda.set_stream(compute)
    T, K, N = 24576, 4096, 4096
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    src = torch.randn(32 << 20, device=dev, dtype=torch.bfloat16)  # 64 MB
    dst = torch.empty_like(src)
    if not args.reserve:
        side = torch.cuda.Stream(priority=-1)
    for _ in range(3):  # warm-up: handles, heuristics, code objects
        torch.matmul(x, w.t())
        dst.copy_(src)
    torch.cuda.synchronize()

    def run(n_gemm=40, n_copy=20):
        main = torch.cuda.current_stream()
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c1 = torch.cuda.Event(enable_timing=True)
        g0.record(main)
        for _ in range(n_gemm):
            torch.matmul(x, w.t())
        g1.record(main)
        side.wait_event(g0)
        with torch.cuda.stream(side):
            for _ in range(n_copy):
                dst.copy_(src)
            c1.record(side)
        torch.cuda.synchronize()
        return g0.elapsed_time(g1), g0.elapsed_time(c1)

    alone_copy = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(side):
        alone_copy[0].record()
        for _ in range(20):
            dst.copy_(src)
        alone_copy[1].record()
    torch.cuda.synchronize()
    copies_alone = alone_copy[0].elapsed_time(alone_copy[1])
    gemm_only = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(40):
            torch.matmul(x, w.t())
        b.record()
        torch.cuda.synchronize()
        gemm_only.append(a.elapsed_time(b))
    res = [run() for _ in range(3)]
    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("TENSILE_")},
                      "reserve": args.reserve, "spread": args.spread,
                      "gemm_chain_alone_ms": round(min(gemm_only), 3), "copies_alone_ms": round(copies_alone, 3),
                      "with_side_copies": [{"gemm_chain_ms": round(g, 3), "copies_done_at_ms": round(c, 3)}
                                           for g, c in res]}))


if __name__ == "__main__":
    main()
