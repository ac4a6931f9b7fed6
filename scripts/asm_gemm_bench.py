"""Hand-written gfx950 assembly GEMM (csrc/asm/gemm_gen.py) vs hipBLASLt at
the Llama-3-8B forward / data-gradient forms, in-process interleaved rounds on
random operands (guide section 5.4 rules 24/25).

    python scripts/asm_gemm_bench.py --check        # numerics only (small shapes)
    python scripts/asm_gemm_bench.py [--tokens 24576] [--rounds 5] [--reps 5] [--variants 1,2,3]

Arms: asm (toa_gemm_asm), blt_nosk (hipBLASLt non-stream-K table),
blt_heur (torch.matmul), asm_v<n> (the plain kernel's A/B arms,
gemm_gen.py PLAIN_VARIANTS; checked bit-identical to asm), and the fused MLP
ends (asm SwiGLU epilogues vs hipBLASLt + the SwiGLU row kernels).
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "csrc/asm")
from tf_operator_amd.ops import _lib, gemm, llm  # noqa: E402

FORMS = {"qkv": (4096, 6144), "o": (4096, 4096), "gate_up": (4096, 28672), "down": (14336, 4096),
         "lm_head": (4096, 128256)}


def asm(x, w, y):
    M, K = x.shape
    N = w.shape[0]
    _lib.call("toa_gemm_asm", _lib.ptr(x), x.stride(0), _lib.ptr(w), w.stride(0), _lib.ptr(y), y.stride(0), M, N, K,
              _lib.stream(x))


def asm_swiglu(x, wgu):
    M, F = x.shape[0], wgu.shape[0] // 2
    gu = torch.empty(M, 2 * F, device=x.device, dtype=x.dtype)
    s = torch.empty(M, F, device=x.device, dtype=x.dtype)
    _lib.call("toa_gemm_asm_swiglu", _lib.ptr(x), x.stride(0), _lib.ptr(wgu), wgu.stride(0), _lib.ptr(gu), 2 * F,
              _lib.ptr(s), F, M, F, x.shape[1], _lib.stream(x))
    return gu, s


def asm_swiglu_bwd(d2, wdt, gu):
    M, F = d2.shape[0], wdt.shape[0]
    dgu = torch.empty_like(gu)
    _lib.call("toa_gemm_asm_swiglu_bwd", _lib.ptr(d2), d2.stride(0), _lib.ptr(wdt), wdt.stride(0), _lib.ptr(gu),
              2 * F, _lib.ptr(dgu), 2 * F, M, F, d2.shape[1], _lib.stream(d2))
    return dgu


def with_phase(kind, word, fn):
    """Run fn with the first-wave start offsets of kernel family `kind`
    (0 plain, 1 SwiGLU fwd, 2 SwiGLU bwd) set to `word` (gemm_gen.phase_delay),
    then back to 0."""
    _lib.call("toa_gemm_asm_set_phase", kind, word)
    try:
        return fn()
    finally:
        _lib.call("toa_gemm_asm_set_phase", kind, 0)


def asm_swiglu_bwd_variant(v, d2, wdt, gu, dgu):
    M, F = d2.shape[0], wdt.shape[0]
    _lib.call("toa_gemm_asm_swiglu_bwd_variant", v, _lib.ptr(d2), d2.stride(0), _lib.ptr(wdt), wdt.stride(0),
              _lib.ptr(gu), 2 * F, _lib.ptr(dgu), 2 * F, M, F, d2.shape[1], _lib.stream(d2))


def asm_variant(v, x, w, y):
    M, K = x.shape
    N = w.shape[0]
    _lib.call("toa_gemm_asm_variant", v, _lib.ptr(x), x.stride(0), _lib.ptr(w), w.stride(0), _lib.ptr(y), y.stride(0),
              M, N, K, _lib.stream(x))


def asm_map(tmap, x, w, y):
    M, K = x.shape
    N = w.shape[0]
    _lib.call("toa_gemm_asm_map", tmap, _lib.ptr(x), x.stride(0), _lib.ptr(w), w.stride(0), _lib.ptr(y), y.stride(0),
              M, N, K, _lib.stream(x))


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


def check():
    torch.manual_seed(0)
    res = {}
    for (M, N, K) in ((256, 256, 128), (512, 768, 320), (1024, 512, 4096), (768, 1280, 192)):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        y = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        asm(x, w, y)
        torch.cuda.synchronize()
        res[f"plain_{M}x{N}x{K}"] = rel(y, x.float() @ w.float().t())
    # strided rows (ld > K) and an output with ld > N
    x = torch.randn(512, 384, device="cuda").to(torch.bfloat16)[:, :256]
    w = torch.randn(256, 320, device="cuda").to(torch.bfloat16)[:, :256]
    yb = torch.zeros(512, 512, device="cuda", dtype=torch.bfloat16)
    asm(x, w, yb[:, 128:384])
    torch.cuda.synchronize()
    res["plain_strided"] = rel(yb[:, 128:384], x.float() @ w.float().t())
    res["plain_strided_untouched"] = float(yb[:, :128].abs().sum() + yb[:, 384:].abs().sum())
    M, F, K = 512, 384, 256
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    wgu = (torch.randn(2 * F, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    gu, s = asm_swiglu(x, wgu)
    torch.cuda.synchronize()
    ref = (x.float() @ wgu.float().t())
    res["swiglu_fwd_gu"] = rel(gu, ref)
    g, u = ref.bfloat16().float().split(F, 1)
    res["swiglu_fwd_s"] = rel(s, torch.nn.functional.silu(g) * u)
    M, F, K = 512, 512, 384
    d2 = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    wdt = (torch.randn(F, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    gu = torch.randn(M, 2 * F, device="cuda").to(torch.bfloat16)
    dgu = asm_swiglu_bwd(d2, wdt, gu)
    torch.cuda.synchronize()
    ds = (d2.float() @ wdt.float().t()).bfloat16().float()
    g, u = gu.float().split(F, 1)
    sg = torch.sigmoid(g)
    res["swiglu_bwd_dg"] = rel(dgu[:, :F], ds * u * sg * (1 + g * (1 - sg)))
    res["swiglu_bwd_du"] = rel(dgu[:, F:], ds * g * sg)
    print(json.dumps({"check": res}), flush=True)
    bad = {k: v for k, v in res.items() if not (v < 1e-2) and k != "plain_strided_untouched"}
    if bad or res["plain_strided_untouched"] != 0:
        raise SystemExit(f"asm GEMM numerics FAILED: {bad} untouched={res['plain_strided_untouched']}")


def probe():
    """Run the diagnostic kernel (plain prologue + register dump) and compare
    its dump with the CPU emulator's run of the same instructions on the same
    argument block.  Prints every differing SGPR / per-thread word."""
    import os
    import numpy as np
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "asm"))
    import emu
    import gemm_gen
    import host_args

    res = {}
    text = gemm_gen.generate()
    # SGPRs that legitimately differ: kernarg pointer, per-wave values (the
    # last wave to store wins), never-written scratch
    skip = {0, 1, 27, 31, 48, 49, 50, 51, 52, 67, 68, 69, 70, 71, 72}
    for (M, N, K) in ((256, 256, 128), (512, 768, 320), (768, 1280, 192), (1024, 512, 4096), (2048, 2048, 512)):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        y = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        nwg = (M // 256) * (N // 256)
        out = torch.zeros(nwg * gemm_gen.PROBE_WORDS, device="cuda", dtype=torch.int32)
        _lib.call("toa_gemm_asm_probe", _lib.ptr(out), _lib.ptr(x), K, _lib.ptr(w), K, _lib.ptr(y), N, M, N, K,
                  _lib.stream(x))
        torch.cuda.synchronize()
        hw = out.cpu().numpy().view(np.uint32).reshape(nwg, -1)
        karg = bytearray(host_args.pack(x.data_ptr(), w.data_ptr(), y.data_ptr(), out.data_ptr(), 2 * K, 2 * K,
                                        2 * N, 0, K, M // 256, N // 256, gemm_gen.PROBE_MAGIC[0],
                                        gemm_gen.PROBE_MAGIC[1]))
        mem = emu.Memory()
        ref = np.zeros(nwg * gemm_gen.PROBE_WORDS, np.uint32)
        mem.add_at(out.data_ptr(), ref)
        e = emu.Emu(text, "toa_gemm_tn_asm_probe")
        for b in range(nwg):
            e.run(bytes(karg), b, mem)
        ref = ref.reshape(nwg, -1)
        diff = [(b, int(i), hex(int(hw[b, i])), hex(int(ref[b, i]))) for b in range(nwg)
                for i in np.nonzero(hw[b] != ref[b])[0] if int(i) not in skip]
        res[f"{M}x{N}x{K}"] = {"nwg": nwg, "n_diff": len(diff), "first": diff[:40]}
    print(json.dumps({"probe": res}), flush=True)


def trace(shapes):
    """Run the trace kernel per shape; print every wave's last marker (also
    after a device fault: the records live in host-coherent memory)."""
    import ctypes
    import numpy as np
    lib = _lib.lib()
    for sh in shapes.split(","):
        M, N, K = (int(v) for v in sh.split("x"))
        nwg = (M // 256) * (N // 256)
        nbytes = nwg * 4 * 32
        host = lib.toa_host_coherent_alloc(nbytes)
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        y = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        err = None
        try:
            _lib.call("toa_gemm_asm_trace", ctypes.c_void_p(host), _lib.ptr(x), K, _lib.ptr(w), K, _lib.ptr(y), N,
                      M, N, K, _lib.stream(x))
            torch.cuda.synchronize()
        except Exception as e:  # a device fault: the trace is still readable
            err = repr(e)[:300]
        rec = np.frombuffer(ctypes.string_at(host, nbytes), dtype=np.uint32).reshape(nwg * 4, 8)
        codes = {}
        for r in rec:
            codes[int(r[0])] = codes.get(int(r[0]), 0) + 1
        out = {"shape": sh, "error": err, "last_code_counts": codes,
               "records_first": rec[:8].tolist(), "records_min_code": rec[rec[:, 0].argmin()].tolist()}
        if err is None:
            out["rel"] = rel(y, x.float() @ w.float().t())
        print(json.dumps(out), flush=True)
        if err is not None:
            raise SystemExit(1)


def timing(a):
    """Where the product kernel's cycles go (the timing kernel, gemm_gen.py
    SCHED["timing"]): per form, the mean over (workgroup, wave) of the cycles
    parked in the next-tile vmcnt wait + barrier, the X-free and W-free
    barriers, the epilogue, as shares of start -> end."""
    import numpy as np

    T = a.tokens
    res = {}
    for name, (K, N) in FORMS.items():
        for kind, (kk, nn) in (("fwd", (K, N)), ("dgrad_wt", (N, K))):
            if a.forms and f"{name}.{kind}" not in a.forms.split(","):
                continue
            x = torch.randn(T, kk, device="cuda").to(torch.bfloat16)
            w = (torch.randn(nn, kk, device="cuda") / kk ** 0.5).to(torch.bfloat16)
            y = torch.empty(T, nn, device="cuda", dtype=torch.bfloat16)
            nwg = (T // 256) * (nn // 256)
            rec = torch.zeros(nwg * 32, device="cuda", dtype=torch.int32)
            for _ in range(3):  # warm (clocks, caches); the last run's records are read
                _lib.call("toa_gemm_asm_timing", 2, _lib.ptr(rec), _lib.ptr(x), kk, _lib.ptr(w), kk, _lib.ptr(y), nn,
                          T, nn, kk, _lib.stream(x))
            torch.cuda.synchronize()
            r2 = rec.cpu().numpy().view(np.uint32).reshape(nwg, 4, 8).astype(np.float64)
            loops = np.maximum(r2[:, :, 5] - 2, 1)  # main-loop iterations (the two tail tiles carry no DMA)
            import gemm_gen  # csrc/asm: the product slot map's stretch lengths
            nm = gemm_gen.span_mfmas(gemm_gen.SLOT_MAPS[gemm_gen.SCHED["map"]])
            spans = dict(zip(("xdma_cyc_per_mfma", "wdma_pre_wait_cyc_per_mfma", "wdma_post_wait_cyc_per_mfma"), nm))
            sp = {k: round(float((r2[:, :, i] / loops).mean() / n), 2) for i, (k, n) in enumerate(spans.items())}
            for _ in range(3):
                _lib.call("toa_gemm_asm_timing", 1, _lib.ptr(rec), _lib.ptr(x), kk, _lib.ptr(w), kk, _lib.ptr(y), nn,
                          T, nn, kk, _lib.stream(x))
            torch.cuda.synchronize()
            r = rec.cpu().numpy().view(np.uint32).reshape(nwg, 4, 8).astype(np.float64)
            tot = r[:, :, 3] + r[:, :, 4]
            res[f"{name}.{kind}"] = {**sp,
                "cycles_per_tile": round(float(tot.mean()), 0),
                "loop_cycles_per_ktile": round(float((r[:, :, 3] / r[:, :, 5]).mean()), 1),
                "vm_wait_pct": round(float(100 * (r[:, :, 0] / tot).mean()), 2),
                "xbar_pct": round(float(100 * (r[:, :, 1] / tot).mean()), 2),
                "wbar_pct": round(float(100 * (r[:, :, 2] / tot).mean()), 2),
                "epilogue_pct": round(float(100 * (r[:, :, 4] / tot).mean()), 2),
                "tile_cycles_p10_p90": [float(np.percentile(tot, 10)), float(np.percentile(tot, 90))]}
            print(json.dumps({f"{name}.{kind}": res[f"{name}.{kind}"]}), flush=True)
            del x, w, y
            torch.cuda.empty_cache()
    print(json.dumps({"timing": res}))


WGRAD_FORMS = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
               "lm_head": (128256, 4096)}


def wgrad(a):
    """Weight gradient g[N][K] = dy^T x at T tokens: the assembly NT kernel
    (toa_wgrad_asm), the HIP kernel (toa_wgrad), hipBLASLt (torch.mm);
    auto plans, interleaved rounds; asm checked against the HIP kernel."""
    T = a.tokens
    torch.manual_seed(0)
    res = {}
    for name, (N, K) in WGRAD_FORMS.items():
        if a.forms and f"{name}.wgrad" not in a.forms.split(","):
            continue
        dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        g = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        g2 = torch.empty_like(g)
        nbytes = int(_lib.call_ret("toa_wgrad_workspace", N, K, T, 0))
        ws = torch.empty(max(nbytes, 16) // 4, device="cuda", dtype=torch.float32)

        def hip():
            _lib.call("toa_wgrad", _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(g2), K, _lib.ptr(ws), N, K, T, 0, 0,
                      _lib.stream(dy))

        def asm_():
            _lib.call("toa_wgrad_asm", _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(g), K, _lib.ptr(ws), N, K, T, 0, 0,
                      _lib.stream(dy))

        g3 = torch.empty_like(g)

        def asm_v1():  # the round-4 schedule of the same kernel
            _lib.call("toa_wgrad_asm_variant", 1, _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(g3), K, _lib.ptr(ws), N,
                      K, T, 0, 0, _lib.stream(dy))

        arms = [("asm", asm_), ("asm_v1", asm_v1), ("hip", hip), ("blt", lambda: torch.mm(dy.t(), x))]
        g4 = torch.empty_like(g)

        def mapped(tm_):   # the product kernel with another tile order (toa_wgrad_asm_set_map)
            _lib.call("toa_wgrad_asm_set_map", tm_)
            try:
                _lib.call("toa_wgrad_asm", _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(g4), K, _lib.ptr(ws), N, K, T,
                          0, 0, _lib.stream(dy))
            finally:
                _lib.call("toa_wgrad_asm_set_map", -1)

        wmaps = [int(v) for v in a.wgrad_maps.split(",") if v]
        for tm_ in wmaps:
            arms.append((f"asm_map{tm_}", lambda tm_=tm_: mapped(tm_)))
        for sp in (int(v) for v in a.wgrad_splits.split(",") if v):
            # every tile cut into `sp` K-pieces (1: none) instead of the auto plan
            if sp * (N // 256) * (K // 256) >= (1 << 14) or T % (64 * sp):
                continue
            need = int(_lib.call_ret("toa_wgrad_workspace", N, K, T, sp))
            wsp = torch.empty(max(need, 16) // 4, device="cuda", dtype=torch.float32)

            def forced(sp=sp, wsp=wsp):
                _lib.call("toa_wgrad_asm", _lib.ptr(dy), N, _lib.ptr(x), K, _lib.ptr(g2), K, _lib.ptr(wsp), N, K, T,
                          sp, 0, _lib.stream(dy))

            arms.append((f"asm_split{sp}", forced))
        ts = {k: [] for k, _ in arms}
        for _ in range(a.rounds):
            for k, f in arms:
                ts[k].append(timer(f, a.reps))
        asm_()
        hip()
        torch.cuda.synchronize()
        fl = 2.0 * T * N * K
        rec = {k: {"ms": round(statistics.median(v), 4), "TFps": round(fl / statistics.median(v) / 1e9, 1)}
               for k, v in ts.items()}
        rec["asm_vs_hip_rel"] = round(rel(g, g2), 6)
        asm_v1()
        torch.cuda.synchronize()
        rec["asm_v1_bit_identical"] = bool(torch.equal(g, g3))
        for tm_ in wmaps:
            mapped(tm_)
            torch.cuda.synchronize()
            rec[f"asm_map{tm_}_bit_identical"] = bool(torch.equal(g, g4))
        res[f"{name}.wgrad"] = rec
        print(json.dumps({f"{name}.wgrad": rec}), flush=True)
        del dy, x, g, g2, ws
        torch.cuda.empty_cache()
    print(json.dumps({"wgrad": res}))


def timer(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def bench(a):
    T = a.tokens
    torch.manual_seed(0)
    out = {"tokens": T, "forms": {}}
    variants = [int(v) for v in a.variants.split(",") if v]
    maps = [int(v) for v in a.maps.split(",") if v]
    phases = [int(v, 0) for v in a.phases.split(",") if v]
    for name, (K, N) in FORMS.items():
        for kind, (kk, nn) in (("fwd", (K, N)), ("dgrad_wt", (N, K))):
            if a.forms and f"{name}.{kind}" not in a.forms.split(","):
                continue
            x = torch.randn(T, kk, device="cuda").to(torch.bfloat16)
            w = (torch.randn(nn, kk, device="cuda") / kk ** 0.5).to(torch.bfloat16)
            y = torch.empty(T, nn, device="cuda", dtype=torch.bfloat16)
            arms = [("asm", lambda: asm(x, w, y)),
                    ("blt_nosk", lambda: (gemm.set_mode("nosk"), gemm.linear_fwd(x, w))),
                    ("blt_heur", lambda: torch.matmul(x, w.t()))]
            yv = torch.empty_like(y)
            for v in variants:
                arms.append((f"asm_v{v}", lambda v=v: asm_variant(v, x, w, yv)))
            for tm_ in maps:
                arms.append((f"asm_map{tm_}", lambda tm_=tm_: asm_map(tm_, x, w, yv)))
            for ph in phases:
                arms.append((f"asm_ph{ph:#x}", lambda ph=ph: with_phase(0, ph, lambda: asm(x, w, yv))))
            ts = {k: [] for k, _ in arms}
            for _ in range(a.rounds):
                for k, f in arms:
                    ts[k].append(timer(f, a.reps))
            asm(x, w, y)
            same = {}
            for v in variants:
                asm_variant(v, x, w, yv)
                same[f"asm_v{v}"] = bool(torch.equal(y, yv))
            for tm_ in maps:
                asm_map(tm_, x, w, yv)
                same[f"asm_map{tm_}"] = bool(torch.equal(y, yv))
            for ph in phases:
                with_phase(0, ph, lambda: asm(x, w, yv))
                same[f"asm_ph{ph:#x}"] = bool(torch.equal(y, yv))
            err = rel(y, x.float() @ w.float().t()) if T * nn <= 24576 * 28672 else -1.0
            fl = 2.0 * T * nn * kk
            rec = {k: {"ms": round(statistics.median(v), 4), "TFps": round(fl / statistics.median(v) / 1e9, 1)}
                   for k, v in ts.items()}
            rec["asm_rel_err"] = round(err, 5)
            if same:
                rec["variants_bit_identical"] = same
            out["forms"][f"{name}.{kind}"] = rec
            print(json.dumps({f"{name}.{kind}": rec}), flush=True)
            del x, w, y
            torch.cuda.empty_cache()
    if a.mlp:
        F_, Hd = 14336, 4096
        x = torch.randn(T, Hd, device="cuda").to(torch.bfloat16)
        wgu = (torch.randn(2 * F_, Hd, device="cuda") / Hd ** 0.5).to(torch.bfloat16)
        wdt = (torch.randn(F_, Hd, device="cuda") / Hd ** 0.5).to(torch.bfloat16)
        d2 = torch.randn(T, Hd, device="cuda").to(torch.bfloat16)
        gu, _ = asm_swiglu(x, wgu)
        arms = [("asm_fused_fwd", lambda: asm_swiglu(x, wgu)),
                ("blt_unfused_fwd", lambda: (gemm.set_mode("nosk"), llm.swiglu(gemm.linear_fwd(x, wgu)))),
                ("asm_fused_bwd", lambda: asm_swiglu_bwd(d2, wdt, gu)),
                ("blt_unfused_bwd", lambda: (gemm.set_mode("nosk"), llm.swiglu_bwd(gemm.linear_fwd(d2, wdt), gu)))]
        dgu_v = torch.empty_like(gu)

        def mapped(tm_, fn):
            _lib.call("toa_gemm_asm_set_map", tm_)
            try:
                return fn()
            finally:
                _lib.call("toa_gemm_asm_set_map", -1)

        for tm_ in maps:
            arms += [(f"asm_fused_fwd_map{tm_}", lambda tm_=tm_: mapped(tm_, lambda: asm_swiglu(x, wgu))),
                     (f"asm_fused_bwd_map{tm_}", lambda tm_=tm_: mapped(tm_, lambda: asm_swiglu_bwd(d2, wdt, gu)))]
        for v in [int(t) for t in a.swiglu_variants.split(",") if t]:
            arms.append((f"asm_fused_bwd_b{v}", lambda v=v: asm_swiglu_bwd_variant(v, d2, wdt, gu, dgu_v)))
        def persistent(bit, fn):
            _lib.call("toa_gemm_asm_set_swiglu_persist", bit)
            try:
                return fn()
            finally:
                _lib.call("toa_gemm_asm_set_swiglu_persist", 0)

        if a.swiglu_persist:
            arms += [("asm_fused_fwd_p1", lambda: persistent(1, lambda: asm_swiglu(x, wgu))),
                     ("asm_fused_bwd_p1", lambda: persistent(2, lambda: asm_swiglu_bwd(d2, wdt, gu)))]
        for ph in phases:
            arms += [(f"asm_fused_fwd_ph{ph:#x}", lambda ph=ph: with_phase(1, ph, lambda: asm_swiglu(x, wgu))),
                     (f"asm_fused_bwd_ph{ph:#x}", lambda ph=ph: with_phase(2, ph, lambda: asm_swiglu_bwd(d2, wdt, gu)))]
        ts = {k: [] for k, _ in arms}
        for _ in range(a.rounds):
            for k, f in arms:
                ts[k].append(timer(f, a.reps))
        out["mlp_ms"] = {k: round(statistics.median(v), 4) for k, v in ts.items()}
        if phases:   # the start offsets change when a tile runs, never what it computes
            ref_f, ref_b = asm_swiglu(x, wgu), asm_swiglu_bwd(d2, wdt, gu)
            out["mlp_phase_bit_identical"] = {
                f"{ph:#x}": bool(all(torch.equal(p_, q_) for p_, q_ in zip(
                    with_phase(1, ph, lambda: asm_swiglu(x, wgu)), ref_f))
                    and torch.equal(with_phase(2, ph, lambda: asm_swiglu_bwd(d2, wdt, gu)), ref_b))
                for ph in phases}
        if a.swiglu_persist:   # the persistent arms compute what the product kernels compute
            ref_f, ref_b = asm_swiglu(x, wgu), asm_swiglu_bwd(d2, wdt, gu)
            pf, pb = persistent(1, lambda: asm_swiglu(x, wgu)), persistent(2, lambda: asm_swiglu_bwd(d2, wdt, gu))
            out["mlp_persist_bit_identical"] = bool(all(torch.equal(p_, q_) for p_, q_ in zip(pf, ref_f))
                                                    and torch.equal(pb, ref_b))
        print(json.dumps({"mlp_ms": out["mlp_ms"], **({"persist_same": out["mlp_persist_bit_identical"]}
                                                      if a.swiglu_persist else {})}), flush=True)
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--trace", default="", help="diagnostic: MxNxK shapes for the trace kernel, comma-separated")
    ap.add_argument("--stage", type=int, default=-1, help="diagnostic: run the plain kernel to this stage only")
    ap.add_argument("--tokens", type=int, default=24576)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--forms", default="")
    ap.add_argument("--mlp", type=int, default=1)
    ap.add_argument("--variants", default="", help="plain-kernel A/B arms to add, e.g. 1,2,3")
    ap.add_argument("--maps", default="", help="tile orders to add as arms (kernarg map words, e.g. 2,3,18,20)")
    ap.add_argument("--swiglu-variants", default="", help="fused SwiGLU backward diagnostic arms (1..5) "
                                                          "added to the MLP arms (gemm_gen.SWIGLU_BWD_VARIANTS)")
    ap.add_argument("--swiglu-persist", action="store_true", help="add the persistent fused SwiGLU arms (p1)")
    ap.add_argument("--phases", default="", help="first-wave start-offset words to add as arms (n | log2 g << 16, "
                                                 "e.g. 0x10028,0x20014): plain forms and the fused MLP")
    ap.add_argument("--timing", action="store_true", help="wait-cycle breakdown of the product kernel (--forms)")
    ap.add_argument("--wgrad", action="store_true", help="weight-gradient forms: asm NT vs HIP vs hipBLASLt")
    ap.add_argument("--wgrad-maps", default="", help="weight-gradient tile orders as extra arms (map words: "
                                                     "log2 group | 16 for column groups; the per-shape default "
                                                     "is gemm_asm.hip wgrad_tile_map)")
    ap.add_argument("--wgrad-splits", default="", help="extra asm arms with every tile cut into S K-pieces, e.g. 1,2,3")
    a = ap.parse_args()
    if a.probe:
        probe()
        return
    if a.trace:
        trace(a.trace)
        return
    if a.timing:
        timing(a)
        return
    if a.wgrad:
        wgrad(a)
        return
    if a.stage >= 0:
        M, N, K = 256, 256, 128
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        y = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        _lib.call("toa_gemm_asm_stage", a.stage, _lib.ptr(x), K, _lib.ptr(w), K, _lib.ptr(y), N, M, N, K,
                  _lib.stream(x))
        torch.cuda.synchronize()
        print(json.dumps({"stage": a.stage, "ok": True,
                          "rel": rel(y, x.float() @ w.float().t()) if a.stage == 0 else None}), flush=True)
        return
    check()
    if not a.check:
        bench(a)


if __name__ == "__main__":
    main()
