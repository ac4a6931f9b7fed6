"""In-model A/B of a kernel choice on the Llama-3-8B bench step, in ONE
process (one model, one set of buffers): alternating timed windows of
`--steps` steps under each arm after a shared warm-up, median ms/step per arm.

    python scripts/wgrad_inmodel_ab.py [--rounds 3] [--steps 4] [--arms wgrad=asm+gemm=nosk,wgrad=hip+gemm=nosk]

An arm is settings joined by '+': wgrad=asm|hip|asm_v1 (ops.gemm.set_wgrad_kernel),
gemm=asm|nosk (ops.gemm.set_mode: forward / data-gradient policy), attnf=N /
attnb=N / attnd=N (toa_attn_set_fwd_variant / _bwd_variant / _dkdv_variant forms),
epi=r4|pipe (the fused SwiGLU GEMMs' epilogues, toa_gemm_asm_set_epi_variant),
wmap=N (the weight-gradient tile order, toa_wgrad_asm_set_map; -1 = the per-shape rule),
persist=N (the plain TN kernel's persistent form, toa_gemm_asm_set_persist; -1 = the per-shape rule),
swp=N (the fused SwiGLU GEMMs' persistent forms, toa_gemm_asm_set_swiglu_persist: bit 0 fwd, bit 1 bwd),
ovl=0|1 (AdamW per bucket on a side stream under the next forward, FlatAdamW overlap),
ovlcu=n[:mode] (that side stream limited to n CUs, toa_stream_create_cu_mask; 0 = unmasked),
xent=N (cross-entropy backward chunks per thread), tpose=0|1 (the W^T refresh's transpose kernel),
fnorm=0|1 (the clipping norm from the weight-gradient kernels' partials, or the full pass),
adamwt=0|1 (AdamW writes the W^T copies itself, or the refresh transposes after it),
qkvrope=0|1 (the QKV projection's GEMM applies RoPE and the head-major relayout, or the RoPE pass does),
dfused=0|1 (the attention delta rows from the output projection's GEMM, or the attention's own pass),
resadd=0|1 (the residual add in the output projection's epilogue, or in the RMSNorm),
adamcap=N (the flat AdamW grid cap / 1024, toa_set_stream_variant),
or the presets r4 (every round-4 default kernel: nosk GEMMs, the round-4
weight-gradient schedule, the HIP attention forward and dK/dV) and head
(this tree's defaults).  Same-process windows remove the box-to-box spread
(about +-2.5 %) from the comparison:

    python scripts/wgrad_inmodel_ab.py --arms r4,head --rounds 8
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from tf_operator_amd.ops import _lib, gemm  # noqa: E402
from tf_operator_amd.train.llm import LlamaTrainer  # noqa: E402


TR = None   # the trainer (arms that switch trainer state: ovl)


def apply(arm: str):
    """arm: settings joined by '+', e.g. wgrad=hip+gemm=nosk."""
    presets = {"r4": "gemm=nosk+wgrad=asm_v1+attnf=1+attnd=0+epi=r4",
               "head": "gemm=asm+wgrad=asm+attnf=-1+attnd=-1+epi=pipe"}
    arm = presets.get(arm, arm)
    for part in arm.split("+"):
        key, val = part.split("=")
        if key == "wgrad":
            gemm.set_wgrad_kernel(val)
        elif key == "gemm":
            gemm.set_mode(val)
        elif key == "attnf":
            _lib.call("toa_attn_set_fwd_variant", int(val))
        elif key == "attnb":
            _lib.call("toa_attn_set_bwd_variant", int(val))
        elif key == "attnd":
            _lib.call("toa_attn_set_dkdv_variant", int(val))
        elif key == "epi":   # the fused SwiGLU GEMMs' epilogues: r4 (drained per row block) or pipe
            _lib.call("toa_gemm_asm_set_epi_variant", 1 if val == "r4" else 0)
        elif key == "dkpk":   # the assembly dK/dV with round 5's packed P / dS VALU (1) or the scalar product (0)
            _lib.call("toa_attn_dkdv_asm_set_arm", int(val))
        elif key == "persist":   # TN plain kernel: -1 = the per-shape rule, 0 = never persistent, 1 = always
            _lib.call("toa_gemm_asm_set_persist", int(val))
        elif key == "swp":   # fused SwiGLU GEMMs persistent: bit 0 forward, bit 1 backward
            _lib.call("toa_gemm_asm_set_swiglu_persist", int(val))
        elif key == "ovl":   # AdamW per bucket on a side stream under the next forward (FlatAdamW overlap)
            TR.opt.wait_all()
            TR.opt.overlap = bool(int(val))
        elif key == "ovlcu":   # the overlapped update's stream: n CUs (mode 1: spread; n:mode), 0 = unmasked
            from tf_operator_amd.ops.optim import masked_stream
            TR.opt.wait_all()
            torch.cuda.synchronize()
            n, _, mode = val.partition(":")
            TR.opt.side = (masked_stream(int(n), int(mode or 1), TR.device) if int(n)
                           else torch.cuda.Stream(device=TR.device))
        elif key == "xent":   # cross-entropy backward chunks per thread (1, 2, 4)
            _lib.call("toa_xent_set_unroll", int(val))
        elif key == "tpose":   # W^T refresh: 1 LDS-staged 128 x 128 tiles, 0 the register kernel
            _lib.call("toa_transpose_set_variant", int(val))
        elif key == "fnorm":   # clipping norm from the weight-gradient partials (1) or the full pass (0)
            sess = getattr(TR, "_sumsq", None)
            if sess is None:
                raise SystemExit("fnorm: the trainer has no SumsqSession (TOA_FUSED_NORM=0?)")
            if int(val):
                gemm._SESSIONS.add(sess)
                TR.opt.sumsq = sess
            else:
                gemm._SESSIONS.discard(sess)
                TR.opt.sumsq = None
        elif key == "adamwt":   # the update writes the W^T copies itself (1) or they are refreshed after it (0)
            if not hasattr(TR, "_fused_wt_saved"):
                TR._fused_wt_saved = TR.opt.fused_wt
            TR.opt.fused_wt = TR._fused_wt_saved if int(val) else None
        elif key == "qkvrope":   # the QKV GEMM writes rotated head-major q | k | v (1) or qkv + the RoPE pass (0)
            import os
            os.environ["TOA_QKV_ROPE"] = val
        elif key == "dfused":   # attention delta rows from the output projection's GEMM (1) or its own pass (0)
            import os
            os.environ["TOA_ATTN_DELTA_FUSED"] = val
        elif key == "resadd":   # the residual add in the output projection's epilogue (1) or in the RMSNorm (0)
            import os
            os.environ["TOA_RESADD_FUSED"] = val
        elif key == "wmap":   # weight-gradient tile order: -1 = the per-shape rule, else a map word
            _lib.call("toa_wgrad_asm_set_map", int(val))
        elif key == "adamcap":
            _lib.call_ret("toa_set_stream_variant", 1 | 2 | (int(val) << 8))
        else:
            raise SystemExit(f"unknown arm {arm}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--arms", default="wgrad=asm+gemm=nosk,wgrad=hip+gemm=nosk,wgrad=asm+gemm=asm")
    ap.add_argument("--micro-batch", type=int, default=6)
    ap.add_argument("--abba", type=int, default=1, help="reverse the arm order every other round")
    a = ap.parse_args()
    arms = a.arms.split(",")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    global TR
    tr = TR = LlamaTrainer("llama3-8b", dev, micro_batch=a.micro_batch, seq_len=4096,
                           overlap_optimizer=True if "ovl=" in a.arms else None)
    batch = [tr.synthetic_batch()]
    for arm in arms:  # every arm warm (code objects, plans)
        apply(arm)
        for _ in range(a.warmup):
            tr.step(batch)
    torch.cuda.synchronize()
    times = {arm: [] for arm in arms}
    for r in range(a.rounds):
        # ABBA: every other round runs the arms in reverse, so a linear drift
        # (the chip warming over the run) does not favour the first arm
        order = arms if (r % 2 == 0 or not a.abba) else arms[::-1]
        for arm in order:
            apply(arm)
            tr.step(batch)  # one untimed step after the switch
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                loss = tr.step(batch)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.steps
            times[arm].append(ms)
            print(json.dumps({"round": r, "arm": arm, "ms_per_step": round(ms, 2), "loss": float(loss)}), flush=True)
    out = {"median_ms_per_step": {k: round(statistics.median(v), 2) for k, v in times.items()}, "all": times}
    if len(arms) >= 2 and a.rounds >= 2:
        # paired per-round differences against the first arm: mean and its standard error
        base = times[arms[0]]
        for arm in arms[1:]:
            d = [x - y for x, y in zip(times[arm], base)]
            se = statistics.stdev(d) / len(d) ** 0.5
            out.setdefault("paired_vs_" + arms[0], {})[arm] = {
                "mean_ms": round(statistics.fmean(d), 2), "stderr_ms": round(se, 2),
                "pct": round(100 * statistics.fmean(d) / statistics.fmean(base), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
