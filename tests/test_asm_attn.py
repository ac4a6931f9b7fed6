"""CPU tests of the hand-written gfx950 attention forward
(csrc/asm/attn_gen.py): every workgroup of small problems run instruction by
instruction in csrc/asm/emu.py, compared with an fp64 causal attention of
the same bf16 inputs.  Covers both block orders (generic and XCD-grouped),
GQA, both O layouts, the unmasked / masked / tail loop bodies, and the
out-of-line rescale (scores that grow by > 2^8 per tile)."""
from __future__ import annotations

import math
import os
import struct
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "csrc", "asm"))
import attn_gen  # noqa: E402
import emu  # noqa: E402

TEXT = attn_gen.generate()
LOG2E = 1.4426950408889634


def bf16(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 bits (uint16), round to nearest even."""
    return emu.bf16_rne(np.asarray(x, np.float32)).astype(np.uint16)


def unbf16(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(np.float32)


def reference(q, k, v, scale):
    """fp64 causal attention; q [B,H,S,D], k / v [B,Hk,S,D] -> O [B,H,S,D], LSE [B,H,S]."""
    B, H, S, D = q.shape
    rep = H // k.shape[1]
    k = np.repeat(k, rep, axis=1).astype(np.float64)
    v = np.repeat(v, rep, axis=1).astype(np.float64)
    s = np.einsum("bhqd,bhkd->bhqk", q.astype(np.float64), k) * scale
    s = np.where(np.tril(np.ones((S, S), bool)), s, -np.inf)
    m = s.max(-1, keepdims=True)
    p = np.exp(s - m)
    l = p.sum(-1, keepdims=True)
    return np.einsum("bhqk,bhkd->bhqd", p / l, v), (m + np.log(l))[..., 0]


def run(q, k, v, scale, bshd, g8=None, hits=None):
    B, H, S, D = q.shape
    Hk = k.shape[1]
    assert D == 128 and S % 256 == 0
    nqb = S // 256
    if g8 is None:
        g8 = (B * Hk) % 8 == 0
    mem = emu.Memory()
    qa, ka, va = (mem.add(bf16(x)) for x in (q, k, v))
    o = np.zeros((B, S, H, D) if bshd else (B, H, S, D), np.uint16)
    lse = np.zeros((B, H, S), np.float32)
    oa, la = mem.add(o), mem.add(lse)
    c = float(np.float32(scale * LOG2E))
    karg = struct.pack("<5Q4If5IQ", qa, ka, va, oa, la, B, H, Hk, S, c, 3 if bshd else 1, nqb, H // Hk, int(g8), 0, 0)
    assert len(karg) == attn_gen.KARG_BYTES
    e = emu.Emu(TEXT, attn_gen.NAME)
    if hits is not None:      # count entries into the out-of-line rescale blocks
        resc = {pc for name, pc in e.labels.items() if "resc" in name}
        step = e.step

        def counting_step(w):
            if w.pc in resc:
                hits[0] += 1
            return step(w)
        e.step = counting_step
    for wg in range(nqb * H * B):
        e.run(karg, wg, mem)
    # the emulator wrote into the buffers' own bytes
    o_out = next(b for base, b in mem.bufs if base == oa).view(np.uint16).reshape(o.shape)
    l_out = next(b for base, b in mem.bufs if base == la).view(np.float32).reshape(lse.shape)
    o_f = unbf16(o_out)
    if bshd:
        o_f = o_f.transpose(0, 2, 1, 3)
    return o_f, l_out


def check(q, k, v, bshd=False, g8=None, atol=2e-2, hits=None):
    D = q.shape[-1]
    scale = 1.0 / math.sqrt(D)
    qb, kb, vb = (unbf16(bf16(x)) for x in (q, k, v))
    o, lse = run(q, k, v, scale, bshd, g8, hits)
    o_ref, lse_ref = reference(qb, kb, vb, scale)
    err = np.abs(o - o_ref).max()
    assert err < atol, f"O max err {err}"
    lerr = np.abs(lse - lse_ref).max()
    assert lerr < 2e-3 * max(1.0, np.abs(lse_ref).max()), f"LSE max err {lerr}"
    return err


def rnd(shape, seed, s=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * s).astype(np.float32)


def test_kernel_assembles_to_the_expected_size():
    lines = [ln for ln in TEXT.splitlines() if ln.startswith("  v_mfma")]
    # prologue QK (32) + 4 QK bodies x 72 + 2 tails x 40
    assert len(lines) == 32 + 4 * 72 + 2 * 40


def test_attn_fwd_generic_order_masked_only():
    """S = 512: query blocks 0 and 1 (T = 4, 8): masked + unmasked + tail
    bodies of both parities, generic block order, [B, H, S, D] output."""
    B, H, Hk, S = 1, 2, 1, 512
    check(rnd((B, H, S, 128), 1), rnd((B, Hk, S, 128), 2), rnd((B, Hk, S, 128), 3))


def test_attn_fwd_xcd_order_gqa_bshd():
    """B Hk % 8 == 0: the XCD-grouped block order; GQA rep 2; O as [B, S, H, D]."""
    B, H, Hk, S = 1, 16, 8, 256
    check(rnd((B, H, S, 128), 4), rnd((B, Hk, S, 128), 5), rnd((B, Hk, S, 128), 6), bshd=True)


@pytest.mark.slow
def test_attn_fwd_three_blocks():
    """S = 768: query block 2 runs 7 unmasked bodies (odd count: the
    unrolled loop's mid exit)."""
    B, H, Hk, S = 1, 1, 1, 768
    check(rnd((B, H, S, 128), 7), rnd((B, Hk, S, 128), 8), rnd((B, Hk, S, 128), 9), bshd=True)


def test_attn_fwd_rescale_path():
    """Scores growing by ~64 (8.2 in log2 units at scale 1/sqrt(128)) per key
    tile: every tile's max exceeds the deferred threshold, so the
    out-of-line rescale runs on every loop body."""
    B, H, Hk, S = 1, 1, 1, 512
    q = np.ones((B, H, S, 128), np.float32)
    keys = np.arange(S, dtype=np.float32)[None, None, :, None] / 128.0
    k = np.broadcast_to(keys, (B, Hk, S, 128)).astype(np.float32) * (1 + 0.01 * rnd((B, Hk, S, 128), 10))
    v = rnd((B, Hk, S, 128), 11)
    hits = [0]
    check(q, k, v, hits=hits)
    # wave w of query block qb rescales for tiles 1 .. 4 qb + w (later tiles
    # are past its diagonal, fully masked): block 1 sum(4 + w), block 0 sum(w)
    assert hits[0] == sum(4 + w for w in range(4)) + sum(range(4))


def test_timing_arm_is_bit_identical_and_records():
    """The s_memtime arm (attn_gen.py VARIANTS "t1"): same O / LSE bits as
    the product kernel, one record per (workgroup, wave) with its tile count
    and query block."""
    B, H, Hk, S = 1, 1, 1, 512
    q, k, v = rnd((B, H, S, 128), 12), rnd((B, Hk, S, 128), 13), rnd((B, Hk, S, 128), 14)
    text = attn_gen.generate_all()
    outs = []
    for name in (attn_gen.NAME, attn_gen.NAME + "_t1"):
        mem = emu.Memory()
        qa, ka, va = (mem.add(bf16(x)) for x in (q, k, v))
        oa = mem.add(np.zeros((B, H, S, 128), np.uint16))
        la = mem.add(np.zeros((B, H, S), np.float32))
        dbg = np.zeros((2 * 4, 8), np.uint32)
        da = mem.add(dbg)
        c = float(np.float32(LOG2E / math.sqrt(128)))
        karg = struct.pack("<5Q4If5IQ", qa, ka, va, oa, la, B, H, Hk, S, c, 1, 2, 1, 0, 0, da)
        e = emu.Emu(text, name)
        for wg in range(2):
            e.run(karg, wg, mem)
        bufs = {base: b for base, b in mem.bufs}
        outs.append((bufs[oa].copy(), bufs[la].copy(), bufs[da].view(np.uint32).reshape(8, 8).copy()))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    rec = outs[1][2]
    # generic order: workgroup 0 = query block 1 (8 tiles), workgroup 1 = block 0 (4 tiles)
    assert list(rec[:4, 3]) == [8] * 4 and list(rec[4:, 3]) == [4] * 4
    assert list(rec[:4, 4]) == [1] * 4 and list(rec[4:, 4]) == [0] * 4
    assert (rec[:, :3] > 0).all()
