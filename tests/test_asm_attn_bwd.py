"""CPU tests of the hand-written gfx950 attention dK / dV backward
(csrc/asm/attn_bwd_gen.py): every workgroup of small problems run
instruction by instruction in csrc/asm/emu.py, compared with an fp64 causal
attention backward of the same bf16 inputs -- dK, dV and every dS block of
the dQ GEMM's packed layout.  Covers GQA (several query-head passes per kv
head), both dO layouts, the RoPE epilogue (d(qkv) rows), the masked /
unmasked loop-body variants, the clamped last DMA and the dropped stores of
blocks above the diagonal."""
from __future__ import annotations

import math
import os
import struct
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "csrc", "asm"))
import attn_bwd_gen  # noqa: E402
import emu  # noqa: E402

TEXT = attn_bwd_gen.generate()
LOG2E = 1.4426950408889634


def bf16(x: np.ndarray) -> np.ndarray:
    return emu.bf16_rne(np.asarray(x, np.float32)).astype(np.uint16)


def unbf16(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(np.float32)


def rnd(shape, seed, s=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * s).astype(np.float32)


def reference(q, k, v, do, scale):
    """fp64 causal attention forward + backward pieces; all [B, H(k), S, D]."""
    B, H, S, D = q.shape
    rep = H // k.shape[1]
    kk = np.repeat(k, rep, axis=1).astype(np.float64)
    vv = np.repeat(v, rep, axis=1).astype(np.float64)
    q64, do64 = q.astype(np.float64), do.astype(np.float64)
    s = np.einsum("bhqd,bhkd->bhqk", q64, kk) * scale
    causal = np.tril(np.ones((S, S), bool))
    s = np.where(causal, s, -np.inf)
    m = s.max(-1, keepdims=True)
    p = np.exp(s - m)
    l = p.sum(-1, keepdims=True)
    lse = (m + np.log(l))[..., 0]
    p = p / l
    o = np.einsum("bhqk,bhkd->bhqd", p, vv)
    return p, o, lse, kk, vv


def run(q, k, v, do, bshd=False, rope=False, seed=0, text=None, name=None):
    B, H, S, D = q.shape
    Hk = k.shape[1]
    rep = H // Hk
    scale = 1.0 / math.sqrt(D)
    qb, kb, vb, dob = (unbf16(bf16(x)) for x in (q, k, v, do))
    p, o, lse, kk, vv = reference(qb, kb, vb, dob, scale)
    ob = unbf16(bf16(o.astype(np.float32))).astype(np.float64)
    delta = (dob.astype(np.float64) * ob).sum(-1)                      # [B, H, S]
    dp = np.einsum("bhqd,bhkd->bhqk", dob.astype(np.float64), vv)
    ds = p * (dp - delta[..., None])                                   # unscaled
    dv = np.einsum("bhqk,bhqd->bhkd", p, dob.astype(np.float64)).reshape(B, Hk, rep, S, D).sum(2)
    dk = scale * np.einsum("bhqk,bhqd->bhkd", ds, qb.astype(np.float64)).reshape(B, Hk, rep, S, D).sum(2)
    # inputs as the kernel sees them
    mem = emu.Memory()
    qa = mem.add(bf16(qb))
    ka, va = mem.add(bf16(kb)), mem.add(bf16(vb))
    do_l = dob.transpose(0, 2, 1, 3).copy() if bshd else dob
    doa = mem.add(bf16(do_l))
    nlse = mem.add((-lse * LOG2E).astype(np.float32))
    ndel = mem.add((-delta).astype(np.float32))
    nb = S // 32
    nblk = nb * (nb + 1) // 2
    ds_buf = np.full((B, H, nblk, 1024), 0x7FC1, np.uint16)             # NaN: every slot must be written
    dsa = mem.add(ds_buf)
    H3 = H + 2 * Hk
    if rope:
        pos = np.arange(S)[:, None].astype(np.float64)
        inv = 10000.0 ** (-np.arange(D // 2) * 2.0 / D)
        ang = pos * inv[None, :]
        cosv, sinv = np.cos(ang).astype(np.float32), np.sin(ang).astype(np.float32)
        cosa, sina = mem.add(cosv), mem.add(sinv)
        dqkv = np.zeros((B, S, H3, D), np.uint16)
        dka = dva = mem.add(dqkv)
    else:
        cosa = sina = 0
        dka = mem.add(np.zeros((B, Hk, S, D), np.uint16))
        dva = mem.add(np.zeros((B, Hk, S, D), np.uint16))
    c = float(np.float32(scale * LOG2E))
    flags = (1 if bshd else 0) | (2 if rope else 0)
    nkb = S // 128
    karg = struct.pack("<12Q4I2f4I2I", qa, ka, va, doa, nlse, ndel, dka, dva, dsa, cosa, sina, 0,
                       B, H, Hk, S, scale, c, flags, rep, nkb, H3, 0, 0)
    assert len(karg) == attn_bwd_gen.KARG_BYTES
    e = emu.Emu(text or TEXT, name or attn_bwd_gen.NAME)
    e.dropped = 0
    for wg in range(nkb * B * Hk):
        e.run(karg, wg, mem)
    bufs = {base: b for base, b in mem.bufs}
    if rope:
        out = unbf16(bufs[dka].view(np.uint16).reshape(B, S, H3, D)).astype(np.float64)
        dk_out = out[:, :, H:H + Hk].transpose(0, 2, 1, 3)
        dv_out = out[:, :, H + Hk:].transpose(0, 2, 1, 3)
        # RoPE backward on the reference: dx1 = dy1 c + dy2 s, dx2 = dy2 c - dy1 s
        c64, s64 = cosv.astype(np.float64), sinv.astype(np.float64)
        d1, d2 = dk[..., :D // 2], dk[..., D // 2:]
        dk = np.concatenate([d1 * c64 + d2 * s64, d2 * c64 - d1 * s64], -1)
    else:
        dk_out = unbf16(bufs[dka].view(np.uint16).reshape(B, Hk, S, D)).astype(np.float64)
        dv_out = unbf16(bufs[dva].view(np.uint16).reshape(B, Hk, S, D)).astype(np.float64)
    ds_out = bufs[dsa].view(np.uint16).reshape(B, H, nblk, 1024)
    return dict(dk=dk, dv=dv, ds=ds, dk_out=dk_out, dv_out=dv_out, ds_out=ds_out, dropped=e.dropped, nb=nb)


def unpack_ds(ds_out, nb, S):
    """Packed dS blocks -> dense [B, H, S, S] (zeros above the diagonal blocks)."""
    B, H = ds_out.shape[:2]
    dense = np.zeros((B, H, S, S), np.float64)
    for qi in range(nb):
        for ki in range(qi + 1):
            blk = unbf16(ds_out[:, :, qi * (qi + 1) // 2 + ki]).reshape(B, H, 4, 32, 8)   # [g][key][q % 8]
            dense[:, :, qi * 32:(qi + 1) * 32, ki * 32:(ki + 1) * 32] = blk.transpose(0, 1, 2, 4, 3).reshape(B, H, 32, 32)
    return dense


def check(r, S):
    for name in ("dk", "dv"):
        ref, got = r[name], r[name + "_out"]
        err = np.abs(got - ref).max()
        assert err < 2e-2 * max(1.0, np.abs(ref).max()), f"{name} max err {err}"
    got = unpack_ds(r["ds_out"], r["nb"], S)
    assert np.isfinite(got).all(), "a dS block slot was never written"
    ref = np.tril(np.ones((S, S))) * r["ds"]
    err = np.abs(got - ref).max()
    assert err < 1e-2 * max(1.0, np.abs(ref).max()), f"dS max err {err}"


def expected_drops(B, H, Hk, S, per_block=None):
    """Stores of blocks wholly above the diagonal: per (kv head, query head,
    key block kb) step mod < 2, half m, wave w with 2 mod + m < w -- two
    16-B stores each (four 8-B ones in round 5's form, arm s8)."""
    if per_block is None:
        per_block = 2 if attn_bwd_gen.KNOBS["dswide"] else 4
    rep = H // Hk
    per = sum(1 for mod in range(2) for m in range(2) for w in range(4) if 2 * mod + m < w)
    return per_block * per * B * Hk * rep * (S // 128)


def test_kernel_mfma_count():
    lines = [ln for ln in TEXT.splitlines() if ln.startswith("  v_mfma")]
    # fill (32) + 3 buffer phases x (4 iteration variants x 64 + 2 tails x 32)
    assert len(lines) == 32 + 3 * (4 * 64 + 2 * 32)


def test_dkdv_single_head_s256():
    """S = 256: key blocks 0 (4 steps: both masked steps, unmasked, tail) and 1
    (2 steps: masked then the tail; the DMA clamped to the last tile)."""
    B, H, Hk, S = 1, 1, 1, 256
    r = run(rnd((B, H, S, 128), 1), rnd((B, Hk, S, 128), 2), rnd((B, Hk, S, 128), 3), rnd((B, H, S, 128), 4))
    check(r, S)
    assert r["dropped"] == expected_drops(B, H, Hk, S)


def test_dkdv_gqa_bshd():
    """GQA rep 2 (two query-head passes: the mask variants recur at each
    pass start), dO as [B, S, H, D]."""
    B, H, Hk, S = 1, 2, 1, 256
    r = run(rnd((B, H, S, 128), 5), rnd((B, Hk, S, 128), 6), rnd((B, Hk, S, 128), 7), rnd((B, H, S, 128), 8),
            bshd=True)
    check(r, S)
    assert r["dropped"] == expected_drops(B, H, Hk, S)


def test_dkdv_rope_epilogue():
    """flags bit 1: dK rotated back and dK / dV written into d(qkv) rows."""
    B, H, Hk, S = 1, 2, 1, 256
    r = run(rnd((B, H, S, 128), 9), rnd((B, Hk, S, 128), 10), rnd((B, Hk, S, 128), 11), rnd((B, H, S, 128), 12),
            bshd=True, rope=True)
    check(r, S)


@pytest.mark.slow
def test_dkdv_s512_two_kv_heads():
    """S = 512 (8-step passes: every iteration variant), B Hk = 2."""
    B, H, Hk, S = 1, 4, 2, 512
    r = run(rnd((B, H, S, 128), 13), rnd((B, Hk, S, 128), 14), rnd((B, Hk, S, 128), 15), rnd((B, H, S, 128), 16))
    check(r, S)


def test_dkdv_packed_valu_arm_matches():
    """Arm s7 (round 5's P / dS on packed v_pk_fma_f32 / v_pk_mul_f32 pairs;
    the product kernel now uses scalar ops): the same dK / dV / dS to fp64
    tolerance, the diagonal blocks' stores dropped the same way."""
    knobs = dict(attn_bwd_gen.VARIANTS)["s7"]
    text = attn_bwd_gen.generate([attn_bwd_gen.variant_kernel("s7", knobs)])
    B, H, Hk, S = 1, 2, 1, 256
    r = run(rnd((B, H, S, 128), 5), rnd((B, Hk, S, 128), 6), rnd((B, Hk, S, 128), 7), rnd((B, H, S, 128), 8),
            bshd=True, text=text, name=attn_bwd_gen.NAME + "_s7")
    check(r, S)
    assert r["dropped"] == expected_drops(B, H, Hk, S)   # (s7 keeps the 16-B stores)


def test_dkdv_wide_store_arm_matches():
    """Arm s8 (two 16-B dS stores per block built by permlane32 swaps instead
    of the product's four 8-B ones; the barrier's vmcnt counts two): the same
    outputs under the strict-VMEM emulator, two drops per block."""
    knobs = dict(attn_bwd_gen.VARIANTS)["s8"]
    text = attn_bwd_gen.generate([attn_bwd_gen.variant_kernel("s8", knobs)])
    B, H, Hk, S = 1, 2, 1, 256
    r = run(rnd((B, H, S, 128), 5), rnd((B, Hk, S, 128), 6), rnd((B, Hk, S, 128), 7), rnd((B, H, S, 128), 8),
            bshd=True, text=text, name=attn_bwd_gen.NAME + "_s8")
    check(r, S)
    assert r["dropped"] == expected_drops(B, H, Hk, S, per_block=2)
