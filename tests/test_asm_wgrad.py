"""CPU tests of the hand-written gfx950 assembly weight-gradient GEMM
(csrc/asm/wgrad_gen.py): its LDS image (one-DMA blocks, conflict-free
transposed reads, immediate fragment offsets) and the kernel's full
instruction stream in the functional emulator (csrc/asm/emu.py) against a
float64 reference: whole-K tiles with beta 0 / 1 and the split-K pieces'
fp32 partials.  tests/test_ops_gpu.py runs it on an MI355X."""
import itertools
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "csrc", "asm"))

import emu  # noqa: E402
import host_args  # noqa: E402
import wgrad_gen as W  # noqa: E402

TEXT = W.generate()


def bf16(x):
    return emu.bf16_rne(np.asarray(x, np.float32)).astype(np.uint16)


def tof(b):
    return (b.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def tr_addr(lane, f, k0, hi, colw=0):
    g, q, p = lane >> 4, (lane >> 2) & 3, lane & 3
    r = k0 + 8 * g + q + (4 if hi else 0)
    c = ((16 * f + colw) >> 3) + (p >> 1)
    return W.pos(r, c) + 8 * (p & 1)


def test_lds_image_blocks_and_banks():
    offs = sorted(W.pos(r, c) for r in range(64) for c in range(32))
    assert len(set(offs)) == 64 * 32 and offs[-1] + 16 == W.OPER
    for b in range(32):  # each row pair is one contiguous 1-KiB DMA block
        got = sorted(W.pos(2 * b + s, c) - W.blockbase(b) for s in range(2) for c in range(32))
        assert got == [16 * l for l in range(64)]
    assert W.LDS_BYTES <= 160 * 1024
    for f, k0, hi, colw in itertools.product(range(8), (0, 32), (0, 1), (0, 128)):
        addrs = [tr_addr(l, f, k0, hi, colw) for l in range(64)]
        for grp in (range(0, 32), range(32, 64)):  # ds_read_b64_tr_b16 lane groups, 64 banks
            banks = {}
            for l in grp:
                for d in range(2):
                    banks.setdefault((addrs[l] // 4 + d) % 64, set()).add(addrs[l] // 4 + d)
            assert max(len(v) for v in banks.values()) == 1, (f, k0, hi, colw)
        d = {tr_addr(l, f, k0, hi, colw) - tr_addr(l, 0, 0, hi, 0) for l in range(64)}
        assert d == {64 * f + W.SUB1 * (k0 // 32) + 4 * colw}  # an immediate per fragment


def run(M, N, T, beta, split=None, seed=0):
    rng = np.random.default_rng(seed)
    A = bf16(rng.standard_normal((T, M)))
    B = bf16(rng.standard_normal((T, N)))
    C0 = bf16(rng.standard_normal((M, N)))
    full, sp = host_args.wgrad_plan(M, N, T) if split is None else (0, split)
    tiles = (M // 256) * (N // 256)
    rem = tiles - full
    mem = emu.Memory()
    aa, ab, ac = mem.add(A), mem.add(B), mem.add(C0.copy())
    aw = mem.add(np.zeros(max(1, sp * rem) * 65536, np.float32))
    karg = host_args.pack_nt(aa, ab, ac, aw, 2 * M, 2 * N, 2 * N, beta, T, M // 256, N // 256, full, sp)
    e = emu.Emu(TEXT, "toa_wgrad_nt_asm")
    for wg in range(full + rem * sp):
        e.run(karg, wg, mem)
    C = tof(mem.bufs[2][1].view(np.uint16).reshape(M, N))
    ws = mem.bufs[3][1].view(np.float32)
    ref = tof(A).T @ tof(B) + (tof(C0) if beta else 0)
    return C, ws, ref, full, rem, sp


@pytest.mark.parametrize("beta,tile_map", [(0, 3), (1, 18)])
def test_wgrad_asm_sumsq_partials_emulated(beta, tile_map):
    """Kernarg "sq": each whole-K tile writes 256 per-lane sums of squares of
    its final fp32 values at slot (tm tiles_n + tn) 256 + tid, whatever the
    tile order; C is the same bit for bit as without the partials; the tile
    slots sum to the squared norm of the tile (fp32 values, before the bf16
    rounding of C)."""
    M, N, T = 512, 768, 256
    rng = np.random.default_rng(9)
    A = bf16(rng.standard_normal((T, M)))
    B = bf16(rng.standard_normal((T, N)))
    C0 = bf16(rng.standard_normal((M, N)))
    tm_n, tn_n = M // 256, N // 256
    outs = []
    for with_sq in (False, True):
        mem = emu.Memory()
        aa, ab, ac = mem.add(A), mem.add(B), mem.add(C0.copy())
        aw = mem.add(np.zeros(65536, np.float32))
        asq = mem.add(np.full(tm_n * tn_n * 256, np.nan, np.float32))
        karg = host_args.pack_nt(aa, ab, ac, aw, 2 * M, 2 * N, 2 * N, beta, T, tm_n, tn_n, tm_n * tn_n, 1,
                                 tile_map=tile_map, sq=asq if with_sq else 0)
        e = emu.Emu(TEXT, "toa_wgrad_nt_asm")
        for wg in range(tm_n * tn_n):
            e.run(karg, wg, mem)
        outs.append((mem.bufs[2][1].copy(), mem.bufs[4][1].view(np.float32).copy()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.isnan(outs[0][1]).all()                     # "sq" = 0: nothing written
    sq = outs[1][1].reshape(tm_n, tn_n, 256).astype(np.float64)
    ref = tof(A).T @ tof(B) + (tof(C0) if beta else 0)
    for tm in range(tm_n):
        for tn in range(tn_n):
            want = (ref[256 * tm:256 * (tm + 1), 256 * tn:256 * (tn + 1)] ** 2).sum()
            assert abs(sq[tm, tn].sum() - want) <= 1e-4 * want, (tm, tn)


@pytest.mark.parametrize("beta", [0, 1])
def test_wgrad_asm_full_tiles_emulated(beta):
    C, _, ref, full, rem, sp = run(256, 512, 256, beta, seed=beta)
    assert rem == 0
    err = np.abs(C - ref).max() / np.abs(ref).max()
    assert err < 8e-3, err


def test_wgrad_asm_k_pieces_emulated():
    """Every tile split into 2 k-pieces: the fp32 partials, tile-major, sum
    to the product (the reduce kernel's job on the GPU)."""
    M, N, T = 256, 256, 512
    C, ws, ref, full, rem, sp = run(M, N, T, 0, split=2, seed=3)
    tot = ws[:65536].reshape(256, 256).astype(np.float64) + ws[65536:131072].reshape(256, 256)
    err = np.abs(tot - ref).max() / np.abs(ref).max()
    assert err < 1e-5, err


def test_wgrad_round4_arm_matches_product_kernel():
    """The A/B arm with the round-4 schedule (toa_wgrad_nt_asm_v1: "spread"
    slot map, accumulators zeroed before the prologue DMA) writes the product
    kernel's C bit for bit, whole-K tiles and k-pieces."""
    import gemm_gen

    text = gemm_gen.generate()
    M, N, T = 256, 512, 384
    rng = np.random.default_rng(9)
    A = bf16(rng.standard_normal((T, M)))
    B = bf16(rng.standard_normal((T, N)))
    outs = []
    for name in ("toa_wgrad_nt_asm", "toa_wgrad_nt_asm_v1"):
        mem = emu.Memory()
        aa, ab, ac = mem.add(A), mem.add(B), mem.add(np.zeros((M, N), np.uint16))
        aw = mem.add(np.zeros(65536 * 4, np.float32))
        karg = host_args.pack_nt(aa, ab, ac, aw, 2 * M, 2 * N, 2 * N, 0, T, M // 256, N // 256, 0, 2)
        e = emu.Emu(text, name)
        for wg in range(4):
            e.run(karg, wg, mem)
        outs.append(mem.bufs[3][1].copy())
    assert np.array_equal(outs[0], outs[1])


def _map_coords(t, tm_n, tn_n, tile_map):
    """wgrad_gen / wgrad.hip wg_tile_coords_map: tile index -> (tm, tn)."""
    lg, walk = tile_map & 15, tile_map >> 4
    a_n, b_n = (tn_n, tm_n) if walk else (tm_n, tn_n)
    group, within = divmod(t, b_n << lg)
    first = group << lg
    gsz = min(a_n - first, 1 << lg)
    ta, tb = first + within % gsz, within // gsz
    return (tb, ta) if walk else (ta, tb)


@pytest.mark.parametrize("tile_map", [0, 2, 18, 20])
def test_wgrad_tile_maps_same_output(tile_map):
    """Other tile orders of the weight-gradient kernel (kernarg map, the TN
    kernels' encoding) give the default order's result bit for bit: whole-K
    tiles write the same C, and the k-pieces' fp32 partials -- slot j holding
    tail tile full + j of the ORDER, which the map-aware reduce kernel places
    by the same map -- assemble the same sums."""
    M, N, T = 768, 512, 256
    tm_n, tn_n = M // 256, N // 256
    rng = np.random.default_rng(23)
    A = bf16(rng.standard_normal((T, M)))
    B = bf16(rng.standard_normal((T, N)))
    outs = []
    for tmap, (full, sp) in ((3, (6, 1)), (tile_map, (6, 1)), (3, (0, 2)), (tile_map, (0, 2))):
        mem = emu.Memory()
        aa, ab, ac = mem.add(A), mem.add(B), mem.add(np.zeros((M, N), np.uint16))
        aw = mem.add(np.zeros(6 * 2 * 65536, np.float32))
        karg = host_args.pack_nt(aa, ab, ac, aw, 2 * M, 2 * N, 2 * N, 0, T, tm_n, tn_n, full, sp,
                                 tile_map=tmap)
        e = emu.Emu(TEXT, "toa_wgrad_nt_asm")
        for wg in range(full + (6 - full) * sp):
            e.run(karg, wg, mem)
        if sp == 1:
            outs.append(mem.bufs[2][1].copy())
            continue
        ws = mem.bufs[3][1].view(np.float32).reshape(sp, 6, 256, 256)
        C = np.zeros((M, N), np.float32)
        for j in range(6):
            tm, tn = _map_coords(full + j, tm_n, tn_n, tmap)
            C[256 * tm:256 * tm + 256, 256 * tn:256 * tn + 256] = ws[0, j] + ws[1, j]
        outs.append(C)
    assert np.array_equal(outs[0], outs[1])
    assert np.array_equal(outs[2], outs[3])
