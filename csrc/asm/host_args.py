"""Kernel-argument packing for the generated assembly GEMMs, shared by the
CPU emulator tests and documented against csrc/hip/gemm_asm.hip, which packs
the same 80 bytes on the host side of the real launch."""
from __future__ import annotations

import struct

from gemm_gen import KARG, KARG_BYTES, MAP_DEFAULT  # noqa: E402  (csrc/asm on sys.path)


def grid_params(tiles_m: int, tiles_n: int):
    nwg = tiles_m * tiles_n
    return nwg, nwg >> 3, nwg & 7, 8 * tiles_n


def pack(X, W, C, S, ldx_b, ldw_b, ldc_b, lds_b, K, tiles_m, tiles_n, fw_b=0, fc_b=0, grid=None,
         tile_map=MAP_DEFAULT, phase=0) -> bytes:
    """grid: a persistent kernel's workgroup count; tile_map: the tile order
    (gemm_gen.KARG "map": log2 group | 16 for column groups); phase: the
    first wave's start offsets (gemm_gen.phase_delay)."""
    nwg, xq, xr, pg = grid_params(tiles_m, tiles_n)
    buf = bytearray(KARG_BYTES)
    struct.pack_into("<QQQQ", buf, KARG["X"], X, W, C, S)
    struct.pack_into("<IIII", buf, KARG["ldx"], ldx_b, ldw_b, ldc_b, lds_b)
    struct.pack_into("<IIIIII", buf, KARG["ktiles"], K // 64, tiles_m, tiles_n, xq, xr, pg)
    struct.pack_into("<II", buf, KARG["fw"], fw_b, fc_b)
    struct.pack_into("<II", buf, KARG["map"], tile_map, grid or 0)
    struct.pack_into("<I", buf, KARG["phase"], phase)
    return bytes(buf)


def tile_order(tiles_m: int, tiles_n: int, tile_map: int = MAP_DEFAULT) -> list[tuple[int, int]]:
    """(tm, tn) of workgroups 0, 1, ... as the prologue computes them: the
    XCD remap (workgroups b, b + 8, ... share an XCD; each XCD gets a
    contiguous range of the tile order), then groups of 2^lg tiles of the
    grouped dimension walking the other one."""
    nwg, xq, xr, _ = grid_params(tiles_m, tiles_n)
    lg, walk = tile_map & 15, tile_map >> 4
    a_n, b_n = (tiles_n, tiles_m) if walk else (tiles_m, tiles_n)
    out = []
    for b in range(nwg):
        xcd, bq = b & 7, b >> 3
        tile = (xcd * (xq + 1) if xcd < xr else xr * (xq + 1) + (xcd - xr) * xq) + bq
        group, within = divmod(tile, b_n << lg)
        first = group << lg
        gsz = min(a_n - first, 1 << lg)
        ta, tb = first + within % gsz, within // gsz
        out.append((tb, ta) if walk else (ta, tb))
    return out


def wgrad_plan(M: int, N: int, K: int) -> tuple[int, int]:
    """(full, split) of csrc/hip/wgrad.hip's wg_plan: whole-K tiles for
    whole waves of 256 CUs, the tail cut into 2..4 K-pieces that fill it."""
    tiles = (M // 256) * (N // 256)
    rem = tiles % 256
    if rem == 0:
        return tiles, 1
    best = 1
    for s in range(2, 5):
        if rem * s <= 256 and K % (128 * s) == 0 and K // s >= 512:
            best = s
    return (tiles, 1) if best == 1 else (tiles - rem, best)


def pack_nt(A, B, C, WS, lda_b, ldb_b, ldc_b, beta, K, tiles_m, tiles_n, full, split, tile_map=3, sq=0) -> bytes:
    """The weight-gradient kernel's block (csrc/asm/wgrad_gen.py KARG): the
    same bytes, with beta / full / rem / split in the forward kernels'
    lds / xq / xr / per_group slots and the tile order in the map slot
    (wgrad_gen.MAP_DEFAULT = 3: groups of 8 row tiles walk the columns)."""
    rem = tiles_m * tiles_n - full
    buf = bytearray(KARG_BYTES)
    struct.pack_into("<QQQQ", buf, 0, A, B, C, WS)
    struct.pack_into("<IIII", buf, 32, lda_b, ldb_b, ldc_b, beta)
    struct.pack_into("<IIIIII", buf, 48, K // 64, tiles_m, tiles_n, full, rem, split)
    struct.pack_into("<I", buf, KARG["map"], tile_map)
    struct.pack_into("<Q", buf, 88, sq)     # wgrad_gen.KARG "sq": the sum-of-squares partials (0 = off)
    return bytes(buf)
