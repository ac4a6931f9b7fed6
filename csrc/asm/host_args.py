"""Kernel-argument packing for the generated assembly GEMMs, shared by the
CPU emulator tests and documented against csrc/hip/gemm_asm.hip, which packs
the same 80 bytes on the host side of the real launch."""
from __future__ import annotations

import struct

from gemm_gen import KARG, KARG_BYTES  # noqa: E402  (csrc/asm on sys.path)


def grid_params(tiles_m: int, tiles_n: int):
    nwg = tiles_m * tiles_n
    return nwg, nwg >> 3, nwg & 7, 8 * tiles_n


def pack(X, W, C, S, ldx_b, ldw_b, ldc_b, lds_b, K, tiles_m, tiles_n, fw_b=0, fc_b=0) -> bytes:
    nwg, xq, xr, pg = grid_params(tiles_m, tiles_n)
    buf = bytearray(KARG_BYTES)
    struct.pack_into("<QQQQ", buf, KARG["X"], X, W, C, S)
    struct.pack_into("<IIII", buf, KARG["ldx"], ldx_b, ldw_b, ldc_b, lds_b)
    struct.pack_into("<IIIIII", buf, KARG["ktiles"], K // 64, tiles_m, tiles_n, xq, xr, pg)
    struct.pack_into("<II", buf, KARG["fw"], fw_b, fc_b)
    return bytes(buf)
