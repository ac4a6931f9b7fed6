#!/usr/bin/env python3
"""Generator of the hand-written gfx950 assembly weight-gradient GEMM ("NT").

    C[m][n] (+)= sum_t A[t][m] * B[t][n]      bf16 in, fp32 accumulate

with A = dY [T][M] (row stride lda), B = X [T][N] (ldb), C = dW [M][N] (ldc):
dW = dY^T X without a transpose.  Both operands are contiguous along the
OUTPUT dimensions, so the MFMA operands come out of LDS transposed by
``ds_read_b64_tr_b16``.  The schedule is the forward kernel's
(csrc/asm/gemm_gen.py: 4 waves, one per SIMD, 128 x 128 of C per wave,
v_mfma_f32_16x16x32_bf16 into 256 AGPR accumulators, LDS-DMA two tiles
ahead, pieces spread over the iteration); what differs is the LDS image:

  LDS image   per operand and stage 64 rows (t) x 256 columns.  Row pair
              (2b, 2b+1) is one 1-KiB block -- one LDS-DMA instruction, its
              64 lanes' 16-B pieces contiguous -- at blockbase(b) =
              1216 b + 128 [b mod 8 in {1, 4, 6, 7}].  Inside a block, chunk
              c (8 columns) of row 2b + s sits at 64 (c >> 1) + 16 (2 s +
              (c & 1)).  For a transposed read (32 lanes: rows {0..3, 8..11}
              + k0, or {16..19, 24..27}, 16 B per row pair of chunks) the
              eight 32-B segments land in eight distinct 32-B bank slots
              (2 LDS cycles per read, conflict-free), and fragment f is
              +64 f bytes from fragment 0, sub-step 1 +19456 bytes: every
              read is base + immediate (two base VGPRs per operand, rows
              +0 and +4).  Checked by tests/test_asm_wgrad.py.
  staging     wave w issues the blocks b = 8 w + j (j = 0..7) of each
              operand: lane l loads row 2b + ((l >> 1) & 1), chunk
              2 (l >> 2) + (l & 1); the row pair's stride is a per-piece
              SGPR offset, M0 steps through blockbase.
  split-K     like csrc/hip/wgrad.hip: the `full` tiles run over the whole
              T and store bf16 (beta: read-modify-write); the tiles of a
              part-empty last wave are cut into `split` k-pieces that store
              fp32 partials tile-major into the workspace, summed in a
              fixed order by wgrad_tile_reduce_kernel (deterministic).
  epilogue    lane l of wave (wm, wn) holds C[m][n .. n+3] with m = 128 wm +
              16 i + (l & 15), n = 128 wn + 16 j + 4 (l >> 4): 8-byte stores
              (bf16) or 16-byte stores (fp32 partials).

Kernarg (80 B, the forward kernels' block; csrc/hip/gemm_asm.hip
toa_wgrad_asm): A, B, C, WS pointers, lda/ldb/ldc bytes, beta, K tiles of
the whole T, tiles_m, tiles_n, full, rem, split.

Reference anchor: SURVEY.md K1/K2 (the training step's GEMMs); the
reference itself has no kernels.
"""
from __future__ import annotations

import sys

import gemm_gen as G
from gemm_gen import Asm, ar, sr, vr

BLOCK = 1216
HMASK = 0xD2                       # blocks b with b % 8 in {1, 4, 6, 7} sit 128 B further
OPER = 31 * BLOCK + 128 + 1024     # 38848 B per operand and stage
STAGE = 2 * OPER                   # 77696
LDS_BYTES = 2 * STAGE              # 155392
SUB1 = 16 * BLOCK                  # rows + 32 = blocks + 16: 19456 B


def blockbase(b: int) -> int:
    return BLOCK * b + 128 * ((HMASK >> (b % 8)) & 1)


def pos(r: int, c: int) -> int:
    """Byte offset of row r (0..63), 16-B chunk c (0..31) in one operand image."""
    return blockbase(r >> 1) + 64 * (c >> 1) + 16 * (2 * (r & 1) + (c & 1))


# kernarg block (byte offsets)
KARG = {"A": 0, "B": 8, "C": 16, "WS": 24, "lda": 32, "ldb": 36, "ldc": 40, "beta": 44, "ktiles": 48,
        "tiles_m": 52, "tiles_n": 56, "full": 60, "rem": 64, "split": 68, "map": 80, "sq": 88}
MAP_DEFAULT = 3     # groups of 8 row tiles (dW rows) walk the column tiles: the round-4/5 order

# SGPRs
S_A, S_B, S_C, S_WS = 4, 6, 8, 10
S_LDA, S_LDB, S_LDC, S_BETA = 12, 13, 14, 15
S_KT, S_TM_N, S_TN_N, S_FULL, S_REM, S_SPLIT = 16, 17, 18, 19, 20, 21
S_TILE, S_TM, S_TN = 24, 25, 26
S_T0, S_T1, S_T2, S_T3 = 27, 28, 29, 30
SRD_A, SRD_B, SRD_C, SRD_WS = 32, 36, 40, 44
S_M0A, S_M0AT, S_M0B, S_M0BT = 48, 49, 50, 51
S_LOOP = 52
S_SOA = 53          # s53..s59: A row-pair offsets of pieces 1..7
S_SOB = 60          # s60..s66
S_E0, S_E1 = 67, 68
S_Q, S_R = 69, 70
S_S, S_J, S_PIECE = 71, 72, 73   # k-piece index, tail tile index, 1 for a k-piece workgroup
S_ADVA, S_ADVB, S_KTP = 74, 75, 76   # 64 lda, 64 ldb, k-tiles of this workgroup
S_MAPW, S_LG, S_WALK = 77, 78, 79    # kernarg tile order (gemm_gen.KARG "map"): word, log2 group, walk flag
SRD_SQ = 80         # s80..s83: the sum-of-squares partials (kernarg "sq" in s[80:81]; 0 = off)
N_SGPR = 84

# VGPRs
V_DA, V_RALO, V_RAHI = 1, 2, 3
V_FA0, V_FA1, V_FB0, V_FB1 = 4, 36, 68, 100     # fragments: A (m) / B (n), sub-steps 0 / 1
V_TID, V_DB, V_RBLO, V_RBHI = 132, 133, 134, 135
V_T = 136                                        # 136..139 scratch
V_TGALO, V_TGAHI, V_TGBLO, V_TGBHI = 140, 141, 142, 143
V_E = 144                                        # 144..255 epilogue scratch
V_SQ = V_E + 100                                 # 244..247: sum-of-squares accumulators (whole-K tiles)

# slot map: the forward kernel's product placement (gemm_gen.SLOT_MAPS
# "lib0": barriers one MFMA after their waits, M0 / resource advances one
# MFMA behind the pieces); KNOBS["map"] selects another for an A/B arm
KNOBS = {"map": "lib0", "zero_late": True}


def prologue(a: Asm):
    a(f"s_load_dwordx16 {sr(4, 16)}, s[0:1], 0x0")
    a(f"s_load_dwordx4 {sr(20, 4)}, s[0:1], 0x40")
    a(f"s_load_dword {sr(S_MAPW)}, s[0:1], {KARG['map']:#x}")
    a(f"s_load_dwordx2 {sr(SRD_SQ, 2)}, s[0:1], {KARG['sq']:#x}")
    a("s_mov_b32 m0, 0")
    a(f"v_mov_b32 {vr(V_TID)}, v0")
    a("s_waitcnt lgkmcnt(0)")
    # argument guard: 2 <= ktiles / split, split in 1..4, s2 < full + rem * split
    a(f"s_cmp_lt_u32 {sr(S_SPLIT)}, 1")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_cmp_gt_u32 {sr(S_SPLIT)}, 4")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_mul_i32 {sr(S_T0)}, {sr(S_REM)}, {sr(S_SPLIT)}")
    a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_FULL)}")
    a(f"s_cmp_ge_u32 s2, {sr(S_T0)}")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_mul_i32 {sr(S_T1)}, {sr(S_TM_N)}, {sr(S_TN_N)}")
    a(f"s_add_u32 {sr(S_T2)}, {sr(S_FULL)}, {sr(S_REM)}")
    a(f"s_cmp_lg_u32 {sr(S_T1)}, {sr(S_T2)}")
    a(f"s_cbranch_scc1 {a.abort}")
    # --- which tile / k-piece: blocks [0, full) whole-K tiles, then the pieces
    l_piece, l_done = a.fresh("piece"), a.fresh("mapped")
    a(f"s_mov_b32 {sr(S_S)}, 0")
    a(f"s_mov_b32 {sr(S_PIECE)}, 0")
    a(f"s_mov_b32 {sr(S_KTP)}, {sr(S_KT)}")
    a(f"s_cmp_ge_u32 s2, {sr(S_FULL)}")
    a(f"s_cbranch_scc1 {l_piece}")
    xcd_remap(a, S_TILE, "s2", S_FULL)
    a(f"s_branch {l_done}")
    a.label(l_piece)
    a(f"s_sub_u32 {sr(S_T3)}, s2, {sr(S_FULL)}")
    a(f"s_mul_i32 {sr(S_T0)}, {sr(S_REM)}, {sr(S_SPLIT)}")
    xcd_remap(a, S_E0, sr(S_T3), S_T0)                 # w2
    G.udiv(a, S_Q, S_R, S_E0, S_REM)                  # s = w2 / rem, j = w2 % rem
    a(f"s_mov_b32 {sr(S_S)}, {sr(S_Q)}")
    a(f"s_mov_b32 {sr(S_J)}, {sr(S_R)}")
    a(f"s_add_u32 {sr(S_TILE)}, {sr(S_FULL)}, {sr(S_R)}")
    a(f"s_mov_b32 {sr(S_PIECE)}, 1")
    G.udiv(a, S_Q, S_R, S_KT, S_SPLIT)                # k-tiles per piece
    a(f"s_mov_b32 {sr(S_KTP)}, {sr(S_Q)}")
    a.label(l_done)
    a(f"s_cmp_lt_u32 {sr(S_KTP)}, 2")
    a(f"s_cbranch_scc1 {a.abort}")
    # --- tile -> (tm, tn) by the kernarg map (the TN kernels' encoding,
    # gemm_gen.tile_setup): groups of 2^lg tiles of the grouped dimension
    # (rows of dW; columns when the walk bit is set) walk the other one.
    # A word the host never packs (lg > 6, bits above the walk flag) ends
    # the workgroup before any memory access.
    a(f"s_and_b32 {sr(S_LG)}, {sr(S_MAPW)}, 15")
    a(f"s_cmp_gt_u32 {sr(S_LG)}, 6")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_cmp_ge_u32 {sr(S_MAPW)}, 32")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_lshr_b32 {sr(S_WALK)}, {sr(S_MAPW)}, 4")
    a(f"s_cmp_eq_u32 {sr(S_WALK)}, 0")
    a(f"s_cselect_b32 {sr(S_E0)}, {sr(S_TM_N)}, {sr(S_TN_N)}")   # grouped count
    a(f"s_cselect_b32 {sr(S_E1)}, {sr(S_TN_N)}, {sr(S_TM_N)}")   # walked count
    a(f"s_lshl_b32 {sr(S_T3)}, {sr(S_E1)}, {sr(S_LG)}")          # tiles per group
    G.udiv(a, S_Q, S_R, S_TILE, S_T3)
    a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_Q)}, {sr(S_LG)}")          # first grouped tile
    a(f"s_sub_u32 {sr(S_T1)}, {sr(S_E0)}, {sr(S_T0)}")
    a(f"s_lshl_b32 {sr(S_T2)}, 1, {sr(S_LG)}")
    a(f"s_min_u32 {sr(S_T1)}, {sr(S_T1)}, {sr(S_T2)}")          # this group's size
    a(f"s_mov_b32 {sr(S_T2)}, {sr(S_R)}")
    G.udiv(a, S_Q, S_R, S_T2, S_T1)
    a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_R)}")           # grouped-dimension tile
    a(f"s_cmp_eq_u32 {sr(S_WALK)}, 0")
    a(f"s_cselect_b32 {sr(S_TM)}, {sr(S_T0)}, {sr(S_Q)}")
    a(f"s_cselect_b32 {sr(S_TN)}, {sr(S_Q)}, {sr(S_T0)}")

    # --- buffer resources: 64 rows x 256 columns from row k_begin, column 256 tm / tn
    a(f"s_mul_i32 {sr(S_T3)}, {sr(S_S)}, {sr(S_KTP)}")
    a(f"s_lshl_b32 {sr(S_T3)}, {sr(S_T3)}, 6")         # k_begin (rows)
    for srd_, base, ld, t, adv in ((SRD_A, S_A, S_LDA, S_TM, S_ADVA), (SRD_B, S_B, S_LDB, S_TN, S_ADVB)):
        G.mul64(a, S_T0, S_T1, S_T3, ld)              # k_begin * ld
        a(f"s_lshl_b32 {sr(S_T2)}, {sr(t)}, 9")       # 256 columns * 2 B
        a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_T2)}")
        a(f"s_addc_u32 {sr(S_T1)}, {sr(S_T1)}, 0")
        a(f"s_mul_i32 {sr(S_T2)}, {sr(ld)}, 63")
        a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, 512")
        G.srd(a, srd_, base, S_T0, S_T1, S_T2)
        a(f"s_lshl_b32 {sr(adv)}, {sr(ld)}, 6")
    # C: rows 256 tm, columns 256 tn (bf16); WS: tile (s * rem + j) of 256 x 256 fp32
    a(f"s_lshl_b32 {sr(S_T2)}, {sr(S_TM)}, 8")
    G.mul64(a, S_T0, S_T1, S_T2, S_LDC)
    a(f"s_lshl_b32 {sr(S_T2)}, {sr(S_TN)}, 9")
    a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_T2)}")
    a(f"s_addc_u32 {sr(S_T1)}, {sr(S_T1)}, 0")
    a(f"s_lshl_b32 {sr(S_T2)}, {sr(S_LDC)}, 8")
    G.srd(a, SRD_C, S_C, S_T0, S_T1, S_T2)
    a(f"s_mul_i32 {sr(S_T2)}, {sr(S_S)}, {sr(S_REM)}")
    a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_J)}")
    a(f"s_lshl_b32 {sr(S_T2)}, {sr(S_T2)}, 18")        # 256 KiB per fp32 tile
    a(f"s_lshr_b32 {sr(S_T3)}, {sr(S_T2)}, 0")
    # (tile index < 2^14 pieces: the byte offset stays 32-bit; host checks)
    a(f"s_mov_b32 {sr(S_T1)}, 0")
    a(f"s_mov_b32 {sr(S_T0)}, {sr(S_T2)}")
    a(f"s_mov_b32 {sr(S_T2)}, 0x40000")
    G.srd(a, SRD_WS, S_WS, S_T0, S_T1, S_T2)

    # --- DMA lane offsets: wave w's piece j is block b = 8 w + j; lane l loads
    # row 2 b + ((l >> 1) & 1), chunk 2 (l >> 2) + (l & 1)
    v = V_T
    a(f"v_lshrrev_b32 {vr(v)}, 6, {vr(V_TID)}")                 # w
    a(f"v_and_b32 {vr(v + 1)}, 63, {vr(V_TID)}")                # lane
    a(f"v_bfe_u32 {vr(v + 2)}, {vr(v + 1)}, 1, 1")              # s
    a(f"v_lshl_add_u32 {vr(v + 2)}, {vr(v)}, 4, {vr(v + 2)}")   # row = 16 w + s
    a(f"v_lshrrev_b32 {vr(v + 3)}, 2, {vr(v + 1)}")
    a(f"v_and_b32 {vr(V_E)}, 1, {vr(v + 1)}")
    a(f"v_lshl_add_u32 {vr(v + 3)}, {vr(v + 3)}, 1, {vr(V_E)}")  # chunk
    a(f"v_lshlrev_b32 {vr(v + 3)}, 4, {vr(v + 3)}")             # chunk bytes
    a(f"v_mul_lo_u32 {vr(V_DA)}, {vr(v + 2)}, {sr(S_LDA)}")
    a(f"v_add_u32 {vr(V_DA)}, {vr(V_DA)}, {vr(v + 3)}")
    a(f"v_mul_lo_u32 {vr(V_DB)}, {vr(v + 2)}, {sr(S_LDB)}")
    a(f"v_add_u32 {vr(V_DB)}, {vr(V_DB)}, {vr(v + 3)}")
    for j in range(1, 8):
        a(f"s_mul_i32 {sr(S_SOA + j - 1)}, {sr(S_LDA)}, {2 * j}")
        a(f"s_mul_i32 {sr(S_SOB + j - 1)}, {sr(S_LDB)}, {2 * j}")
    # M0 bases: stage 0, operand image, wave block 8 w
    a("s_nop 4")
    a(f"v_readfirstlane_b32 {sr(S_T0)}, {vr(v)}")
    a("s_nop 4")
    a(f"s_mul_i32 {sr(S_M0A)}, {sr(S_T0)}, {blockbase(8)}")
    a(f"s_add_u32 {sr(S_M0AT)}, {sr(S_M0A)}, {STAGE}")
    a(f"s_xor_b32 {sr(S_M0AT)}, {sr(S_M0AT)}, {sr(S_M0A)}")
    a(f"s_add_u32 {sr(S_M0B)}, {sr(S_M0A)}, {OPER}")
    a(f"s_add_u32 {sr(S_M0BT)}, {sr(S_M0B)}, {STAGE}")
    a(f"s_xor_b32 {sr(S_M0BT)}, {sr(S_M0BT)}, {sr(S_M0B)}")

    # --- fragment read bases: lane (g, q, p) = (l >> 4, (l >> 2) & 3, l & 3):
    # blockbase(4 g + (q >> 1)) + 32 (q & 1) + 8 p + 512 (wave column half);
    # the +4-row read at blockbase(... + 2)
    a(f"v_lshrrev_b32 {vr(v + 2)}, 4, {vr(v + 1)}")             # g
    a(f"v_bfe_u32 {vr(v + 3)}, {vr(v + 1)}, 3, 1")              # q >> 1
    a(f"v_lshl_add_u32 {vr(v + 2)}, {vr(v + 2)}, 2, {vr(v + 3)}")   # beta = 4 g + (q >> 1)
    a(f"v_bfe_u32 {vr(v + 3)}, {vr(v + 1)}, 2, 1")              # q & 1
    a(f"v_and_b32 {vr(V_E)}, 3, {vr(v + 1)}")                   # p
    a(f"v_lshlrev_b32 {vr(V_E)}, 3, {vr(V_E)}")
    a(f"v_lshl_add_u32 {vr(V_E)}, {vr(v + 3)}, 5, {vr(V_E)}")   # 32 (q & 1) + 8 p
    for dst, dbeta in ((V_RALO, 0), (V_RAHI, 2)):
        a(f"v_add_u32 {vr(V_E + 1)}, {dbeta}, {vr(v + 2)}")
        blockbase_v(a, V_E + 2, V_E + 1, V_E + 3)
        a(f"v_add_u32 {vr(dst)}, {vr(V_E + 2)}, {vr(V_E)}")
    a(f"v_and_b32 {vr(v + 3)}, 1, {vr(v)}")                     # wm
    a(f"v_lshlrev_b32 {vr(v + 3)}, 9, {vr(v + 3)}")
    a(f"v_lshrrev_b32 {vr(V_E + 1)}, 1, {vr(v)}")               # wn
    a(f"v_lshlrev_b32 {vr(V_E + 1)}, 9, {vr(V_E + 1)}")
    a(f"v_add_u32 {vr(V_RBLO)}, {vr(V_RALO)}, {vr(V_E + 1)}")
    a(f"v_add_u32 {vr(V_RBHI)}, {vr(V_RAHI)}, {vr(V_E + 1)}")
    a(f"v_add_u32 {vr(V_RBLO)}, {OPER}, {vr(V_RBLO)}")
    a(f"v_add_u32 {vr(V_RBHI)}, {OPER}, {vr(V_RBHI)}")
    a(f"v_add_u32 {vr(V_RALO)}, {vr(V_RALO)}, {vr(v + 3)}")
    a(f"v_add_u32 {vr(V_RAHI)}, {vr(V_RAHI)}, {vr(v + 3)}")
    for base, tg in ((V_RALO, V_TGALO), (V_RAHI, V_TGAHI), (V_RBLO, V_TGBLO), (V_RBHI, V_TGBHI)):
        a(f"v_add_u32 {vr(tg)}, {STAGE}, {vr(base)}")
        a(f"v_xor_b32 {vr(tg)}, {vr(tg)}, {vr(base)}")
    if not KNOBS["zero_late"]:
        zero_acc(a)


def zero_acc(a: Asm):
    for i in range(256):
        a(f"v_accvgpr_write_b32 {ar(i)}, 0")


def blockbase_v(a: Asm, dst: int, b: int, t: int):
    """dst = blockbase(b) = 1216 b + 128 ((HMASK >> (b & 7)) & 1) (VALU)."""
    a(f"v_and_b32 {vr(t)}, 7, {vr(b)}")
    a(f"v_mov_b32 {vr(dst)}, {HMASK}")
    a(f"v_lshrrev_b32 {vr(t)}, {vr(t)}, {vr(dst)}")
    a(f"v_and_b32 {vr(t)}, 1, {vr(t)}")
    a(f"v_lshlrev_b32 {vr(t)}, 7, {vr(t)}")
    a(f"v_mul_u32_u24 {vr(dst)}, {BLOCK}, {vr(b)}")
    a(f"v_add_u32 {vr(dst)}, {vr(dst)}, {vr(t)}")


def xcd_remap(a: Asm, dst: int, bid: str, n: int):
    """dst = the XCD-contiguous order of block `bid` among s[n] blocks."""
    a(f"s_lshr_b32 {sr(S_E1)}, {sr(n)}, 3")                 # q
    a(f"s_and_b32 {sr(S_R)}, {sr(n)}, 7")                   # r
    a(f"s_and_b32 {sr(S_T0)}, {bid}, 7")                    # xcd
    a(f"s_lshr_b32 {sr(S_T1)}, {bid}, 3")                   # b / 8
    a(f"s_add_u32 {sr(S_T2)}, {sr(S_E1)}, 1")
    a(f"s_mul_i32 {sr(S_Q)}, {sr(S_T0)}, {sr(S_T2)}")       # xcd (q + 1)
    a(f"s_mul_i32 {sr(dst)}, {sr(S_R)}, {sr(S_T2)}")        # r (q + 1)
    a(f"s_sub_u32 {sr(S_T2)}, {sr(S_T0)}, {sr(S_R)}")
    a(f"s_mul_i32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_E1)}")
    a(f"s_add_u32 {sr(dst)}, {sr(dst)}, {sr(S_T2)}")
    a(f"s_cmp_lt_u32 {sr(S_T0)}, {sr(S_R)}")
    a(f"s_cselect_b32 {sr(dst)}, {sr(S_Q)}, {sr(dst)}")
    a(f"s_add_u32 {sr(dst)}, {sr(dst)}, {sr(S_T1)}")


def dma_pieces(half: str) -> tuple[int, int, int, int]:
    return (SRD_A, V_DA, S_SOA, S_M0A) if half == "a" else (SRD_B, V_DB, S_SOB, S_M0B)


def prologue_dma(a: Asm, half: str):
    srd_, vo, so, m0 = dma_pieces(half)
    a(f"s_mov_b32 m0, {sr(m0)}")
    a("s_nop 0")
    for j in range(8):
        soff = "0" if j == 0 else sr(so + j - 1)
        a(f"buffer_load_dwordx4 {vr(vo)}, {sr(srd_, 4)}, {soff} offen lds")
        if j < 7:
            a(f"s_add_u32 m0, m0, {blockbase(j + 1) - blockbase(j)}")
            a("s_nop 0")


def advance(half: str) -> list[str]:
    srd_ = SRD_A if half == "a" else SRD_B
    adv = S_ADVA if half == "a" else S_ADVB
    return [f"s_add_u32 {sr(srd_)}, {sr(srd_)}, {sr(adv)}", f"s_addc_u32 {sr(srd_ + 1)}, {sr(srd_ + 1)}, 0"]


def frag_reads(kind: str, f: int, sub: int) -> list[str]:
    lo, hi = (V_RALO, V_RAHI) if kind == "a" else (V_RBLO, V_RBHI)
    dst = ((V_FA0 if sub == 0 else V_FA1) if kind == "a" else (V_FB0 if sub == 0 else V_FB1)) + 4 * f
    off = 64 * f + SUB1 * sub
    return [f"ds_read_b64_tr_b16 {vr(dst, 2)}, {vr(lo)} offset:{off}",
            f"ds_read_b64_tr_b16 {vr(dst + 2, 2)}, {vr(hi)} offset:{off}"]


def mfma(i: int, j: int, sub: int) -> str:
    """acc[i][j] += B_j (srcA: n) x A_i (srcB: m): the lane holds 4
    consecutive n of one row m."""
    fa = (V_FA0 if sub == 0 else V_FA1) + 4 * i
    fb = (V_FB0 if sub == 0 else V_FB1) + 4 * j
    acc = 4 * (8 * i + j)
    return f"v_mfma_f32_16x16x32_bf16 {ar(acc, 4)}, {vr(fb, 4)}, {vr(fa, 4)}, {ar(acc, 4)}"


def iteration(a: Asm, with_dma: bool, next_reads: bool):
    """One 64-row (t) tile on the forward kernel's slot map (the same keys:
    split / m0_lag / adv, gemm_gen.iteration_map)."""
    m = G.SLOT_MAPS[KNOBS["map"]]
    split, lag = m.get("split", 0), m.get("m0_lag", 0)
    slots: dict[int, list[str]] = {n: [] for n in range(128)}
    for j, n in enumerate(m["x1"]):
        slots[n] += frag_reads("a", j, 1)
    for i, n in enumerate(m["w1"]):
        slots[n] += frag_reads("b", i, 1)
    vm = 0
    if with_dma:
        for bar in (m["xbar"], m["wbar"]):
            slots[bar].append("s_waitcnt lgkmcnt(0)")
            slots[bar + split].append("s_barrier")
        for half, key, bar in (("a", "xdma", m["xbar"]), ("b", "wdma", m["wbar"])):
            srd_, vo, so, m0 = dma_pieces(half)
            p = m[key]
            assert p[0] > bar + split
            slots[p[0] - 1].append(f"s_mov_b32 m0, {sr(m0)}")
            for j, n in enumerate(p):
                soff = "0" if j == 0 else sr(so + j - 1)
                slots[n].append(f"buffer_load_dwordx4 {vr(vo)}, {sr(srd_, 4)}, {soff} offen lds")
                if j < 7:
                    assert p[j + 1] > n + lag
                    slots[n + lag].append(f"s_add_u32 m0, m0, {blockbase(j + 1) - blockbase(j)}")
            adv = m.get("adv", {}).get("x" if half == "a" else "w", p[-1])
            slots[adv] += advance(half) + [f"s_xor_b32 {sr(m0)}, {sr(m0)}, {sr(m0 + 1)}"]
        vm = sum(1 for n in m["xdma"] + m["wdma"] if n < m["wait"])
    if next_reads:
        w = m["wait"]
        slots[w].append(f"s_waitcnt vmcnt({vm})")
        slots[w + split] += ["s_barrier"] + [
            f"v_xor_b32 {vr(b)}, {vr(b)}, {vr(t)}" for b, t in ((V_RALO, V_TGALO), (V_RAHI, V_TGAHI),
                                                                  (V_RBLO, V_TGBLO), (V_RBHI, V_TGBHI))]
        assert min(m["x0"] + m["w0"]) > w + split
        for j, n in enumerate(m["x0"]):
            slots[n] += frag_reads("a", j, 0)
        for i, n in enumerate(m["w0"]):
            slots[n] += frag_reads("b", i, 0)
        slots[126].append("s_waitcnt lgkmcnt(0)")
    for n in range(128):
        sub, mm = divmod(n, 64)
        i, j = divmod(mm, 8)
        if n == 64:
            a("s_waitcnt lgkmcnt(0)")
        a(".p2alignl 3, 0xbf800000")
        a(mfma(i, j, sub))
        for ins in slots[n]:
            a(ins)


def epilogue(a: Asm):
    """Per (i, j): 4 fp32 of row m, columns n .. n+3.  Whole-K tiles: bf16,
    C (+)= (beta); k-pieces: fp32 partials into the workspace tile."""
    v = V_T
    a(f"v_lshrrev_b32 {vr(v)}, 6, {vr(V_TID)}")              # w
    a(f"v_and_b32 {vr(v + 1)}, 63, {vr(V_TID)}")             # lane
    a(f"v_and_b32 {vr(v + 2)}, 15, {vr(v + 1)}")             # row in fragment
    a(f"v_and_b32 {vr(v + 3)}, 1, {vr(v)}")                  # wm
    a(f"v_lshl_add_u32 {vr(v + 2)}, {vr(v + 3)}, 7, {vr(v + 2)}")   # m_local
    a(f"v_lshrrev_b32 {vr(v + 1)}, 4, {vr(v + 1)}")          # lane >> 4
    a(f"v_lshrrev_b32 {vr(v)}, 1, {vr(v)}")                  # wn
    a(f"v_lshl_add_u32 {vr(v + 1)}, {vr(v)}, 5, {vr(v + 1)}")   # n_local / 4
    # V_E: C byte offset (m_local ldc + 8 (n_local / 4)); V_E+1: WS byte offset
    a(f"v_mul_lo_u32 {vr(V_E)}, {vr(v + 2)}, {sr(S_LDC)}")
    a(f"v_lshl_add_u32 {vr(V_E)}, {vr(v + 1)}, 3, {vr(V_E)}")
    a(f"v_lshlrev_b32 {vr(V_E + 1)}, 10, {vr(v + 2)}")        # m_local * 1024
    a(f"v_lshl_add_u32 {vr(V_E + 1)}, {vr(v + 1)}, 4, {vr(V_E + 1)}")
    l_piece, l_end = a.fresh("epi_piece"), a.fresh("epi_end")
    a(f"s_cmp_eq_u32 {sr(S_PIECE)}, 1")
    a(f"s_cbranch_scc1 {l_piece}")
    # --- bf16 into C, beta = 0 or 1
    l_nobeta = a.fresh("nobeta")
    a(f"s_lshl_b32 {sr(S_E1)}, {sr(S_LDC)}, 4")             # 16 rows
    a(f"s_mov_b32 {sr(S_E0)}, 0")
    for r in range(4):
        a(f"v_mov_b32 {vr(V_SQ + r)}, 0")
    for i in range(8):
        # pk alternates between two register sets and nothing waits for the
        # stores (the TN epilogue re-uses its store registers at once: the
        # data is read at issue); a row block's stores drain under the next
        f, pk, old = V_E + 8, V_E + 40 + 16 * (i & 1), V_E + 72
        for j in range(8):
            G.read_acc4(a, f + 4 * j, 4 * (8 * i + j))
        a(f"s_cmp_eq_u32 {sr(S_BETA)}, 0")
        a(f"s_cbranch_scc1 {l_nobeta}_{i}")
        for j in range(8):
            a(f"buffer_load_dwordx2 {vr(old + 2 * j, 2)}, {vr(V_E)}, {sr(SRD_C, 4)}, {sr(S_E0)} offen offset:{32 * j}")
        a("s_waitcnt vmcnt(0)")
        for j in range(8):
            G.unpack_bf16(a, V_E + 88, old + 2 * j)
            for r in range(4):
                a(f"v_add_f32 {vr(f + 4 * j + r)}, {vr(f + 4 * j + r)}, {vr(V_E + 88 + r)}")
        a.label(f"{l_nobeta}_{i}")
        # the gradient-norm partials: squares of the tile's final fp32 values
        # (four chains; the clipping norm of train/llm.py, ops/gemm.SumsqSession)
        for j in range(8):
            for r in range(4):
                a(f"v_fma_f32 {vr(V_SQ + r)}, {vr(f + 4 * j + r)}, {vr(f + 4 * j + r)}, {vr(V_SQ + r)}")
        for j in range(8):
            G.cvt_pack(a, pk + 2 * j, f + 4 * j)
        for j in range(8):
            a(f"buffer_store_dwordx2 {vr(pk + 2 * j, 2)}, {vr(V_E)}, {sr(SRD_C, 4)}, {sr(S_E0)} offen offset:{32 * j}")
        a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_E1)}")
    sumsq_store(a)
    a(f"s_branch {l_end}")
    # --- fp32 partials into the workspace tile (256 x 256 x 4 B, row-major)
    a.label(l_piece)
    a(f"s_mov_b32 {sr(S_E0)}, 0")
    for i in range(8):
        f = V_E + 8 + 32 * (i & 1)                           # two sets, as pk above
        for j in range(8):
            G.read_acc4(a, f + 4 * j, 4 * (8 * i + j))
        for j in range(8):
            a(f"buffer_store_dwordx4 {vr(f + 4 * j, 4)}, {vr(V_E + 1)}, {sr(SRD_WS, 4)}, {sr(S_E0)} offen offset:{64 * j}")
        a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {16 * 1024}")
    a.label(l_end)


def sumsq_store(a: Asm):
    """Whole-K tiles with a partials buffer (kernarg "sq" != 0): lane l of wave
    w stores its sum of squares at float (tm tiles_n + tn) 256 + 64 w + l --
    a slot per tile independent of the tile order, so the host's sum over the
    buffer is deterministic.  The k-piece tiles' slots are written by
    wgrad_tile_reduce_kernel (csrc/hip/wgrad.hip)."""
    l_do, l_skip = a.fresh("sq_do"), a.fresh("sq_skip")
    a(f"s_cmp_lg_u32 {sr(SRD_SQ)}, 0")
    a(f"s_cbranch_scc1 {l_do}")
    a(f"s_cmp_lg_u32 {sr(SRD_SQ + 1)}, 0")
    a(f"s_cbranch_scc0 {l_skip}")
    a.label(l_do)
    a(f"v_add_f32 {vr(V_SQ)}, {vr(V_SQ)}, {vr(V_SQ + 1)}")
    a(f"v_add_f32 {vr(V_SQ + 2)}, {vr(V_SQ + 2)}, {vr(V_SQ + 3)}")
    a(f"v_add_f32 {vr(V_SQ)}, {vr(V_SQ)}, {vr(V_SQ + 2)}")
    a(f"s_mul_i32 {sr(S_T0)}, {sr(S_TM)}, {sr(S_TN_N)}")
    a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_TN)}")
    a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_T0)}, 10")          # 256 floats per tile
    a(f"s_mul_i32 {sr(SRD_SQ + 2)}, {sr(S_TM_N)}, {sr(S_TN_N)}")
    a(f"s_lshl_b32 {sr(SRD_SQ + 2)}, {sr(SRD_SQ + 2)}, 10")   # num_records: the whole buffer
    a(f"s_mov_b32 {sr(SRD_SQ + 3)}, 0x20000")
    a(f"v_lshlrev_b32 {vr(V_SQ + 1)}, 2, {vr(V_TID)}")
    a(f"buffer_store_dword {vr(V_SQ)}, {vr(V_SQ + 1)}, {sr(SRD_SQ, 4)}, {sr(S_T0)} offen")
    a.label(l_skip)


def kernel(variant: str = "") -> tuple[str, str]:
    name = "toa_wgrad_nt_asm" + (f"_{variant}" if variant else "")
    a = Asm(prefix="nt_" + (variant + "_" if variant else ""))
    a.raw(f".globl {name}")
    a.raw(".p2align 8")
    a.raw(f".type {name},@function")
    a.raw(f"{name}:")
    prologue(a)
    for half in ("a", "b"):                     # tile 0 -> stage 0
        prologue_dma(a, half)
        for ins in advance(half):
            a(ins)
    a(f"s_xor_b32 {sr(S_M0A)}, {sr(S_M0A)}, {sr(S_M0AT)}")
    a(f"s_xor_b32 {sr(S_M0B)}, {sr(S_M0B)}, {sr(S_M0BT)}")
    for half in ("a", "b"):                     # tile 1 -> stage 1
        prologue_dma(a, half)
        for ins in advance(half):
            a(ins)
    a(f"s_xor_b32 {sr(S_M0A)}, {sr(S_M0A)}, {sr(S_M0AT)}")
    a(f"s_xor_b32 {sr(S_M0B)}, {sr(S_M0B)}, {sr(S_M0BT)}")
    if KNOBS["zero_late"]:
        zero_acc(a)                             # under the first tiles' DMA flight
    a("s_waitcnt vmcnt(16)")                    # own tile-0 pieces
    a("s_barrier")
    for j in range(8):
        for ins in frag_reads("a", j, 0):
            a(ins)
    for i in range(8):
        for ins in frag_reads("b", i, 0):
            a(ins)
    a("s_waitcnt lgkmcnt(0)")
    a(f"s_sub_u32 {sr(S_LOOP)}, {sr(S_KTP)}, 2")
    l_loop, l_tail = a.fresh("loop"), a.fresh("tail")
    a(f"s_cmp_eq_u32 {sr(S_LOOP)}, 0")
    a(f"s_cbranch_scc1 {l_tail}")
    a(".p2alignl 6, 0xbf800000")
    a.label(l_loop)
    iteration(a, with_dma=True, next_reads=True)
    a(f"s_sub_u32 {sr(S_LOOP)}, {sr(S_LOOP)}, 1")
    a(f"s_cmp_eq_u32 {sr(S_LOOP)}, 0")
    a(f"s_cbranch_scc0 {l_loop}")
    a.label(l_tail)
    iteration(a, with_dma=False, next_reads=True)
    iteration(a, with_dma=False, next_reads=False)
    a("s_nop 15")
    a("s_nop 15")
    epilogue(a)
    a.label(a.abort)
    a("s_endpgm")
    a.raw(f".size {name}, .-{name}")
    desc, meta = G._descriptor(name, lds_bytes=LDS_BYTES, n_sgpr=N_SGPR)
    return "\n".join(a.out) + "\n" + desc, meta


def generate() -> str:
    body, meta = kernel()
    parts = ['.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', ".amdhsa_code_object_version 5", ".text", body,
             ".text\n.p2alignl 6, 3212836864\n.fill 256, 4, 3212836864",
             ".amdgpu_metadata\n---\namdhsa.version:\n  - 1\n  - 2\namdhsa.target: amdgcn-amd-amdhsa--gfx950\n"
             "amdhsa.kernels:\n" + meta + "...\n.end_amdgpu_metadata"]
    return "\n".join(parts) + "\n"


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else "wgrad_nt_asm.s"
    with open(out, "w") as f:
        f.write(generate())
