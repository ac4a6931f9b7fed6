#!/usr/bin/env python3
"""Generator of the hand-written gfx950 (CDNA4) assembly GEMM kernels.

    python csrc/asm/gemm_gen.py OUT.s

Emits one code object source with the forward / data-gradient GEMM of the
training step in the "TN" form (both operands contiguous along the
reduction), written instruction by instruction rather than through hipcc:

    C[m][n] = sum_k X[m][k] * W[n][k]      bf16 in, fp32 accumulate

Why assembly: the one-wave-per-SIMD schedule that gives the lowest energy
per MFMA (128 x 128 of C per wave, a third fewer LDS bytes per MFMA than
128 x 64) needs its latency hidden by software pipelining -- fragment reads
for the next k-step issued between the current k-step's MFMAs, the global
prefetch two tiles ahead, accumulators that never leave the AGPRs.  hipcc
did not hold that schedule (round 3: `gemm_tn4w_kernel` shuttled
accumulators and waited `vmcnt(0)`, 0.96-1.02 PF/s; docs/kernels.md).

Structure (every number below is what the generator emits):

  workgroup   256 threads = 4 waves (one per SIMD), tile 256 x 256, BK = 64
  wave        (wm, wn) = (wave & 1, wave >> 1): 128 rows of X x 128 rows of W
              = 8 x 8 tiles of v_mfma_f32_16x16x32_bf16, 256 AGPR accumulators
  LDS         two stages of 66 KiB (X half, W half).  A half is 32 "lines" of
              1056 B (1024 B of data + 32 B pad): line i of the wave-row block
              holds tile rows i, i+16, ..., i+112 (128 B = 64 k each).  A
              fragment read (ds_read_b128: lane l reads line l & 15, 16-B
              chunk l >> 4) is serviced in 4 lane groups of 16; with lines 264
              dwords = 8 banks apart every group covers the 64 banks once, 4
              LDS cycles per read (a 16-B pad, 4 banks apart, collides chunk 1
              of line i with chunk 0 of line i + 1 inside a group: 8 cycles)
  staging     LDS-DMA (`buffer_load_dwordx4 ... lds`): one instruction per
              wave fills one line = 8 rows x 128 B (8 whole cache lines), the
              swizzle-free image needs no source permutation.  16 DMA
              instructions per wave per 64-k tile, bounded by the buffer
              resource (num_records): an address past the tensor reads 0
  pipeline    tile t+2 is staged into the stage tile t just vacated (two
              stages, prefetch distance two), k-step halves of 32:
                phase 1: 64 MFMAs on sub-step 0 fragments; between them the
                         sub-step 1 fragment reads of the same stage, then a
                         barrier per operand half after which that half's
                         DMA for tile t+2 starts
                phase 2: 64 MFMAs on sub-step 1; the rest of the DMA, one
                         counted vmcnt (tile t+1 landed) + barrier, then the
                         next tile's sub-step 0 fragment reads
              three barriers per 64-k tile, vmcnt never 0 inside the loop
  epilogue    accumulators -> bf16 (v_cvt_pk_bf16_f32) -> buffer stores, each
              lane 4 consecutive columns of one row (the W fragment is the
              MFMA's A operand); fused variants:
                plain        C
                swiglu_fwd   gate|up projection: the workgroup's 256 W rows are
                             128 gate rows and the SAME 128 up rows (W keeps
                             its [gate; up] layout); writes gu and
                             s = silu(gate) * up
                swiglu_bwd   down-projection data gradient: ds is never stored;
                             reads gu, writes dgu = [ds*up*silu'(g) | ds*silu(g)]
  grid        one workgroup per tile, XCD-aware: the 8 XCDs get contiguous
              ranges of the tile order, which walks groups of 8 row tiles
              across the column tiles (a group's X strips + the current W
              strip stay in the XCD's L2)

Reference anchor: SURVEY.md K1/K2/K19 and section 7.1 item 5 (MFMA tiles with
fused epilogues); the reference itself has no kernels
(/root/reference/examples/v1/dist-mnist/dist_mnist.py:188-189 is the GEMM +
bias + activation these generalise).  This file is not derived from any
library source: the schedule class (4 waves x 128 x 128, prefetch distance
two) is the one docs/kernels.md and profiles/r3_tn_pmc measured as the
energy-efficient form on MI355X.
"""
from __future__ import annotations

import sys

LINE = 1056              # one LDS line: 8 tile rows x 128 B + 32 B pad
HALF = 32 * LINE         # 256 rows of one operand = 33792 B
STAGE = 2 * HALF         # X half + W half = 67584 B
LDS_BYTES = 2 * STAGE    # 135168 B
KARG_BYTES = 96

# kernarg layout (byte offsets; mirrored by csrc/hip/gemm_asm.hip).  `map`:
# the tile order, bits [3:0] log2 of the group size, bit 4 set = groups of
# COLUMN tiles walk the row tiles (clear: groups of row tiles walk the
# column tiles); `grid`: a persistent kernel's workgroup count.
KARG = {
    "X": 0, "W": 8, "C": 16, "S": 24,
    "ldx": 32, "ldw": 36, "ldc": 40, "lds": 44,
    "ktiles": 48, "tiles_m": 52, "tiles_n": 56, "xq": 60, "xr": 64,
    "per_group": 68, "fw": 72, "fc": 76, "map": 80, "grid": 84, "phase": 88,
}
MAP_WALK_COLS = 16
MAP_DEFAULT = 2          # groups of 4 row tiles walk the column tiles

EPIS = ("plain", "swiglu_fwd", "swiglu_bwd", "rope", "delta", "resadd")

# ---------------------------------------------------------------- registers
# SGPRs: s[0:1] kernarg pointer, s2 workgroup id (the descriptor's order)
S_ARGS = 4          # s[4:23]: the 80 B of kernarg
S_X, S_W, S_C, S_S = 4, 6, 8, 10
S_LDX, S_LDW, S_LDC, S_LDS = 12, 13, 14, 15
S_KT, S_TM_N, S_TN_N, S_XQ = 16, 17, 18, 19
S_XR, S_PG, S_FW, S_FC = 20, 21, 22, 23
S_TILE, S_TM, S_TN = 24, 25, 26
S_T0, S_T1, S_T2, S_T3 = 27, 28, 29, 30
S_PHASE = 31        # kernarg `phase` word (start offsets of the first wave, phase_delay)
SRD_X, SRD_W, SRD_C, SRD_S = 32, 36, 40, 44
S_M0X, S_M0XT, S_M0W, S_M0WT = 48, 49, 50, 51
S_LOOP = 52
S_SOX = 53          # s53..s59: X DMA row offsets, instructions 1..7
S_SOW = 60          # s60..s66: W DMA row offsets
S_E0, S_E1 = 67, 68  # epilogue scratch
S_Q, S_R = 69, 70   # division results
# timing kernel: s72..s83 six
# s_memtime stamps (aligned pairs), s84..s86 accumulated waits (vm, X-free
# barrier, W-free barrier), s88..s89 the kernel's start stamp
S_TMT, S_ACC, S_T_START = 72, 84, 88
S_ITER, S_GRID = 90, 91   # persistent arms: this workgroup's tile-order index, the grid size
# deferred-store arm (SCHED "defer", never with the timing kernel, whose stamps
# use s72..s89): the previous tile's C resource, its row-block offset and step
SRD_D, S_DOFF, S_DSTEP = 72, 76, 77
S_MAP, S_KGRID = 92, 93   # kernarg map / grid words (s94, s95: the map's decoded log2 group, walk flag)
S_LG, S_WALK = 94, 95
N_SGPR = 96

# VGPRs
V_TID = 132
V_DX, V_DW = 1, 133        # DMA lane offsets (bytes)
V_RX, V_RW = 2, 3          # LDS fragment-read bases
V_RXT, V_RWT = 134, 135    # stage toggles (xor masks)
V_FX0, V_FX1 = 4, 36       # X fragments, sub-steps 0 / 1 (8 x 4 VGPRs each)
V_FW0, V_FW1 = 68, 100     # W fragments
V_T = 136                  # 136..139 scratch
V_E = 140                  # 140..255 epilogue scratch

UNIT_GATE_ROWS = 64        # swiglu_fwd: W rows per wave column per half


class Asm:
    def __init__(self, prefix: str = ""):
        self.out: list[str] = []
        self.nlab = 0
        self.prefix = prefix
        self.abort = f"L_{prefix}abort"
        self.stage_exit = f"L_{prefix}stage_exit"

    def __call__(self, s: str):
        self.out.append("  " + s)

    def label(self, name: str):
        self.out.append(name + ":")

    def fresh(self, stem: str) -> str:
        self.nlab += 1
        return f"L_{self.prefix}{stem}_{self.nlab}"

    def raw(self, s: str):
        self.out.append(s)


def vr(base: int, n: int = 1) -> str:
    return f"v{base}" if n == 1 else f"v[{base}:{base + n - 1}]"


def sr(base: int, n: int = 1) -> str:
    return f"s{base}" if n == 1 else f"s[{base}:{base + n - 1}]"


def ar(base: int, n: int = 1) -> str:
    return f"a{base}" if n == 1 else f"a[{base}:{base + n - 1}]"


# ---------------------------------------------------------------- helpers
def udiv(a: Asm, q: int, r: int, num: int, den: int):
    """s_q = s_num / s_den, s_r = s_num % s_den (unsigned, both < 2^24):
    float reciprocal estimate on the VALU, then one exact correction step
    each way on the SALU."""
    # Explicit wait states (hipcc inserts these; hand-written code must):
    # a transcendental's result forwarded to the next VALU, and a VALU
    # result read by v_readfirstlane, both need padding on gfx950 -- without
    # the second, v_readfirstlane returned the PRE-conversion float bits
    # (measured: tile coordinate 0x3fc00000 = 1.5 for 3 / 2; the probe kernel).
    a(f"v_cvt_f32_u32 {vr(V_T)}, {sr(den)}")
    a(f"v_cvt_f32_u32 {vr(V_T + 1)}, {sr(num)}")
    a("s_nop 4")
    a(f"v_rcp_iflag_f32 {vr(V_T)}, {vr(V_T)}")
    a("s_nop 4")
    a(f"v_mul_f32 {vr(V_T)}, {vr(V_T)}, {vr(V_T + 1)}")
    a("s_nop 4")
    a(f"v_cvt_u32_f32 {vr(V_T)}, {vr(V_T)}")
    a("s_nop 4")
    a(f"v_readfirstlane_b32 {sr(q)}, {vr(V_T)}")
    a("s_nop 4")
    a(f"s_mul_i32 {sr(r)}, {sr(q)}, {sr(den)}")
    a(f"s_sub_i32 {sr(r)}, {sr(num)}, {sr(r)}")
    l1, l2 = a.fresh("div"), a.fresh("div")
    a(f"s_cmp_lt_i32 {sr(r)}, 0")
    a(f"s_cbranch_scc0 {l1}")
    a(f"s_sub_u32 {sr(q)}, {sr(q)}, 1")
    a(f"s_add_u32 {sr(r)}, {sr(r)}, {sr(den)}")
    a.label(l1)
    a(f"s_cmp_ge_u32 {sr(r)}, {sr(den)}")
    a(f"s_cbranch_scc0 {l2}")
    a(f"s_add_u32 {sr(q)}, {sr(q)}, 1")
    a(f"s_sub_u32 {sr(r)}, {sr(r)}, {sr(den)}")
    a.label(l2)


def srd(a: Asm, dst: int, base_lo: int, off_lo: int, off_hi: int, nrec: int):
    """dst[0:3] = buffer resource at 64-bit s[base] + (off_hi:off_lo),
    num_records s[nrec] bytes, raw (stride 0), 32-bit dword data format."""
    a(f"s_add_u32 {sr(dst)}, {sr(base_lo)}, {sr(off_lo)}")
    a(f"s_addc_u32 {sr(dst + 1)}, {sr(base_lo + 1)}, {sr(off_hi)}")
    a(f"s_mov_b32 {sr(dst + 2)}, {sr(nrec)}")
    a(f"s_mov_b32 {sr(dst + 3)}, 0x20000")


def mul64(a: Asm, lo: int, hi: int, x: int, y: int):
    """(s_hi:s_lo) = s_x * s_y (unsigned 32 x 32 -> 64)."""
    a(f"s_mul_hi_u32 {sr(hi)}, {sr(x)}, {sr(y)}")
    a(f"s_mul_i32 {sr(lo)}, {sr(x)}, {sr(y)}")


# ---------------------------------------------------------------- prologue
def prologue_args(a: Asm, epi: str = "plain"):
    a(f"s_load_dwordx16 {sr(S_ARGS, 16)}, s[0:1], 0x0")
    a(f"s_load_dwordx4 {sr(S_ARGS + 16, 4)}, s[0:1], 0x40")
    a(f"s_load_dwordx2 {sr(S_MAP, 2)}, s[0:1], 0x50")
    a(f"s_load_dword {sr(S_PHASE)}, s[0:1], {KARG['phase']:#x}")
    a("s_mov_b32 m0, 0")
    a(f"v_mov_b32 {vr(V_TID)}, v0")
    a("s_waitcnt lgkmcnt(0)")
    # defensive: an argument block the host launcher never packs ends the
    # workgroup before any memory access (2 <= ktiles <= 65536, s2 < nwg)
    a(f"s_cmp_lt_u32 {sr(S_KT)}, 2")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_cmp_gt_u32 {sr(S_KT)}, 65536")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_mul_i32 {sr(S_T0)}, {sr(S_TM_N)}, {sr(S_TN_N)}")
    a(f"s_cmp_ge_u32 s2, {sr(S_T0)}")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_lshl_b32 {sr(S_T1)}, {sr(S_XQ)}, 3")
    a(f"s_add_u32 {sr(S_T1)}, {sr(S_T1)}, {sr(S_XR)}")
    a(f"s_cmp_lg_u32 {sr(S_T1)}, {sr(S_T0)}")
    a(f"s_cbranch_scc1 {a.abort}")
    # tile order: log2 group <= 6, nothing above the walk bit
    a(f"s_and_b32 {sr(S_LG)}, {sr(S_MAP)}, 15")
    a(f"s_cmp_gt_u32 {sr(S_LG)}, 6")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_cmp_ge_u32 {sr(S_MAP)}, {2 * MAP_WALK_COLS}")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_lshr_b32 {sr(S_WALK)}, {sr(S_MAP)}, 4")
    if epi != "delta":      # (its kernarg bytes 88..95 are the delta pointer, not a phase word)
        phase_delay(a)
    if SCHED["persist"]:
        # persistent: the grid size; 0 would walk one tile forever
        a(f"s_cmp_eq_u32 {sr(S_KGRID)}, 0")
        a(f"s_cbranch_scc1 {a.abort}")
        a(f"s_mov_b32 {sr(S_GRID)}, {sr(S_KGRID)}")
        a(f"s_mov_b32 {sr(S_ITER)}, s2")


PHASE_FIRST_WAVE = 256   # workgroups 0..255: the first one on each of the 256 CUs


def phase_delay(a: Asm):
    """Start offsets for the first wave of workgroups (kernarg `phase`:
    bits [15:0] n, bits [19:16] log2 g; 0 = off).  Every tile of these
    kernels takes the same time, so the 256 workgroups that start together
    keep finishing together, and their epilogues -- a burst of HBM traffic
    with the MFMA pipe idle (the SwiGLU backward loads 256 KiB of gate / up
    and stores 256 KiB per tile) -- all hit memory at once.  Workgroup b of
    the first wave sleeps ((b >> 3) mod g) * n * 512 cycles before its
    prologue: its CU then runs g phase groups apart for the rest of the
    kernel (the next workgroups are dispatched to whichever CU frees first),
    so each epilogue burst meets 1/g of the chip's traffic.  (b >> 3: the
    dispatcher deals workgroups round-robin over the 8 XCDs, so every XCD
    gets every phase.)"""
    l_done, l_sleep = a.fresh("phase_done"), a.fresh("phase_sleep")
    a(f"s_cmp_ge_u32 s2, {PHASE_FIRST_WAVE}")
    a(f"s_cbranch_scc1 {l_done}")
    a(f"s_and_b32 {sr(S_T0)}, {sr(S_PHASE)}, 0xffff")            # n
    a(f"s_lshr_b32 {sr(S_T1)}, {sr(S_PHASE)}, 16")
    a(f"s_and_b32 {sr(S_T1)}, {sr(S_T1)}, 15")                   # log2 g
    a(f"s_lshl_b32 {sr(S_T2)}, 1, {sr(S_T1)}")
    a(f"s_sub_u32 {sr(S_T2)}, {sr(S_T2)}, 1")
    a(f"s_lshr_b32 {sr(S_T3)}, s2, 3")
    a(f"s_and_b32 {sr(S_T3)}, {sr(S_T3)}, {sr(S_T2)}")           # phase group
    a(f"s_mul_i32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_T3)}")           # sleeps of 512 cycles
    a.label(l_sleep)
    a(f"s_cmp_eq_u32 {sr(S_T0)}, 0")
    a(f"s_cbranch_scc1 {l_done}")
    a("s_sleep 8")
    a(f"s_sub_u32 {sr(S_T0)}, {sr(S_T0)}, 1")
    a(f"s_branch {l_sleep}")
    a.label(l_done)


def tile_setup(a: Asm, epi: str, bid: str = "s2"):
    """Tile of block `bid` -> S_TILE, (S_TM, S_TN), SRD_X / SRD_W."""
    # --- XCD remap: blocks b, b+8, ... share an XCD; give each XCD a
    # contiguous range of the tile order (bijective for any nwg)
    a(f"s_and_b32 {sr(S_T0)}, {bid}, 7")              # xcd
    a(f"s_lshr_b32 {sr(S_T1)}, {bid}, 3")             # b / 8
    a(f"s_add_u32 {sr(S_T2)}, {sr(S_XQ)}, 1")         # q + 1
    a(f"s_mul_i32 {sr(S_T3)}, {sr(S_T0)}, {sr(S_T2)}")  # xcd * (q+1)
    a(f"s_mul_i32 {sr(S_TILE)}, {sr(S_XR)}, {sr(S_T2)}")  # r * (q+1)
    a(f"s_sub_u32 {sr(S_T2)}, {sr(S_T0)}, {sr(S_XR)}")  # xcd - r
    a(f"s_mul_i32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_XQ)}")  # (xcd - r) * q
    a(f"s_add_u32 {sr(S_TILE)}, {sr(S_TILE)}, {sr(S_T2)}")
    a(f"s_cmp_lt_u32 {sr(S_T0)}, {sr(S_XR)}")
    a(f"s_cselect_b32 {sr(S_TILE)}, {sr(S_T3)}, {sr(S_TILE)}")
    a(f"s_add_u32 {sr(S_TILE)}, {sr(S_TILE)}, {sr(S_T1)}")
    # --- tile -> (tm, tn) by the kernarg map: groups of 2^lg tiles of the
    # grouped dimension (rows; columns when the walk bit is set) walk the
    # other dimension's tiles.  A = grouped tile count (S_E0), B = walked (S_E1)
    a(f"s_cmp_eq_u32 {sr(S_WALK)}, 0")
    a(f"s_cselect_b32 {sr(S_E0)}, {sr(S_TM_N)}, {sr(S_TN_N)}")
    a(f"s_cselect_b32 {sr(S_E1)}, {sr(S_TN_N)}, {sr(S_TM_N)}")
    a(f"s_lshl_b32 {sr(S_PG)}, {sr(S_E1)}, {sr(S_LG)}")   # tiles per group (the kernarg's is not used)
    udiv(a, S_Q, S_R, S_TILE, S_PG)                     # group, within
    a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_Q)}, {sr(S_LG)}")  # first tile of the group
    a(f"s_sub_u32 {sr(S_T1)}, {sr(S_E0)}, {sr(S_T0)}")
    a(f"s_lshl_b32 {sr(S_T2)}, 1, {sr(S_LG)}")
    a(f"s_min_u32 {sr(S_T1)}, {sr(S_T1)}, {sr(S_T2)}")  # gsz
    a(f"s_mov_b32 {sr(S_T2)}, {sr(S_R)}")
    udiv(a, S_Q, S_R, S_T2, S_T1)                       # within / gsz, within % gsz
    a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_R)}")   # grouped-dimension tile
    a(f"s_cmp_eq_u32 {sr(S_WALK)}, 0")
    a(f"s_cselect_b32 {sr(S_TM)}, {sr(S_T0)}, {sr(S_Q)}")
    a(f"s_cselect_b32 {sr(S_TN)}, {sr(S_Q)}, {sr(S_T0)}")

    # --- buffer resources at the tile's first row / column
    # X: rows tm*256 .. +255, every k
    a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_TM)}, 8")
    mul64(a, S_T2, S_T3, S_T0, S_LDX)
    a(f"s_lshl_b32 {sr(S_T1)}, {sr(S_LDX)}, 8")       # 256 rows
    srd(a, SRD_X, S_X, S_T2, S_T3, S_T1)
    # W: rows tn*256 (tn*128 for the gate|up projection)
    a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_TN)}, {7 if epi == 'swiglu_fwd' else 8}")
    mul64(a, S_T2, S_T3, S_T0, S_LDW)
    a(f"s_lshl_b32 {sr(S_T1)}, {sr(S_LDW)}, 8")
    if epi == "swiglu_fwd":
        a(f"s_lshr_b32 {sr(S_T1)}, {sr(S_T1)}, 1")    # 128 rows of each half
        a(f"s_add_u32 {sr(S_T1)}, {sr(S_T1)}, {sr(S_FW)}")  # + the up half's offset
    srd(a, SRD_W, S_W, S_T2, S_T3, S_T1)


def tile_c(a: Asm, epi: str):
    """SRD_C (and SRD_S) of the tile at (S_TM, S_TN)."""
    # C (and S): rows tm*256, columns tn*256 (tn*128 for the gate|up epilogue)
    if SCHED["store_same"]:   # DIAGNOSTIC arm: every workgroup stores tile (0, 0)
        a(f"s_mov_b32 {sr(S_TM)}, 0")
        a(f"s_mov_b32 {sr(S_TN)}, 0")
    a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_TM)}, 8")
    mul64(a, S_T2, S_T3, S_T0, S_LDC)
    a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_TN)}, {8 if epi == 'swiglu_fwd' else 9}")  # column bytes
    a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_T0)}")
    a(f"s_addc_u32 {sr(S_T3)}, {sr(S_T3)}, 0")
    a(f"s_lshl_b32 {sr(S_T1)}, {sr(S_LDC)}, 8")
    srd(a, SRD_C, S_C, S_T2, S_T3, S_T1)
    if epi in ("delta", "resadd"):   # O / the residual: the same tile of a tensor laid out like C
        a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_TM)}, 8")
        mul64(a, S_T2, S_T3, S_T0, S_LDC)
        a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_TN)}, 9")
        a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_T0)}")
        a(f"s_addc_u32 {sr(S_T3)}, {sr(S_T3)}, 0")
        a(f"s_lshl_b32 {sr(S_T1)}, {sr(S_LDC)}, 8")
        srd(a, SRD_S, S_S, S_T2, S_T3, S_T1)
    if epi in ("swiglu_fwd", "swiglu_bwd"):
        a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_TM)}, 8")
        mul64(a, S_T2, S_T3, S_T0, S_LDS)
        a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_TN)}, {8 if epi == 'swiglu_fwd' else 9}")
        a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_T0)}")
        a(f"s_addc_u32 {sr(S_T3)}, {sr(S_T3)}, 0")
        a(f"s_lshl_b32 {sr(S_T1)}, {sr(S_LDS)}, 8")
        srd(a, SRD_S, S_S, S_T2, S_T3, S_T1)



def prologue(a: Asm, epi: str):
    prologue_args(a, epi)
    tile_setup(a, epi, sr(S_ITER) if SCHED["persist"] else "s2")
    tile_c(a, epi)
    prologue_lanes(a, epi)


def prologue_lanes(a: Asm, epi: str):
    # --- DMA lane offsets.  Wave w's instruction j fills LDS line w + 4j of
    # the half: rows (w + 4(j%4)) + 16*(lane>>3) [+ 128 for j >= 4], k chunk
    # lane & 7.  Per-lane part -> V_DX / V_DW, per-instruction part -> s[SO*].
    v = V_T
    a(f"v_lshrrev_b32 {vr(v)}, 6, {vr(V_TID)}")            # w
    a(f"v_and_b32 {vr(v + 1)}, 63, {vr(V_TID)}")           # lane
    a(f"v_lshrrev_b32 {vr(v + 2)}, 3, {vr(v + 1)}")        # lane >> 3
    a(f"v_and_b32 {vr(v + 3)}, 7, {vr(v + 1)}")            # lane & 7
    a(f"v_lshlrev_b32 {vr(v + 3)}, 4, {vr(v + 3)}")        # chunk bytes
    # X: row = w + 16 (lane >> 3)
    a(f"v_lshl_add_u32 {vr(V_DX)}, {vr(v + 2)}, 4, {vr(v)}")
    a(f"v_mul_lo_u32 {vr(V_DX)}, {vr(V_DX)}, {sr(S_LDX)}")
    a(f"v_add_u32 {vr(V_DX)}, {vr(V_DX)}, {vr(v + 3)}")
    # W: LDS row t = w + 4 jj + 16 q (q = lane >> 3) holds W row n(t) with
    # n = 32 (q >> 1) + 8 jj + 4 (q & 1) + w, so MFMA fragments 2p and 2p+1
    # give each lane 8 CONSECUTIVE output columns (16-byte epilogue stores).
    # SwiGLU: the same within each 64-row half, q & 3 in place of q, the up
    # half (q >> 2) F rows further.
    qq = v + 2
    a(f"v_and_b32 {vr(V_DW)}, {3 if epi == 'swiglu_fwd' else 7}, {vr(qq)}")
    a(f"v_lshrrev_b32 {vr(V_DW)}, 1, {vr(V_DW)}")                 # (q[&3]) >> 1
    a(f"v_lshlrev_b32 {vr(V_DW)}, 5, {vr(V_DW)}")                 # 32 (q >> 1)
    a(f"v_add_u32 {vr(V_DW)}, {vr(V_DW)}, {vr(v)}")               # + w
    a(f"v_and_b32 {vr(V_E)}, 1, {vr(qq)}")                        # q & 1
    a(f"v_lshl_add_u32 {vr(V_DW)}, {vr(V_E)}, 2, {vr(V_DW)}")     # + 4 (q & 1)
    a(f"v_mul_lo_u32 {vr(V_DW)}, {vr(V_DW)}, {sr(S_LDW)}")
    a(f"v_add_u32 {vr(V_DW)}, {vr(V_DW)}, {vr(v + 3)}")           # + chunk bytes
    if epi == "swiglu_fwd":
        a(f"v_lshrrev_b32 {vr(V_E)}, 2, {vr(qq)}")                # 0 / 1: gate / up
        a(f"v_mul_lo_u32 {vr(V_E)}, {vr(V_E)}, {sr(S_FW)}")
        a(f"v_add_u32 {vr(V_DW)}, {vr(V_DW)}, {vr(V_E)}")
    for j in range(1, 8):
        rows_x = 4 * (j % 4) + 128 * (j // 4)
        rows_w = 8 * (j % 4) + (UNIT_GATE_ROWS if epi == "swiglu_fwd" else 128) * (j // 4)
        a(f"s_mul_i32 {sr(S_SOX + j - 1)}, {sr(S_LDX)}, {rows_x}")
        a(f"s_mul_i32 {sr(S_SOW + j - 1)}, {sr(S_LDW)}, {rows_w}")
    # --- LDS-DMA bases (M0): wave w at line w of the stage's half
    a("s_nop 4")
    a(f"v_readfirstlane_b32 {sr(S_T0)}, {vr(v)}")          # w
    a("s_nop 4")
    a(f"s_mul_i32 {sr(S_M0X)}, {sr(S_T0)}, {LINE}")
    a(f"s_add_u32 {sr(S_M0XT)}, {sr(S_M0X)}, {STAGE}")
    a(f"s_xor_b32 {sr(S_M0XT)}, {sr(S_M0XT)}, {sr(S_M0X)}")
    a(f"s_add_u32 {sr(S_M0W)}, {sr(S_M0X)}, {HALF}")
    a(f"s_add_u32 {sr(S_M0WT)}, {sr(S_M0W)}, {STAGE}")
    a(f"s_xor_b32 {sr(S_M0WT)}, {sr(S_M0WT)}, {sr(S_M0W)}")
    # --- fragment read bases: line (lane & 15), chunk (lane >> 4), wave half
    a(f"v_and_b32 {vr(v + 2)}, 15, {vr(v + 1)}")
    a(f"v_mul_u32_u24 {vr(v + 2)}, {LINE}, {vr(v + 2)}")
    a(f"v_lshrrev_b32 {vr(v + 3)}, 4, {vr(v + 1)}")
    a(f"v_lshl_add_u32 {vr(v + 2)}, {vr(v + 3)}, 4, {vr(v + 2)}")
    a(f"v_and_b32 {vr(v + 3)}, 1, {vr(v)}")                # wm
    a(f"v_mul_u32_u24 {vr(v + 3)}, {16 * LINE}, {vr(v + 3)}")
    a(f"v_add_u32 {vr(V_RX)}, {vr(v + 2)}, {vr(v + 3)}")
    a(f"v_lshrrev_b32 {vr(v + 3)}, 1, {vr(v)}")            # wn
    a(f"v_mul_u32_u24 {vr(v + 3)}, {16 * LINE}, {vr(v + 3)}")
    a(f"v_add_u32 {vr(V_RW)}, {vr(v + 2)}, {vr(v + 3)}")
    a(f"v_add_u32 {vr(V_RW)}, {HALF}, {vr(V_RW)}")
    a(f"v_add_u32 {vr(V_RXT)}, {STAGE}, {vr(V_RX)}")
    a(f"v_xor_b32 {vr(V_RXT)}, {vr(V_RXT)}, {vr(V_RX)}")
    a(f"v_add_u32 {vr(V_RWT)}, {STAGE}, {vr(V_RW)}")
    a(f"v_xor_b32 {vr(V_RWT)}, {vr(V_RWT)}, {vr(V_RW)}")
    if not SCHED["zero_late"]:
        zero_acc(a)


def zero_acc(a: Asm):
    for i in range(256):
        a(f"v_accvgpr_write_b32 {ar(i)}, 0")


# ---------------------------------------------------------------- main loop
def dma(a: Asm, half: str, j: int) -> list[str]:
    """Instructions for DMA piece j (0..7) of the X or W half: set M0 to the
    line, one buffer_load_dwordx4 ... lds."""
    srd_, vo, so, m0 = (SRD_X, V_DX, S_SOX, S_M0X) if half == "x" else (SRD_W, V_DW, S_SOW, S_M0W)
    out = []
    if j == 0:
        out.append(f"s_mov_b32 m0, {sr(m0)}")
    else:
        out.append(f"s_add_u32 m0, m0, {4 * LINE}")
    # gfx9 hazard: an LDS-DMA reads M0 one wait state after the SALU write
    # (LLVM's checkReadM0Hazards; hipcc always separates the two)
    out.append("s_nop 0")
    soff = "0" if j == 0 else sr(so + j - 1)
    out.append(f"buffer_load_dwordx4 {vr(vo)}, {sr(srd_, 4)}, {soff} offen lds")
    return out


def advance(half: str) -> list[str]:
    s = SRD_X if half == "x" else SRD_W
    return [f"s_add_u32 {sr(s)}, {sr(s)}, 128", f"s_addc_u32 {sr(s + 1)}, {sr(s + 1)}, 0"]


def frag_read(kind: str, f: int, sub: int) -> str:
    base = V_RX if kind == "x" else V_RW
    dst = (V_FX0 if sub == 0 else V_FX1) if kind == "x" else (V_FW0 if sub == 0 else V_FW1)
    off = 128 * f + 64 * sub
    return f"ds_read_b128 {vr(dst + 4 * f, 4)}, {vr(base)} offset:{off}"


def mfma(i: int, j: int, sub: int, czero: bool = False) -> str:
    """czero: the accumulator starts at 0 (srcC = inline 0: the tile's first
    k-step, no zeroing pass)."""
    fw = (V_FW0 if sub == 0 else V_FW1) + 4 * i
    fx = (V_FX0 if sub == 0 else V_FX1) + 4 * j
    acc = 4 * (8 * i + j)
    return f"v_mfma_f32_16x16x32_bf16 {ar(acc, 4)}, {vr(fw, 4)}, {vr(fx, 4)}, {'0' if czero else ar(acc, 4)}"


# schedule knobs of the main loop (A/B arms: PLAIN_VARIANTS)
SCHED = {"dma_gap": 4, "prio": False, "wait_slot": 95, "read_gap": 1, "group": 4, "sub1_gap": 1, "xbar": 23,
         "xdma_gap": 3, "merge_bar": False, "timing": 0,
         "align": True, "drain_end": False, "map": "lib0", "persist": False, "dual": "", "zero_late": True,
         "nostore": False, "store_nt": True, "store_same": False, "epi_pipe": True,
         "epi_pk": True, "epi_f32s": True,
         # DIAGNOSTIC arms of the SwiGLU backward epilogue (SWIGLU_BWD_VARIANTS;
         # wrong outputs by design): no gu loads (ds stands in for gate and up),
         # no SwiGLU math (the loaded gu stored as dgu), no dgu stores, no epilogue
         "epi_noload": False, "epi_novalu": False, "epi_nostore": False, "epi_none": False,
         # persistent plain kernel whose C stores are issued in the NEXT tile's
         # first k-iteration (packed bf16 parked in a[128:255]; deferred_pack)
         "defer": False}


def _stamp(k: int) -> str:
    return f"s_memtime {sr(S_TMT + 2 * k, 2)}"


def _accum(acc: int, k_end: int, k_begin: int) -> list[str]:
    """acc += low dword of stamp k_end - stamp k_begin (timing kernel; the
    stamps have returned: called after an lgkmcnt(0))."""
    return [f"s_sub_u32 {sr(S_E0)}, {sr(S_TMT + 2 * k_end)}, {sr(S_TMT + 2 * k_begin)}",
            f"s_add_u32 {sr(S_ACC + acc)}, {sr(S_ACC + acc)}, {sr(S_E0)}"]


def iteration(a: Asm, with_dma: bool, next_reads: bool, vm_after_dma: int, trace_base: int = 0):
    """One 64-k tile: 128 MFMAs with the reads / DMA / waits placed in the
    gaps after MFMA n (n = 0..127; 0..63 phase 1, 64..127 phase 2)."""
    gap = SCHED["dma_gap"]
    slots: dict[int, list[str]] = {n: [] for n in range(128)}
    # phase 1: sub-step 1 fragment reads of this stage (X then W)
    g1 = SCHED["sub1_gap"]
    w0 = 17 if g1 == 2 else 8 * g1
    for j in range(8):
        slots[g1 * j].append(frag_read("x", j, 1))
    xb = SCHED["xbar"]
    assert xb > g1 * 7
    tm = SCHED["timing"] == 1      # waits: vmcnt / X-free / W-free barriers
    sp = SCHED["timing"] == 2      # spans: X-DMA, W-DMA and bare MFMA stretches
    if with_dma:
        slots[xb] += ([_stamp(2)] if tm else []) + ["s_waitcnt lgkmcnt(0)", "s_barrier"] + ([_stamp(3)] if tm else [])
    for i in range(8):
        slots[w0 + g1 * i].append(frag_read("w", i, 1))
    if with_dma and SCHED["merge_bar"]:
        # one barrier frees both halves (every sub-step 1 read is issued
        # before it), then the 16 DMA pieces, X first
        assert w0 + g1 * 7 < xb
        xg = SCHED["xdma_gap"]
        for j in range(16):
            slots[xb + 1 + xg * j] += dma(a, "x" if j < 8 else "w", j % 8)
        assert xb + 1 + xg * 15 < 78
        slots[xb + 1 + xg * 8 - 1] += advance("x")
    elif with_dma:
        xg = SCHED["xdma_gap"]
        assert xb + 1 + xg * 7 < 47 and w0 + g1 * 7 < 47
        for j in range(8):
            slots[xb + 1 + xg * j] += dma(a, "x", j)
        slots[47] += advance("x")
        slots[47] += ([_stamp(4)] if tm else []) + ["s_waitcnt lgkmcnt(0)", "s_barrier"] + ([_stamp(5)] if tm else [])
        for j in range(8):
            slots[48 + gap * j] += dma(a, "w", j)               # 48..76
    if with_dma:
        slots[78] += advance("w")
        slots[78] += [f"s_xor_b32 {sr(S_M0X)}, {sr(S_M0X)}, {sr(S_M0XT)}",
                      f"s_xor_b32 {sr(S_M0W)}, {sr(S_M0W)}, {sr(S_M0WT)}"]
        if trace_base:
            slots[47] += trace_mark(trace_base + 1)
            slots[78] += trace_mark(trace_base + 2)
    if next_reads:
        # the next tile (staged one iteration ago) has landed: own DMA by the
        # counted wait, everyone's by the barrier
        ws, rg = SCHED["wait_slot"], SCHED["read_gap"]
        slots[ws] += ([_stamp(0)] if tm else []) + [f"s_waitcnt vmcnt({vm_after_dma})", "s_barrier"] + ([_stamp(1)] if tm else []) + [
                      f"v_xor_b32 {vr(V_RX)}, {vr(V_RX)}, {vr(V_RXT)}",
                      f"v_xor_b32 {vr(V_RW)}, {vr(V_RW)}, {vr(V_RWT)}"]
        for j in range(8):
            slots[ws + 1 + rg * j].append(frag_read("x", j, 0))
        for i in range(8):
            slots[ws + 1 + rg * (8 + i)].append(frag_read("w", i, 0))
        assert ws + 1 + rg * 15 < 126
        slots[126].append("s_waitcnt lgkmcnt(0)")
        if tm:
            slots[126] += _accum(0, 1, 0)
        if sp and with_dma:
            slots[126] += _accum(0, 1, 0) + _accum(1, 3, 2) + _accum(2, 5, 4)
        if trace_base:
            slots[ws] += trace_mark(trace_base + 3)
    if sp and with_dma:
        # stamps AFTER MFMA n (slot lists run after it): [24, 45] X DMA,
        # [47 after the W barrier, 76] W DMA, [77, 94] bare MFMAs
        assert not SCHED["merge_bar"] and xb == 23 and SCHED["xdma_gap"] == 3 and gap == 4 and ws == 95
        slots[23].append(_stamp(0))
        slots[45].append(_stamp(1))
        slots[47].append(_stamp(2))
        slots[76].append(_stamp(3))
        slots[77].append(_stamp(4))
        slots[94].append(_stamp(5))
    if trace_base:
        slots[127] += trace_mark(trace_base + 4)
    if SCHED["prio"]:
        slots[127].append("s_setprio 0")
    for n in range(128):
        sub, m = divmod(n, 64)
        i, j = divmod(m, 8)
        if n == 0 and SCHED["prio"]:
            a("s_setprio 1")
        if n == 64:
            # phase 2 consumes the sub-step 1 fragments read in phase 1
            a("s_waitcnt lgkmcnt(0)")
            if tm and with_dma:
                for ins in _accum(1, 3, 2) + ([] if SCHED["merge_bar"] else _accum(2, 5, 4)):
                    a(ins)
        if SCHED["align"]:
            # every MFMA (8 B) on an 8-byte boundary: a hand-written stream
            # shifted by 4 mod 8 bytes runs ~13 % slower on gfx950
            # (MI355X_MICROARCH.md, code-placement sensitivity); the
            # assembler pads with a 4-byte s_nop 0 only where needed
            a(".p2alignl 3, 0xbf800000")
        a(mfma(i, j, sub))
        for ins in slots[n]:
            a(ins)


# Explicit slot maps (SCHED["map"]): every fragment read, barrier, DMA piece
# and the next-tile wait placed after a given MFMA (0..127).  M0 is set once
# before the first piece of each half and advanced right AFTER each piece, so
# the next piece (at least one MFMA later) needs no s_nop.  The next-tile wait
# counts the pieces issued before it in this iteration; pieces after it (for
# tile t + 2) land by the NEXT iteration's wait.
SLOT_MAPS = {
    # the placement a well-tuned 4-wave, 256 x 256 x 64 library kernel uses
    # on gfx950 (observed from its instruction stream: pieces spread over the
    # whole iteration, three of the W pieces after the next-tile wait)
    "spread": {"x1": [0, 2, 4, 6, 8, 10, 12, 14], "xbar": 20, "w1": [24, 27, 30, 33, 36, 38, 40, 42], "wbar": 50,
               "xdma": [22, 25, 28, 31, 34, 52, 55, 58], "wdma": [61, 64, 85, 87, 89, 96, 100, 124], "wait": 91,
               "x0": [93, 94, 95, 97, 98, 102, 103, 104], "w0": [105, 106, 109, 112, 114, 117, 120, 123]},
    # the same, pieces evenly every 5-6 MFMAs
    "spread2": {"x1": [0, 2, 4, 6, 8, 10, 12, 14], "xbar": 20, "w1": [24, 27, 30, 33, 36, 38, 40, 42],
                "wbar": 50, "xdma": [22, 27, 32, 37, 42, 47, 52, 57], "wdma": [62, 68, 74, 80, 86, 98, 110, 122],
                "wait": 91, "x0": [93, 94, 95, 97, 99, 101, 103, 104], "w0": [105, 106, 109, 112, 114, 117, 120, 123]},
    # fewer pieces before the wait (10): a longer flight for the rest
    "spread3": {"x1": [0, 2, 4, 6, 8, 10, 12, 14], "xbar": 20, "w1": [24, 27, 30, 33, 36, 38, 40, 42],
                "wbar": 50, "xdma": [22, 26, 30, 34, 38, 44, 52, 58], "wdma": [64, 76, 93, 99, 105, 111, 117, 123],
                "wait": 91, "x0": [94, 95, 96, 97, 98, 100, 101, 102], "w0": [103, 104, 106, 108, 110, 113, 116, 119]},
    # "spread" as the library's main 256 x 256 kernel actually issues it:
    # every barrier one MFMA after its wait, M0 advanced one MFMA after each
    # piece, the resource advances a few MFMAs after the last piece
    "lib0": {"x1": [0, 2, 4, 6, 8, 10, 12, 14], "xbar": 20, "w1": [24, 27, 30, 33, 36, 38, 40, 42], "wbar": 50,
             "xdma": [22, 25, 28, 31, 34, 52, 55, 58], "wdma": [61, 64, 85, 87, 89, 96, 100, 124], "wait": 91,
             "x0": [93, 94, 95, 97, 98, 102, 103, 104], "w0": [105, 106, 109, 112, 114, 117, 120, 123],
             "split": 1, "m0_lag": 1, "adv": {"x": 65, "w": 125}},
    # its partner for the waves on odd SIMDs (the library selects one of two
    # loop bodies by the SIMD id): X pieces and W reads one MFMA apart from
    # lib0's, the last four W pieces non-temporal
    "lib1": {"x1": [0, 2, 4, 6, 8, 10, 12, 14], "xbar": 20, "w1": [22, 25, 28, 31, 34, 38, 40, 42], "wbar": 50,
             "xdma": [23, 26, 29, 32, 35, 53, 56, 59], "wdma": [62, 65, 84, 86, 88, 95, 99, 123], "wait": 91,
             "x0": [93, 94, 96, 97, 98, 102, 103, 104], "w0": [105, 106, 109, 112, 114, 117, 120, 122],
             "split": 1, "m0_lag": 1, "adv": {"x": 66, "w": 125}, "nt_w": [4, 5, 6, 7]},
}


def span_slots(m: dict):
    """Stamp slots of the timing kernel's three stretches (after MFMA lo ..
    after MFMA hi): X pieces, W pieces before the next-tile wait, W pieces
    after it."""
    pre = [n for n in m["wdma"] if n < m["wait"]]
    post = [n for n in m["wdma"] if n > m["wait"]]
    return ((m["xdma"][0] - 1, m["xdma"][-1]), (pre[0] - 1, pre[-1]),
            ((post[0] - 1, post[-1]) if post else (m["wait"] + 1, m["wait"] + 2)))


def span_mfmas(m: dict) -> list[int]:
    return [hi - lo for lo, hi in span_slots(m)]


def iteration_map(a: Asm, with_dma: bool, next_reads: bool, vm_after_dma: int, trace_base: int = 0,
                  mapname: str = "", first: bool = False, extra: dict | None = None):
    """One 64-k tile placed by an explicit slot map (SLOT_MAPS).  Map keys
    beyond the placements: `split` puts each barrier that many MFMAs after
    its wait (the MFMA issued in between runs while the wave waits at the
    barrier); `m0_lag` advances M0 that many MFMAs after each piece instead
    of right behind it; `adv` gives the slots of the X / W resource advances
    (default: with the last piece of the half); `nt_w` the W pieces loaded
    non-temporal.  first: the tile's first k-tile (phase-1 MFMAs start their
    accumulators at 0); extra: {slot: [instructions]} placed after those
    MFMAs (the deferred C stores: their VMEM ops before the next-tile wait
    are counted in its vmcnt)."""
    m = SLOT_MAPS[mapname or SCHED["map"]]
    split, lag = m.get("split", 0), m.get("m0_lag", 0)
    nt_w = set(m.get("nt_w", ()))
    slots: dict[int, list[str]] = {n: [] for n in range(128)}
    for j, n in enumerate(m["x1"]):
        slots[n].append(frag_read("x", j, 1))
    for i, n in enumerate(m["w1"]):
        slots[n].append(frag_read("w", i, 1))
    assert max(m["x1"]) < m["xbar"] and max(m["w1"]) < m["wbar"] and max(m["x1"] + m["w1"]) < 63
    tm, sp = SCHED["timing"] == 1, SCHED["timing"] == 2
    if with_dma:
        for bar in (m["xbar"], m["wbar"]):
            slots[bar].append("s_waitcnt lgkmcnt(0)")
            slots[bar + split].append("s_barrier")
        for half, key, bar in (("x", "xdma", m["xbar"]), ("w", "wdma", m["wbar"])):
            srd_, vo, so, m0 = (SRD_X, V_DX, S_SOX, S_M0X) if half == "x" else (SRD_W, V_DW, S_SOW, S_M0W)
            pos = m[key]
            assert sorted(pos) == pos and pos[0] > bar + split and len(set(pos)) == 8
            slots[pos[0] - 1].append(f"s_mov_b32 m0, {sr(m0)}")
            for j, n in enumerate(pos):
                soff = "0" if j == 0 else sr(so + j - 1)
                nt = " nt" if half == "w" and j in nt_w else ""
                slots[n].append(f"buffer_load_dwordx4 {vr(vo)}, {sr(srd_, 4)}, {soff} offen{nt} lds")
                if j < 7:
                    # an MFMA between every M0 write and the next piece (the
                    # M0 -> LDS-DMA hazard wants one wait state)
                    assert pos[j + 1] > n + lag
                    slots[n + lag].append(f"s_add_u32 m0, m0, {4 * LINE}")
            adv = m.get("adv", {}).get(half, pos[-1])
            assert adv >= pos[-1]
            slots[adv] += advance(half) + [f"s_xor_b32 {sr(m0)}, {sr(m0)}, {sr(m0 + 1)}"]
        # the two halves' pieces must not interleave (one running M0)
        assert max(m["xdma"]) + lag < min(m["wdma"]) - 1
        assert m.get("adv", {}).get("x", 0) < 128 and m.get("adv", {}).get("w", 0) < 128
        vm = sum(1 for n in m["xdma"] + m["wdma"] if n < m["wait"])
    else:
        vm = 0
    for n, ins in (extra or {}).items():
        slots[n] += ins
        if n < m["wait"] or (n == m["wait"] and not next_reads):
            vm += sum(1 for x in ins if x.startswith(("buffer_", "global_")))
    def stamp_around(k, n):
        """stamp k before the wait in slot n, stamp k+1 right after its
        barrier (slot n + split; with a split the MFMA between them counts)"""
        slots[n].insert(slots[n].index(next(x for x in slots[n] if x.startswith("s_waitcnt"))), _stamp(k))
        b = slots[n + split]
        b.insert(b.index("s_barrier") + 1, _stamp(k + 1))

    if with_dma and tm:  # waits: X-free and W-free barriers (the vm wait below)
        for k, bar in ((2, m["xbar"]), (4, m["wbar"])):
            stamp_around(k, bar)
    if with_dma and sp:  # stretches: X pieces, W pieces before the wait, W pieces after it
        (x0, x1), (w0, w1), (v0, v1) = span_slots(m)
        for k, (lo, hi) in enumerate(((x0, x1), (w0, w1), (v0, v1))):
            slots[lo].append(_stamp(2 * k))
            slots[hi].append(_stamp(2 * k + 1))
    if next_reads:
        w = m["wait"]
        wait = [f"s_waitcnt vmcnt({vm if with_dma else vm_after_dma})"]
        toggles = [f"v_xor_b32 {vr(V_RX)}, {vr(V_RX)}, {vr(V_RXT)}",
                   f"v_xor_b32 {vr(V_RW)}, {vr(V_RW)}, {vr(V_RWT)}"]
        slots[w] += wait
        slots[w + split] += ["s_barrier"] + toggles
        assert min(m["x0"] + m["w0"]) > w + split
        if tm and with_dma:
            stamp_around(0, w)
        assert min(m["x0"] + m["w0"]) > w and max(m["x0"] + m["w0"]) < 126
        for j, n in enumerate(m["x0"]):
            slots[n].append(frag_read("x", j, 0))
        for i, n in enumerate(m["w0"]):
            slots[n].append(frag_read("w", i, 0))
        slots[126].append("s_waitcnt lgkmcnt(0)")
        if with_dma and tm:
            slots[126] += _accum(0, 1, 0) + _accum(1, 3, 2) + _accum(2, 5, 4)
        if with_dma and sp:
            slots[126] += _accum(0, 1, 0) + _accum(1, 3, 2) + _accum(2, 5, 4)
    for n in range(128):
        sub, mm = divmod(n, 64)
        i, j = divmod(mm, 8)
        if n == 64:
            a("s_waitcnt lgkmcnt(0)")
        if SCHED["align"]:
            a(".p2alignl 3, 0xbf800000")
        a(mfma(i, j, sub, czero=first and sub == 0))
        for ins in slots[n]:
            a(ins)


# ---------------------------------------------------------------- deferred C stores
DEFER_AGPR = 128          # a[128:255]: the previous tile's C, packed bf16 (32 stores x 4 registers)


def deferred_pack(a: Asm):
    """The finished tile's accumulators -> bf16 pairs parked in a[128:255],
    store k = 4 j + p (row block j, column pair p) in a[128 + 4k : +3]: the
    data of epilogue_plain's store (j, p).  Staged through V4..V131 (the
    fragment registers, free between tiles) because the packs overwrite
    accumulators later row blocks still read."""
    f = V_E + 8                                       # 32 fp32 of one row block
    for j in range(8):
        for p in range(4):
            read_pair(a, f + 8 * p, p, j)
        for p in range(4):
            cvt_pack8(a, V_FX0 + 16 * j + 4 * p, f + 8 * p)
    for r in range(128):
        a(f"v_accvgpr_write_b32 {ar(DEFER_AGPR + r)}, {vr(V_FX0 + r)}")


def deferred_stores() -> dict:
    """{slot: instructions} of the previous tile's 32 C stores, store k after
    MFMA k of the next tile's first k-tile: before MFMA 32 + k, whose
    accumulator (fresh, srcC = 0) is the store's data register.  Row block j
    at S_DOFF (advanced by 16 rows after its 4th store); a resource with
    num_records 0 (the first tile: nothing deferred) drops them all."""
    nt = " nt" if SCHED["store_nt"] else ""
    out = {}
    for k in range(32):
        p = k % 4
        ins = [f"buffer_store_dwordx4 {ar(DEFER_AGPR + 4 * k, 4)}, {vr(V_E)}, {sr(SRD_D, 4)}, {sr(S_DOFF)} offen "
               f"offset:{64 * p}{nt}"]
        if p == 3:
            ins.append(f"s_add_u32 {sr(S_DOFF)}, {sr(S_DOFF)}, {sr(S_DSTEP)}")
        out[k] = ins
    return out


def kernel_defer(name: str) -> tuple[str, str]:
    """The persistent plain kernel with deferred C stores (SCHED "defer"):
    a workgroup per CU walks its tiles; tile t's C leaves as 32 stores spread
    over tile t + 1's first k-iteration (one per MFMA gap, under the matrix
    core's work) instead of a burst with the MFMA pipe idle at the end of
    every tile -- the epilogue's HBM traffic costs the plain kernel 1-5 %
    (the no-store arm, profiles/r6_nostore).  The next tile's first two
    k-tiles are staged before the pack, so their flight hides under it;
    its first k-step starts the accumulators at 0 (no zeroing pass)."""
    a = Asm(prefix="defer_")
    a.raw(f".globl {name}")
    a.raw(".p2align 8")
    a.raw(f".type {name},@function")
    a.raw(f"{name}:")
    prologue(a, "plain")
    a(f"s_cmp_lt_u32 {sr(S_KT)}, 3")                # the first k-iteration is peeled: K >= 192
    a(f"s_cbranch_scc1 {a.abort}")
    epi_offsets(a, "plain")                          # V_E: this lane's C offset, the same in every tile
    a(f"s_lshl_b32 {sr(S_DSTEP)}, {sr(S_LDC)}, 4")  # 16 rows
    for r in range(4):                               # nothing deferred yet: num_records 0 drops the stores
        a(f"s_mov_b32 {sr(SRD_D + r)}, {0x20000 if r == 3 else 0}")
    prologue_dma(a)
    a("s_waitcnt vmcnt(16)")
    a("s_barrier")
    l_tile, l_loop, l_tail, l_last = a.fresh("tile"), a.fresh("loop"), a.fresh("tail"), a.fresh("last")
    a.label(l_tile)
    for j in range(8):
        a(frag_read("x", j, 0))
    for i in range(8):
        a(frag_read("w", i, 0))
    a("s_waitcnt lgkmcnt(0)")
    a(f"s_mov_b32 {sr(S_DOFF)}, 0")
    iteration_map(a, with_dma=True, next_reads=True, vm_after_dma=16, first=True, extra=deferred_stores())
    a(f"s_sub_u32 {sr(S_LOOP)}, {sr(S_KT)}, 3")
    a(f"s_cmp_eq_u32 {sr(S_LOOP)}, 0")
    a(f"s_cbranch_scc1 {l_tail}")
    if SCHED["align"]:
        a(".p2alignl 6, 0xbf800000")
    a.label(l_loop)
    iteration_map(a, with_dma=True, next_reads=True, vm_after_dma=16)
    a(f"s_sub_u32 {sr(S_LOOP)}, {sr(S_LOOP)}, 1")
    a(f"s_cmp_eq_u32 {sr(S_LOOP)}, 0")
    a(f"s_cbranch_scc0 {l_loop}")
    a.label(l_tail)
    iteration_map(a, with_dma=False, next_reads=True, vm_after_dma=0)
    iteration_map(a, with_dma=False, next_reads=False, vm_after_dma=0)
    a("s_nop 15")                                    # MFMA results -> VALU reads
    a("s_nop 15")
    # --- next tile: stage parity back to 0 (M0 bases toggled KT times, read bases KT - 1)
    l_even, l_par = a.fresh("even"), a.fresh("par")
    a(f"s_bitcmp1_b32 {sr(S_KT)}, 0")
    a(f"s_cbranch_scc0 {l_even}")
    a(f"s_xor_b32 {sr(S_M0X)}, {sr(S_M0X)}, {sr(S_M0XT)}")
    a(f"s_xor_b32 {sr(S_M0W)}, {sr(S_M0W)}, {sr(S_M0WT)}")
    a(f"s_branch {l_par}")
    a.label(l_even)
    a(f"v_xor_b32 {vr(V_RX)}, {vr(V_RX)}, {vr(V_RXT)}")
    a(f"v_xor_b32 {vr(V_RW)}, {vr(V_RW)}, {vr(V_RWT)}")
    a.label(l_par)
    a(f"s_add_u32 {sr(S_ITER)}, {sr(S_ITER)}, {sr(S_GRID)}")
    a(f"s_mul_i32 {sr(S_T0)}, {sr(S_TM_N)}, {sr(S_TN_N)}")
    a(f"s_cmp_ge_u32 {sr(S_ITER)}, {sr(S_T0)}")
    a(f"s_cbranch_scc1 {l_last}")
    a("s_barrier")                                   # every wave done reading this tile's LDS
    tile_setup(a, "plain", sr(S_ITER))
    prologue_dma(a)                                  # the next tile's k-tiles 0 and 1, in flight under the pack
    deferred_pack(a)
    for r in range(4):
        a(f"s_mov_b32 {sr(SRD_D + r)}, {sr(SRD_C + r)}")
    tile_c(a, "plain")
    a("s_waitcnt vmcnt(16)")                         # the next tile's k-tile 0 (k-tile 1's 16 pieces are younger)
    a("s_barrier")
    a(f"s_branch {l_tile}")
    a.label(l_last)
    epilogue_plain(a)                                # the last tile: stored at once
    a.label(a.abort)
    a("s_endpgm")
    a.raw(f".size {name}, .-{name}")
    body = "\n".join(a.out)
    desc, meta = _descriptor(name)
    return body + "\n" + desc, meta


# ---------------------------------------------------------------- epilogues
def acc_index(i: int, j: int) -> int:
    return 4 * (8 * i + j)


ROPE_DEPTH = 2   # cos / sin row blocks loaded this many blocks ahead (staging in the fragment VGPRs)


def epilogue_rope(a: Asm):
    """The fused-QKV projection's epilogue with RoPE and the head-major
    relayout (replaces toa_rope_fwd): C is never written as [T, (Hq + 2 Hkv)
    128]; wave (wm, wn) owns head h = 2 tn + wn for 128 tokens and stores
    them rotated (q, k heads; rotate-half pairs (d, d + 64), both in the
    lane: fragment pairs p and p + 2) or as they are (v heads) into out =
    [q: B Hq S 128 | k: B Hkv S 128 | v: B Hkv S 128] bf16 (kernarg C).
    Rotation on the fp32 accumulators (the unfused path rotated the bf16-
    rounded GEMM output).  Kernarg S: cos | sin [2][S][64] fp32; fw = S (a
    multiple of 256, so a tile's 256 tokens are one sequence's), fc = Hq |
    Hkv << 16.  cos / sin rows for row block j + ROPE_DEPTH load while j is
    rotated (counted vmcnt, as epilogue_swiglu_bwd_pipe)."""
    v = V_T
    # ---- wave-uniform: w, wm, wn, head, batch, s0 (SGPRs S_E0.. / S_T*)
    a(f"v_lshrrev_b32 {vr(v)}, 6, {vr(V_TID)}")
    a("s_nop 4")
    a(f"v_readfirstlane_b32 {sr(S_Q)}, {vr(v)}")              # w
    a(f"s_and_b32 {sr(S_R)}, {sr(S_Q)}, 1")                   # wm
    a(f"s_lshr_b32 {sr(S_Q)}, {sr(S_Q)}, 1")                  # wn
    a(f"s_lshl_b32 {sr(S_E0)}, {sr(S_TN)}, 1")
    a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_Q)}")         # head h
    a(f"s_lshl_b32 {sr(S_T3)}, {sr(S_TM)}, 8")                # first token of the tile
    udiv(a, S_T0, S_T1, S_T3, S_FW)                           # b = t0 / S, s_tile = t0 % S
    a(f"s_lshl_b32 {sr(S_R)}, {sr(S_R)}, 7")
    a(f"s_add_u32 {sr(S_T1)}, {sr(S_T1)}, {sr(S_R)}")         # s0 = s_tile + 128 wm
    a(f"s_and_b32 {sr(S_T2)}, {sr(S_FC)}, 0xffff")            # Hq
    a(f"s_lshr_b32 {sr(S_T3)}, {sr(S_FC)}, 16")               # Hkv
    # Btot = tiles_m 256 / S (whole sequences): S_E1
    a(f"s_lshl_b32 {sr(S_Q)}, {sr(S_TM_N)}, 8")
    udiv(a, S_E1, S_R, S_Q, S_FW)
    # head row index (in units of S rows of 128 elements) into out, by section:
    #   q: (b Hq + h) ; k: Btot Hq + b Hkv + (h - Hq) ; v: Btot (Hq + Hkv) + b Hkv + (h - Hq - Hkv)
    l_k, l_v, l_base = a.fresh("rope_k"), a.fresh("rope_v"), a.fresh("rope_base")
    a(f"s_mov_b32 {sr(S_LOOP)}, 1")                           # rotate flag (q and k heads)
    a(f"s_cmp_ge_u32 {sr(S_E0)}, {sr(S_T2)}")
    a(f"s_cbranch_scc1 {l_k}")
    a(f"s_mul_i32 {sr(S_Q)}, {sr(S_T0)}, {sr(S_T2)}")
    a(f"s_add_u32 {sr(S_Q)}, {sr(S_Q)}, {sr(S_E0)}")
    a(f"s_branch {l_base}")
    a.label(l_k)
    a(f"s_sub_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_T2)}")        # h - Hq
    a(f"s_mul_i32 {sr(S_Q)}, {sr(S_E1)}, {sr(S_T2)}")         # Btot Hq
    a(f"s_cmp_ge_u32 {sr(S_E0)}, {sr(S_T3)}")
    a(f"s_cbranch_scc1 {l_v}")
    a(f"s_mul_i32 {sr(S_R)}, {sr(S_T0)}, {sr(S_T3)}")
    a(f"s_add_u32 {sr(S_Q)}, {sr(S_Q)}, {sr(S_R)}")
    a(f"s_add_u32 {sr(S_Q)}, {sr(S_Q)}, {sr(S_E0)}")
    a(f"s_branch {l_base}")
    a.label(l_v)
    a(f"s_mov_b32 {sr(S_LOOP)}, 0")
    a(f"s_sub_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_T3)}")        # h - Hq - Hkv
    a(f"s_mul_i32 {sr(S_R)}, {sr(S_E1)}, {sr(S_T3)}")
    a(f"s_add_u32 {sr(S_Q)}, {sr(S_Q)}, {sr(S_R)}")           # Btot (Hq + Hkv)
    a(f"s_mul_i32 {sr(S_R)}, {sr(S_T0)}, {sr(S_T3)}")
    a(f"s_add_u32 {sr(S_Q)}, {sr(S_Q)}, {sr(S_R)}")
    a(f"s_add_u32 {sr(S_Q)}, {sr(S_Q)}, {sr(S_E0)}")
    a.label(l_base)
    # byte offset of (head row, s0): (S_Q S + s0) 256 -> SRD_C over this wave's 128 rows
    a(f"s_mul_i32 {sr(S_Q)}, {sr(S_Q)}, {sr(S_FW)}")
    a(f"s_add_u32 {sr(S_Q)}, {sr(S_Q)}, {sr(S_T1)}")
    a(f"s_mov_b32 {sr(S_R)}, 256")
    mul64(a, S_T2, S_T3, S_Q, S_R)
    a(f"s_mov_b32 {sr(S_R)}, {128 * 256}")
    srd(a, SRD_C, S_C, S_T2, S_T3, S_R)
    # cos / sin rows s0 .. s0 + 127: SRD_S at cos + s0 256, sin + S 256 (soffset S_E1 = S 256)
    a(f"s_mov_b32 {sr(S_R)}, 256")
    mul64(a, S_T2, S_T3, S_T1, S_R)
    a(f"s_mul_i32 {sr(S_E1)}, {sr(S_FW)}, 256")
    a(f"s_add_u32 {sr(S_R)}, {sr(S_E1)}, {128 * 256}")
    srd(a, SRD_S, S_S, S_T2, S_T3, S_R)
    # ---- per lane: C offset (row l & 15, group g = l >> 4: 16 g bytes), cos offset 32 g bytes
    a(f"v_and_b32 {vr(v + 1)}, 63, {vr(V_TID)}")
    a(f"v_and_b32 {vr(v + 2)}, 15, {vr(v + 1)}")
    a(f"v_lshlrev_b32 {vr(v + 2)}, 8, {vr(v + 2)}")           # row * 256
    a(f"v_lshrrev_b32 {vr(v + 3)}, 4, {vr(v + 1)}")           # g
    a(f"v_lshl_add_u32 {vr(V_E)}, {vr(v + 3)}, 4, {vr(v + 2)}")      # out: 16 g
    a(f"v_lshl_add_u32 {vr(V_E + 1)}, {vr(v + 3)}, 5, {vr(v + 2)}")  # cos: 32 g
    a(f"s_mov_b32 {sr(S_T0)}, 0")                             # row block soffset (out and cos: 16 rows x 256 B)
    a(f"s_mov_b32 {sr(S_T1)}, 0")                             # cos prefetch soffset
    a(f"s_add_u32 {sr(S_T2)}, {sr(S_E1)}, 0")                 # sin prefetch soffset (S 256 + row block)
    l_plain, l_end = a.fresh("rope_plain"), a.fresh("rope_end")
    a(f"s_cmp_eq_u32 {sr(S_LOOP)}, 0")
    a(f"s_cbranch_scc1 {l_plain}")
    D = ROPE_DEPTH
    seq: list = []

    def slot(j):
        return V_FX0 + 32 * (j % D)             # cos 16 regs, sin 16 regs

    def issue(j):
        st = slot(j)
        for p in range(2):
            for h in range(2):
                a(f"buffer_load_dwordx4 {vr(st + 8 * p + 4 * h, 4)}, {vr(V_E + 1)}, {sr(SRD_S, 4)}, {sr(S_T1)} offen offset:{128 * p + 16 * h}")
                a(f"buffer_load_dwordx4 {vr(st + 16 + 8 * p + 4 * h, 4)}, {vr(V_E + 1)}, {sr(SRD_S, 4)}, {sr(S_T2)} offen offset:{128 * p + 16 * h}")
                seq.extend([("L", j), ("L", j)])
        a(f"s_add_u32 {sr(S_T1)}, {sr(S_T1)}, 4096")
        a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, 4096")

    for j in range(min(D, 8)):
        issue(j)
    f, pk, t = V_E + 8, V_E + 40, V_E + 56
    for j in range(8):
        for p in range(4):
            read_pair(a, f + 8 * p, p, j)
        last = max(i for i, x in enumerate(seq) if x == ("L", j))
        a(f"s_waitcnt vmcnt({min(63, len(seq) - last - 1)})")
        cs, sn = slot(j), slot(j) + 16
        for p in range(2):
            for e in range(8):
                x1, x2 = f + 8 * p + e, f + 8 * (p + 2) + e
                c_, s_ = cs + 8 * p + e, sn + 8 * p + e
                a(f"v_mul_f32 {vr(t)}, {vr(x2)}, {vr(s_)}")
                a(f"v_mul_f32 {vr(t + 1)}, {vr(x1)}, {vr(s_)}")
                a(f"v_mul_f32 {vr(t + 2)}, {vr(x1)}, {vr(c_)}")
                a(f"v_fma_f32 {vr(x2)}, {vr(x2)}, {vr(c_)}, {vr(t + 1)}")   # x2 c + x1 s
                a(f"v_sub_f32 {vr(x1)}, {vr(t + 2)}, {vr(t)}")              # x1 c - x2 s
        if j + D < 8:
            issue(j + D)                          # into the slot just consumed
        for p in range(4):
            cvt_pack8(a, pk + 4 * p, f + 8 * p)
        for p in range(4):
            store16(a, pk + 4 * p, V_E, SRD_C, S_T0, p)
        seq.extend([("S", j)] * 4)
        a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, 4096")
        a("s_nop 1")
    a(f"s_branch {l_end}")
    # ---- v heads: the relayout alone
    a.label(l_plain)
    for j in range(8):
        for p in range(4):
            read_pair(a, f + 8 * p, p, j)
        for p in range(4):
            cvt_pack8(a, pk + 4 * p, f + 8 * p)
        for p in range(4):
            store16(a, pk + 4 * p, V_E, SRD_C, S_T0, p)
        a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, 4096")
        a("s_nop 1")
    a.label(l_end)


DELTA_DEPTH = 2      # O row blocks loaded this many blocks ahead
SRD_DL = 72          # s72..s75: the delta rows of this wave (kernarg bytes 88..95)


def epilogue_delta(a: Asm):
    """The attention output projection's data gradient dO = dY Wo (plain C
    stores) with the attention backward's delta fused in: ndelta[(b H + h) S
    + s] = -sum_d dO[t][128 h + d] O[t][128 h + d] over the wave's head h =
    2 tn + wn (kernarg S = O, laid out like C; fw = S, fc = H; bytes 88..95
    = ndelta fp32 [B, H, S]).  dO enters as the bf16 values stored (what the
    attention backward's dP reads).  A row's 128 columns sit in 4 lanes
    (l & 15 fixed); their partial sums meet in 1 KiB of LDS past the
    pipeline's stages; O row blocks load DELTA_DEPTH blocks ahead.  Replaces
    attn_delta_kernel's pass over dO and O (csrc/hip/attention.hip)."""
    v = V_T
    a(f"s_load_dwordx2 {sr(SRD_DL, 2)}, s[0:1], 0x58")
    a(f"v_lshrrev_b32 {vr(v)}, 6, {vr(V_TID)}")
    a("s_nop 4")
    a(f"v_readfirstlane_b32 {sr(S_Q)}, {vr(v)}")              # w
    a(f"s_and_b32 {sr(S_R)}, {sr(S_Q)}, 1")                   # wm
    a(f"s_lshr_b32 {sr(S_T2)}, {sr(S_Q)}, 1")                 # wn
    a(f"s_lshl_b32 {sr(S_T3)}, {sr(S_TN)}, 1")
    a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_T3)}")        # head h
    a(f"s_lshl_b32 {sr(S_T3)}, {sr(S_TM)}, 8")
    udiv(a, S_T0, S_T1, S_T3, S_FW)                           # b, s_tile
    a(f"s_lshl_b32 {sr(S_R)}, {sr(S_R)}, 7")
    a(f"s_add_u32 {sr(S_T1)}, {sr(S_T1)}, {sr(S_R)}")         # s0
    a(f"s_mul_i32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_FC)}")
    a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_T2)}")        # b H + h
    a(f"s_mul_i32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_FW)}")
    a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_T1)}")        # row of s0
    a(f"s_lshl_b32 {sr(S_T0)}, {sr(S_T0)}, 2")
    a("s_waitcnt lgkmcnt(0)")
    a(f"s_add_u32 {sr(SRD_DL)}, {sr(SRD_DL)}, {sr(S_T0)}")
    a(f"s_addc_u32 {sr(SRD_DL + 1)}, {sr(SRD_DL + 1)}, 0")
    a(f"s_mov_b32 {sr(SRD_DL + 2)}, {128 * 4}")
    a(f"s_mov_b32 {sr(SRD_DL + 3)}, 0x20000")
    # lanes: LDS scratch (wave w: 256 B at LDS_BYTES + 256 w), the delta row (l & 15)
    a(f"v_and_b32 {vr(v + 1)}, 63, {vr(V_TID)}")
    a(f"v_lshlrev_b32 {vr(v + 2)}, 2, {vr(V_TID)}")            # 4 (64 w + l)
    a(f"v_add_u32 {vr(v + 2)}, {LDS_BYTES}, {vr(v + 2)}")       # write address
    a(f"v_and_b32 {vr(v + 3)}, 15, {vr(v + 1)}")
    a(f"v_lshlrev_b32 {vr(v + 3)}, 2, {vr(v + 3)}")             # 4 (l & 15): delta offset
    a(f"v_sub_u32 {vr(V_E + 2)}, {vr(v + 2)}, {vr(v + 1)}")    # ... 4 l ...
    a(f"v_sub_u32 {vr(V_E + 2)}, {vr(V_E + 2)}, {vr(v + 1)}")
    a(f"v_sub_u32 {vr(V_E + 2)}, {vr(V_E + 2)}, {vr(v + 1)}")
    a(f"v_sub_u32 {vr(V_E + 2)}, {vr(V_E + 2)}, {vr(v + 1)}")  # wave base: LDS_BYTES + 256 w
    a(f"v_add_u32 {vr(V_E + 2)}, {vr(V_E + 2)}, {vr(v + 3)}")  # + 4 (l & 15): the row's 4 partials at +0/64/128/192
    a(f"s_mov_b32 {sr(S_E0)}, 0")                             # row block offset (C and O)
    a(f"s_lshl_b32 {sr(S_E1)}, {sr(S_LDC)}, 4")
    a(f"s_mov_b32 {sr(S_T2)}, 0")                             # O prefetch row block offset
    D = DELTA_DEPTH
    seq: list = []

    def slot(j):
        return V_FX0 + 16 * (j % D)

    def issue(j):
        for p in range(4):
            a(f"buffer_load_dwordx4 {vr(slot(j) + 4 * p, 4)}, {vr(V_E)}, {sr(SRD_S, 4)}, {sr(S_T2)} offen offset:{64 * p}")
            seq.append(("L", j))
        a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_E1)}")

    for j in range(min(D, 8)):
        issue(j)
    f, pk, ob, acc = V_E + 8, V_E + 40, V_E + 56, V_E + 72
    for j in range(8):
        for p in range(4):
            read_pair(a, f + 8 * p, p, j)
        for p in range(4):
            cvt_pack8(a, pk + 4 * p, f + 8 * p)
        for p in range(4):
            store16(a, pk + 4 * p, V_E, SRD_C, S_E0, p)
        seq.extend([("S", j)] * 4)
        for p in range(4):
            unpack8(a, f + 8 * p, pk + 4 * p)                  # dO as stored (bf16)
        last = max(i for i, x in enumerate(seq) if x == ("L", j))
        a(f"s_waitcnt vmcnt({min(63, len(seq) - last - 1)})")
        for p in range(4):
            unpack8(a, ob + 8 * (p % 2), slot(j) + 4 * p)
            for e in range(8):
                if p == 0 and e == 0:
                    a(f"v_mul_f32 {vr(acc)}, {vr(f)}, {vr(ob)}")
                else:
                    a(f"v_fma_f32 {vr(acc)}, {vr(f + 8 * p + e)}, {vr(ob + 8 * (p % 2) + e)}, {vr(acc)}")
        if j + D < 8:
            issue(j + D)
        a(f"ds_write_b32 {vr(v + 2)}, {vr(acc)}")
        a("s_waitcnt lgkmcnt(0)")
        for q in range(4):
            a(f"ds_read_b32 {vr(acc + 1 + q)}, {vr(V_E + 2)} offset:{64 * q}")
        a("s_waitcnt lgkmcnt(0)")
        a(f"v_add_f32 {vr(acc + 1)}, {vr(acc + 1)}, {vr(acc + 2)}")
        a(f"v_add_f32 {vr(acc + 3)}, {vr(acc + 3)}, {vr(acc + 4)}")
        a(f"v_add_f32 {vr(acc + 1)}, {vr(acc + 1)}, {vr(acc + 3)}")
        a(f"v_sub_f32 {vr(acc + 1)}, 0, {vr(acc + 1)}")        # -delta
        a(f"s_mov_b32 {sr(S_T3)}, {64 * j}")
        a(f"buffer_store_dword {vr(acc + 1)}, {vr(v + 3)}, {sr(SRD_DL, 4)}, {sr(S_T3)} offen")
        seq.append(("S", j))
        a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_E1)}")
        a("s_nop 1")


def epilogue_resadd(a: Asm):
    """C = X W^T + R (bf16 R laid out like C, kernarg S): the residual add of
    the attention output projection in its epilogue, so the RMSNorm after it
    reads one tensor and writes one (ops/llm._AttnOutProj).  R row blocks
    load DELTA_DEPTH blocks ahead (counted vmcnt); the sum is rounded to bf16
    once, as the unfused add of the bf16 GEMM output and R is not (the fused
    path adds in fp32 before the one rounding)."""
    a(f"s_mov_b32 {sr(S_E0)}, 0")
    a(f"s_lshl_b32 {sr(S_E1)}, {sr(S_LDC)}, 4")
    a(f"s_mov_b32 {sr(S_T2)}, 0")
    D = DELTA_DEPTH
    seq: list = []

    def slot(j):
        return V_FX0 + 16 * (j % D)

    def issue(j):
        for p in range(4):
            a(f"buffer_load_dwordx4 {vr(slot(j) + 4 * p, 4)}, {vr(V_E)}, {sr(SRD_S, 4)}, {sr(S_T2)} offen offset:{64 * p}")
            seq.append(("L", j))
        a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_E1)}")

    for j in range(min(D, 8)):
        issue(j)
    f, pk, rb = V_E + 8, V_E + 40, V_E + 56
    for j in range(8):
        for p in range(4):
            read_pair(a, f + 8 * p, p, j)
        last = max(i for i, x in enumerate(seq) if x == ("L", j))
        a(f"s_waitcnt vmcnt({min(63, len(seq) - last - 1)})")
        for p in range(4):
            unpack8(a, rb, slot(j) + 4 * p)
            for e in range(8):
                a(f"v_add_f32 {vr(f + 8 * p + e)}, {vr(f + 8 * p + e)}, {vr(rb + e)}")
        if j + D < 8:
            issue(j + D)
        for p in range(4):
            cvt_pack8(a, pk + 4 * p, f + 8 * p)
        for p in range(4):
            store16(a, pk + 4 * p, V_E, SRD_C, S_E0, p)
        seq.extend([("S", j)] * 4)
        a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_E1)}")
        a("s_nop 1")


def epi_offsets(a: Asm, epi: str):
    """Per-lane output byte offsets.  Lane l of wave (wm, wn) holds, for
    fragments (2p, j) and (2p+1, j): row m = wm*128 + 16 j + (l & 15) and the
    8 columns n = 32 p + 8 (l >> 4) .. +7 of the wave's W rows (the W-row
    permutation of the DMA): one 16-byte store per pair p."""
    v = V_T
    a(f"v_lshrrev_b32 {vr(v)}, 6, {vr(V_TID)}")            # w
    a(f"v_and_b32 {vr(v + 1)}, 63, {vr(V_TID)}")           # lane
    a(f"v_and_b32 {vr(v + 2)}, 15, {vr(v + 1)}")
    a(f"v_and_b32 {vr(v + 3)}, 1, {vr(v)}")
    a(f"v_lshl_add_u32 {vr(v + 2)}, {vr(v + 3)}, 7, {vr(v + 2)}")  # row in tile
    a(f"v_lshrrev_b32 {vr(v + 1)}, 4, {vr(v + 1)}")        # lane >> 4
    a(f"v_lshlrev_b32 {vr(v + 1)}, 4, {vr(v + 1)}")        # 16 B per lane group
    a(f"v_lshrrev_b32 {vr(v)}, 1, {vr(v)}")                # wn
    # column bytes of the wave: plain / bwd 128 cols per wave, fwd 64 units
    a(f"v_lshlrev_b32 {vr(v)}, {8 if epi != 'swiglu_fwd' else 7}, {vr(v)}")
    a(f"v_add_u32 {vr(v + 1)}, {vr(v + 1)}, {vr(v)}")      # col bytes
    # V_E+0: C offset, V_E+1: S offset (fwd: s; bwd: gu)
    a(f"v_mul_lo_u32 {vr(V_E)}, {vr(v + 2)}, {sr(S_LDC)}")
    a(f"v_add_u32 {vr(V_E)}, {vr(V_E)}, {vr(v + 1)}")
    if epi != "plain":
        a(f"v_mul_lo_u32 {vr(V_E + 1)}, {vr(v + 2)}, {sr(S_LDS)}")
        a(f"v_add_u32 {vr(V_E + 1)}, {vr(V_E + 1)}, {vr(v + 1)}")
    if epi == "swiglu_fwd":
        a(f"v_add_u32 {vr(V_E + 2)}, {sr(S_FC)}, {vr(V_E)}")  # up half of gu
    if epi == "swiglu_bwd":
        a(f"v_add_u32 {vr(V_E + 2)}, {sr(S_FC)}, {vr(V_E)}")      # up half of dgu
        a(f"v_add_u32 {vr(V_E + 3)}, {sr(S_FC)}, {vr(V_E + 1)}")  # up half of gu


def read_acc4(a: Asm, dst: int, acc: int):
    for r in range(4):
        a(f"v_accvgpr_read_b32 {vr(dst + r)}, {ar(acc + r)}")


def cvt_pack(a: Asm, dst: int, src: int):
    a(f"v_cvt_pk_bf16_f32 {vr(dst)}, {vr(src)}, {vr(src + 1)}")
    a(f"v_cvt_pk_bf16_f32 {vr(dst + 1)}, {vr(src + 2)}, {vr(src + 3)}")


def unpack_bf16(a: Asm, dst: int, src: int):
    """dst[0..3] = f32 of the 4 bf16 in src[0..1] (element order kept)."""
    a(f"v_lshlrev_b32 {vr(dst)}, 16, {vr(src)}")
    a(f"v_and_b32 {vr(dst + 1)}, 0xffff0000, {vr(src)}")
    a(f"v_lshlrev_b32 {vr(dst + 2)}, 16, {vr(src + 1)}")
    a(f"v_and_b32 {vr(dst + 3)}, 0xffff0000, {vr(src + 1)}")


LOG2E = 1.4426950408889634


def read_pair(a: Asm, dst: int, p: int, j: int, ioff: int = 0):
    """dst[0..7] = the lane's 8 consecutive columns of fragments (2p, j) and
    (2p+1, j) (ioff: fragment offset, 4 for SwiGLU's up half)."""
    read_acc4(a, dst, acc_index(2 * p + ioff, j))
    read_acc4(a, dst + 4, acc_index(2 * p + 1 + ioff, j))


def cvt_pack8(a: Asm, dst: int, src: int):
    cvt_pack(a, dst, src)
    cvt_pack(a, dst + 2, src + 4)


def unpack8(a: Asm, dst: int, src: int):
    unpack_bf16(a, dst, src)
    unpack_bf16(a, dst + 4, src + 2)


def store16(a: Asm, data: int, voff: int, srd_: int, soff: int, p: int):
    nt = " nt" if SCHED["store_nt"] else ""
    a(f"buffer_store_dwordx4 {vr(data, 4)}, {vr(voff)}, {sr(srd_, 4)}, {sr(soff)} offen offset:{64 * p}{nt}")


def epilogue_plain(a: Asm):
    a(f"s_mov_b32 {sr(S_E0)}, 0")                             # row block offset
    a(f"s_lshl_b32 {sr(S_E1)}, {sr(S_LDC)}, 4")              # 16 rows
    for j in range(8):
        f, pk = V_E + 8, V_E + 40                             # 32 f32, 16 packed
        for p in range(4):
            read_pair(a, f + 8 * p, p, j)
        for p in range(4):
            cvt_pack8(a, pk + 4 * p, f + 8 * p)
        for p in range(4):
            if not SCHED["nostore"]:
                store16(a, pk + 4 * p, V_E, SRD_C, S_E0, p)
        a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_E1)}")


def silu_times(a: Asm, out: int, g: int, u: int, t: int, n: int):
    """out[e] = silu(g[e]) * u[e] = g / (1 + 2^(-g log2 e)) * u, e < n
    (batched per op: a transcendental's result is consumed n instructions
    later, past the forwarding hazard).  epi_pk: the non-transcendental ops
    on register pairs (v_pk_*_f32; constants -log2 e and 1.0 as pairs at
    V_E + 4 / V_E + 6)."""
    if SCHED["epi_pk"]:
        for e in range(0, n, 2):
            a(f"v_pk_mul_f32 {vr(t + e, 2)}, {vr(V_E + 4, 2)}, {vr(g + e, 2)}")
        for e in range(n):
            a(f"v_exp_f32 {vr(t + e)}, {vr(t + e)}")
        for e in range(0, n, 2):
            a(f"v_pk_add_f32 {vr(t + e, 2)}, {vr(V_E + 6, 2)}, {vr(t + e, 2)}")
        for e in range(n):
            a(f"v_rcp_f32 {vr(t + e)}, {vr(t + e)}")
        for e in range(0, n, 2):
            a(f"v_pk_mul_f32 {vr(t + e, 2)}, {vr(g + e, 2)}, {vr(t + e, 2)}")
        for e in range(0, n, 2):
            a(f"v_pk_mul_f32 {vr(out + e, 2)}, {vr(t + e, 2)}, {vr(u + e, 2)}")
        return
    for e in range(n):
        a(f"v_mul_f32 {vr(t + e)}, {vr(V_E + 3)}, {vr(g + e)}")
    for e in range(n):
        a(f"v_exp_f32 {vr(t + e)}, {vr(t + e)}")
    for e in range(n):
        a(f"v_add_f32 {vr(t + e)}, 1.0, {vr(t + e)}")
    for e in range(n):
        a(f"v_rcp_f32 {vr(t + e)}, {vr(t + e)}")
    for e in range(n):
        a(f"v_mul_f32 {vr(t + e)}, {vr(g + e)}, {vr(t + e)}")
    for e in range(n):
        a(f"v_mul_f32 {vr(out + e)}, {vr(t + e)}, {vr(u + e)}")


def epilogue_swiglu_fwd(a: Asm):
    """Fragments 0..3 gate, 4..7 the same hidden units' up values: pairs
    p = 0, 1 of each give a lane 8 consecutive units."""
    a(f"s_mov_b32 {sr(S_E0)}, 0")
    a(f"s_lshl_b32 {sr(S_E1)}, {sr(S_LDC)}, 4")
    a(f"s_mov_b32 {sr(S_T0)}, 0")
    a(f"s_lshl_b32 {sr(S_T1)}, {sr(S_LDS)}, 4")
    a(f"v_mov_b32 {vr(V_E + 3)}, {-LOG2E!r}")
    for x in (4, 5):
        a(f"v_mov_b32 {vr(V_E + x)}, {-LOG2E!r}")
    for x in (6, 7):
        a(f"v_mov_b32 {vr(V_E + x)}, 1.0")
    for j in range(8):
        g, u = V_E + 8, V_E + 24            # 16 f32 each (2 pairs)
        for p in range(2):
            read_pair(a, g + 8 * p, p, j)
            read_pair(a, u + 8 * p, p, j, ioff=4)
        pg, pu = V_E + 40, V_E + 48         # packed bf16 (8 regs each)
        for p in range(2):
            cvt_pack8(a, pg + 4 * p, g + 8 * p)
            cvt_pack8(a, pu + 4 * p, u + 8 * p)
        for p in range(2):
            store16(a, pg + 4 * p, V_E, SRD_C, S_E0, p)
            store16(a, pu + 4 * p, V_E + 2, SRD_C, S_E0, p)
        sv, ps = V_E + 88, V_E + 104
        if SCHED["epi_f32s"]:
            # s = silu(g) * u straight from the fp32 accumulators (no bf16 round
            # trip: 32 VALU per row block fewer; the unfused path and round 4
            # used the stored bf16 values, a difference below bf16 rounding)
            for h in range(2):              # scratch: the free V_E + 56 .. 63
                silu_times(a, sv + 8 * h, g + 8 * h, u + 8 * h, V_E + 56, 8)
        else:
            # s = silu(g) * u on the bf16-rounded values (what backward re-reads)
            gf, uf, t = V_E + 56, V_E + 72, V_E + 8   # t: g/u regs, consumed
            for p in range(2):
                unpack8(a, gf + 8 * p, pg + 4 * p)
                unpack8(a, uf + 8 * p, pu + 4 * p)
            for h in range(2):              # 8 elements at a time (scratch t: 8 regs)
                silu_times(a, sv + 8 * h, gf + 8 * h, uf + 8 * h, t, 8)
        for p in range(2):
            cvt_pack8(a, ps + 4 * p, sv + 8 * p)
        for p in range(2):
            store16(a, ps + 4 * p, V_E + 1, SRD_S, S_T0, p)
        a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_E1)}")
        a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_T1)}")
        if not SCHED["epi_pipe"]:
            a("s_waitcnt vmcnt(0)")         # (round 4) scratch reused by the next row block
        # epi_pipe: no drain -- a store reads its data registers within two
        # wait states of issue (cdna_hip_programming.md, asm stores), and the
        # next row block rewrites them dozens of instructions later


EPI_DEPTH = 6    # SwiGLU backward: gu row blocks loaded this many rounds ahead (staging in the free fragment VGPRs)


def epilogue_swiglu_bwd(a: Asm):
    if SCHED["epi_pipe"]:
        return epilogue_swiglu_bwd_pipe(a)
    return epilogue_swiglu_bwd_r4(a)


def epilogue_swiglu_bwd_pipe(a: Asm):
    """The SwiGLU backward epilogue with its gu loads software-pipelined:
    16 rounds (8 row blocks x 2 column halves), round r's 4 loads issued
    EPI_DEPTH rounds ahead into staging slots in the main loop's fragment
    VGPRs (free here), each round waiting only for its own loads (counted
    vmcnt: VMEM completes in issue order) instead of draining every load
    and store per round -- the round-4 form exposed a full memory latency 32
    times per tile (59 % MFMA busy in the model, profiles/r5_pmc)."""
    a(f"s_mov_b32 {sr(S_E0)}, 0")                             # dgu row block
    a(f"s_lshl_b32 {sr(S_E1)}, {sr(S_LDC)}, 4")
    a(f"s_mov_b32 {sr(S_T2)}, 0")                             # gu row block of the next prefetch
    a(f"s_lshl_b32 {sr(S_T1)}, {sr(S_LDS)}, 4")
    a(f"v_mov_b32 {vr(V_E + 4)}, {-LOG2E!r}")
    if SCHED["epi_pk"]:   # pairs: -log2 e (V_E + 4), 1.0 (V_E + 6), -1.0 (V_E + 10)
        a(f"v_mov_b32 {vr(V_E + 5)}, {-LOG2E!r}")
        for x in (6, 7):
            a(f"v_mov_b32 {vr(V_E + x)}, 1.0")
        for x in (10, 11):
            a(f"v_mov_b32 {vr(V_E + x)}, -1.0")
    rounds = [(j, half) for j in range(8) for half in range(2)]
    D = EPI_DEPTH
    seq: list = []     # VMEM ops in issue order: ("L" | "S", round)

    def slot(r):
        return V_FX0 + 16 * (r % D)                           # lg = slot, lu = slot + 8

    noload, novalu, nostore = SCHED["epi_noload"], SCHED["epi_novalu"], SCHED["epi_nostore"]

    def issue_loads(r):
        j, half = rounds[r]
        if noload:
            return
        lg, lu = slot(r), slot(r) + 8
        for q, p in enumerate((2 * half, 2 * half + 1)):
            a(f"buffer_load_dwordx4 {vr(lg + 4 * q, 4)}, {vr(V_E + 1)}, {sr(SRD_S, 4)}, {sr(S_T2)} offen offset:{64 * p}")
            a(f"buffer_load_dwordx4 {vr(lu + 4 * q, 4)}, {vr(V_E + 3)}, {sr(SRD_S, 4)}, {sr(S_T2)} offen offset:{64 * p}")
            seq.extend([("L", r), ("L", r)])
        if half == 1:
            a(f"s_add_u32 {sr(S_T2)}, {sr(S_T2)}, {sr(S_T1)}")   # the next prefetch reads the next row block

    for r in range(min(D, len(rounds))):
        issue_loads(r)
    for r, (j, half) in enumerate(rounds):
        ps_ = (2 * half, 2 * half + 1)
        if novalu:   # DIAGNOSTIC: the loaded gu goes straight back out as dgu
            last = max(i for i, x in enumerate(seq) if x == ("L", r))
            a(f"s_waitcnt vmcnt({min(63, len(seq) - last - 1)})")
            lg, lu = slot(r), slot(r) + 8
            if not nostore:
                for q, p in enumerate(ps_):
                    store16(a, lg + 4 * q, V_E, SRD_C, S_E0, p)
                    store16(a, lu + 4 * q, V_E + 2, SRD_C, S_E0, p)
                seq.extend([("S", r)] * 4)
            a("s_nop 1")
            if r + D < len(rounds):
                issue_loads(r + D)
            if half == 1:
                a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_E1)}")
            continue
        d = V_E + 24                        # 16 f32: ds (no memory dependency: first)
        for q, p in enumerate(ps_):
            read_pair(a, d + 8 * q, p, j)
        pd = V_E + 40                       # bf16-rounded ds, then unpacked
        for q in range(2):
            cvt_pack8(a, pd + 4 * q, d + 8 * q)
        for q in range(2):
            unpack8(a, d + 8 * q, pd + 4 * q)
        if noload:   # DIAGNOSTIC: ds stands in for both gate and up
            lg = lu = pd
        else:
            last = max(i for i, x in enumerate(seq) if x == ("L", r))
            a(f"s_waitcnt vmcnt({min(63, len(seq) - last - 1)})")   # this round's loads only
            lg, lu = slot(r), slot(r) + 8
        gf, uf = V_E + 48, V_E + 64
        for q in range(2):
            unpack8(a, gf + 8 * q, lg + 4 * q)
            unpack8(a, uf + 8 * q, lu + 4 * q)
        if r + D < len(rounds):
            issue_loads(r + D)              # into the slot just unpacked
        sg, tmp, tt = V_E + 80, V_E + 96, V_E + 8
        if SCHED["epi_pk"]:                 # the same math on register pairs
            for e in range(0, 16, 2):       # sg = 1 / (1 + exp(-g))
                a(f"v_pk_mul_f32 {vr(sg + e, 2)}, {vr(V_E + 4, 2)}, {vr(gf + e, 2)}")
            for e in range(16):
                a(f"v_exp_f32 {vr(sg + e)}, {vr(sg + e)}")
            for e in range(0, 16, 2):
                a(f"v_pk_add_f32 {vr(sg + e, 2)}, {vr(V_E + 6, 2)}, {vr(sg + e, 2)}")
            for e in range(16):
                a(f"v_rcp_f32 {vr(sg + e)}, {vr(sg + e)}")
            for e in range(0, 16, 2):       # du = d * g * sg  -> tmp
                a(f"v_pk_mul_f32 {vr(tmp + e, 2)}, {vr(d + e, 2)}, {vr(gf + e, 2)}")
                a(f"v_pk_mul_f32 {vr(tmp + e, 2)}, {vr(tmp + e, 2)}, {vr(sg + e, 2)}")
            for e in range(0, 16, 2):       # dg = d * u * sg * (1 + g (1 - sg)) -> uf
                a(f"v_pk_fma_f32 {vr(tt, 2)}, {vr(sg + e, 2)}, {vr(V_E + 10, 2)}, {vr(V_E + 6, 2)}")
                a(f"v_pk_fma_f32 {vr(tt, 2)}, {vr(gf + e, 2)}, {vr(tt, 2)}, {vr(V_E + 6, 2)}")
                a(f"v_pk_mul_f32 {vr(uf + e, 2)}, {vr(d + e, 2)}, {vr(uf + e, 2)}")
                a(f"v_pk_mul_f32 {vr(uf + e, 2)}, {vr(uf + e, 2)}, {vr(sg + e, 2)}")
                a(f"v_pk_mul_f32 {vr(uf + e, 2)}, {vr(uf + e, 2)}, {vr(tt, 2)}")
        else:
            for e in range(16):             # sg = 1 / (1 + exp(-g))
                a(f"v_mul_f32 {vr(sg + e)}, {vr(V_E + 4)}, {vr(gf + e)}")
            for e in range(16):
                a(f"v_exp_f32 {vr(sg + e)}, {vr(sg + e)}")
            for e in range(16):
                a(f"v_add_f32 {vr(sg + e)}, 1.0, {vr(sg + e)}")
            for e in range(16):
                a(f"v_rcp_f32 {vr(sg + e)}, {vr(sg + e)}")
            for e in range(16):             # du = d * g * sg  -> tmp
                a(f"v_mul_f32 {vr(tmp + e)}, {vr(d + e)}, {vr(gf + e)}")
                a(f"v_mul_f32 {vr(tmp + e)}, {vr(tmp + e)}, {vr(sg + e)}")
            for e in range(16):             # dg = d * u * sg * (1 + g (1 - sg)) -> uf
                a(f"v_sub_f32 {vr(tt)}, 1.0, {vr(sg + e)}")
                a(f"v_fma_f32 {vr(tt)}, {vr(gf + e)}, {vr(tt)}, 1.0")
                a(f"v_mul_f32 {vr(uf + e)}, {vr(d + e)}, {vr(uf + e)}")
                a(f"v_mul_f32 {vr(uf + e)}, {vr(uf + e)}, {vr(sg + e)}")
                a(f"v_mul_f32 {vr(uf + e)}, {vr(uf + e)}, {vr(tt)}")
        pdg, pdu = V_E + 40, V_E + 112      # 8 + 4 regs: reuse gf for the last du pair
        for q in range(2):
            cvt_pack8(a, pdg + 4 * q, uf + 8 * q)
        cvt_pack8(a, pdu, tmp)
        cvt_pack8(a, gf, tmp + 8)
        if not nostore:
            for q, p in enumerate(ps_):
                store16(a, pdg + 4 * q, V_E, SRD_C, S_E0, p)
            store16(a, pdu, V_E + 2, SRD_C, S_E0, ps_[0])
            store16(a, gf, V_E + 2, SRD_C, S_E0, ps_[1])
            seq.extend([("S", r)] * 4)
        a("s_nop 1")                        # store data read before the next round rewrites it
        if half == 1:
            a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_E1)}")


def epilogue_swiglu_bwd_r4(a: Asm):
    """acc = ds (never stored).  gu rows: gate at n, up at F + n; pairs p of
    fragments give 8 consecutive n per lane: 16-byte loads and stores."""
    a(f"s_mov_b32 {sr(S_E0)}, 0")                             # dgu row block
    a(f"s_lshl_b32 {sr(S_E1)}, {sr(S_LDC)}, 4")
    a(f"s_mov_b32 {sr(S_T0)}, 0")                             # gu row block
    a(f"s_lshl_b32 {sr(S_T1)}, {sr(S_LDS)}, 4")
    a(f"v_mov_b32 {vr(V_E + 4)}, {-LOG2E!r}")
    for j in range(8):
        for half in range(2):               # pairs p = 2 half, 2 half + 1
            ps_ = (2 * half, 2 * half + 1)
            lg, lu = V_E + 8, V_E + 16      # loaded packed gate / up (4 regs per pair)
            for q, p in enumerate(ps_):
                a(f"buffer_load_dwordx4 {vr(lg + 4 * q, 4)}, {vr(V_E + 1)}, {sr(SRD_S, 4)}, {sr(S_T0)} offen offset:{64 * p}")
                a(f"buffer_load_dwordx4 {vr(lu + 4 * q, 4)}, {vr(V_E + 3)}, {sr(SRD_S, 4)}, {sr(S_T0)} offen offset:{64 * p}")
            d = V_E + 24                    # 16 f32: ds
            for q, p in enumerate(ps_):
                read_pair(a, d + 8 * q, p, j)
            pd = V_E + 40                   # bf16-rounded ds, then unpacked
            for q in range(2):
                cvt_pack8(a, pd + 4 * q, d + 8 * q)
            for q in range(2):
                unpack8(a, d + 8 * q, pd + 4 * q)
            a("s_waitcnt vmcnt(0)")
            gf, uf = V_E + 48, V_E + 64
            for q in range(2):
                unpack8(a, gf + 8 * q, lg + 4 * q)
                unpack8(a, uf + 8 * q, lu + 4 * q)
            sg, tmp = V_E + 80, V_E + 96
            for e in range(16):             # sg = 1 / (1 + exp(-g))
                a(f"v_mul_f32 {vr(sg + e)}, {vr(V_E + 4)}, {vr(gf + e)}")
            for e in range(16):
                a(f"v_exp_f32 {vr(sg + e)}, {vr(sg + e)}")
            for e in range(16):
                a(f"v_add_f32 {vr(sg + e)}, 1.0, {vr(sg + e)}")
            for e in range(16):
                a(f"v_rcp_f32 {vr(sg + e)}, {vr(sg + e)}")
            for e in range(16):             # du = d * g * sg  -> tmp
                a(f"v_mul_f32 {vr(tmp + e)}, {vr(d + e)}, {vr(gf + e)}")
                a(f"v_mul_f32 {vr(tmp + e)}, {vr(tmp + e)}, {vr(sg + e)}")
            for e in range(16):             # dg = d * u * sg * (1 + g (1 - sg)) -> uf
                a(f"v_sub_f32 {vr(lg)}, 1.0, {vr(sg + e)}")
                a(f"v_fma_f32 {vr(lg)}, {vr(gf + e)}, {vr(lg)}, 1.0")
                a(f"v_mul_f32 {vr(uf + e)}, {vr(d + e)}, {vr(uf + e)}")
                a(f"v_mul_f32 {vr(uf + e)}, {vr(uf + e)}, {vr(sg + e)}")
                a(f"v_mul_f32 {vr(uf + e)}, {vr(uf + e)}, {vr(lg)}")
            pdg, pdu = V_E + 40, V_E + 112  # 8 + 4 regs: reuse gf for the last du pair
            for q in range(2):
                cvt_pack8(a, pdg + 4 * q, uf + 8 * q)
            cvt_pack8(a, pdu, tmp)
            cvt_pack8(a, gf, tmp + 8)
            for q, p in enumerate(ps_):
                store16(a, pdg + 4 * q, V_E, SRD_C, S_E0, p)
            store16(a, pdu, V_E + 2, SRD_C, S_E0, ps_[0])
            store16(a, gf, V_E + 2, SRD_C, S_E0, ps_[1])
            a("s_waitcnt vmcnt(0)")         # scratch registers are reused next round
        a(f"s_add_u32 {sr(S_E0)}, {sr(S_E0)}, {sr(S_E1)}")
        a(f"s_add_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_T1)}")


# ---------------------------------------------------------------- kernel
def kernel(epi: str, trace: bool = False, variant: str = "") -> tuple[str, str]:
    """trace=True: the diagnostic trace variant of the plain kernel (markers
    into a host-coherent buffer in the S slot; toa_gemm_tn_asm_trace).
    variant: an A/B arm of the plain kernel (PLAIN_VARIANTS)."""
    name = "toa_gemm_tn_asm_trace" if trace else f"toa_gemm_tn_asm_{epi}" + (f"_{variant}" if variant else "")
    if SCHED["defer"]:
        assert epi == "plain" and not trace and not SCHED["timing"] and SCHED["persist"] and SCHED["map"]
        return kernel_defer(name)
    if SCHED["timing"]:
        name = "toa_gemm_tn_asm_timing" + ("" if SCHED["timing"] == 1 else str(SCHED["timing"]))
    a = Asm(prefix=("trace_" if trace else epi + "_" + (variant + "_" if variant else "")))
    tb = (lambda base: base) if trace else (lambda base: 0)
    a.raw(f".globl {name}")
    a.raw(".p2align 8")
    a.raw(f".type {name},@function")
    a.raw(f"{name}:")
    prologue(a, epi)
    timing = SCHED["timing"]
    if timing:
        a(f"s_memtime {sr(S_T_START, 2)}")
        for k in range(3):
            a(f"s_mov_b32 {sr(S_ACC + k)}, 0")
    if trace:
        for ins in trace_setup(a) + trace_mark(1):
            a(ins)
    # --- prologue DMA: tile 0 -> stage 0, tile 1 -> stage 1
    prologue_dma(a)
    if SCHED["zero_late"]:
        # 256 accumulator writes while the first tiles are in flight, not
        # ahead of their DMA (~1k issue cycles per tile off the critical path)
        zero_acc(a)
    # both stages toggled twice: M0 bases are back at stage 0 for tile 2
    a("s_waitcnt vmcnt(16)")                       # own tile-0 pieces
    a("s_barrier")                                 # everyone's
    if trace:
        for ins in trace_mark(2):
            a(ins)
    if epi == "plain" and not trace and not variant:
        stage_exit(a, 1)
    persist = SCHED["persist"]
    assert not persist or (not trace and not SCHED["timing"])
    l_tile = a.fresh("tile")
    if persist:
        a.label(l_tile)
    for j in range(8):
        a(frag_read("x", j, 0))
    for i in range(8):
        a(frag_read("w", i, 0))
    a("s_waitcnt lgkmcnt(0)")
    a(f"s_sub_u32 {sr(S_LOOP)}, {sr(S_KT)}, 2")
    l_loop, l_tail = a.fresh("loop"), a.fresh("tail")
    a(f"s_cmp_eq_u32 {sr(S_LOOP)}, 0")
    a(f"s_cbranch_scc1 {l_tail}")
    dual = SCHED["dual"]
    if dual:
        # two loop bodies, picked by the SIMD id's low bit (HW_ID[4]): the
        # waves of SIMDs 1 and 3 run the `dual` map, whose DMA pieces and
        # reads sit one MFMA away from the others'.  Both bodies have the
        # same barriers, so the workgroup stays in step.
        assert SCHED["map"] and not SCHED["timing"]
        l_loop1 = a.fresh("loop1")
        a(f"s_getreg_b32 {sr(S_T0)}, hwreg(HW_REG_HW_ID, 4, 1)")
        a(f"s_cmp_eq_u32 {sr(S_T0)}, 0")
        a(f"s_cbranch_scc0 {l_loop1}")
    if SCHED["align"]:
        a(".p2alignl 6, 0xbf800000")   # loop head on a 64-byte boundary (s_nop padding)
    a.label(l_loop)
    it = iteration_map if SCHED["map"] else iteration
    it(a, with_dma=True, next_reads=True, vm_after_dma=16, trace_base=tb(100))
    a(f"s_sub_u32 {sr(S_LOOP)}, {sr(S_LOOP)}, 1")
    a(f"s_cmp_eq_u32 {sr(S_LOOP)}, 0")
    a(f"s_cbranch_scc0 {l_loop}")
    if dual:
        a(f"s_branch {l_tail}")
        if SCHED["align"]:
            a(".p2alignl 6, 0xbf800000")
        a.label(l_loop1)
        iteration_map(a, with_dma=True, next_reads=True, vm_after_dma=16, mapname=dual)
        a(f"s_sub_u32 {sr(S_LOOP)}, {sr(S_LOOP)}, 1")
        a(f"s_cmp_eq_u32 {sr(S_LOOP)}, 0")
        a(f"s_cbranch_scc0 {l_loop1}")
    a.label(l_tail)
    it(a, with_dma=False, next_reads=True, vm_after_dma=0, trace_base=tb(200))
    it(a, with_dma=False, next_reads=False, vm_after_dma=0, trace_base=tb(300))
    if epi == "plain" and not trace and not variant:
        stage_exit(a, 2)
    if timing:
        a(_stamp(0))                                # main loop done
    # MFMA results -> VALU reads: let the last MFMAs retire
    a("s_nop 15")
    a("s_nop 15")
    if trace:
        for ins in trace_mark(9000):
            a(ins)
    if persist:
        persistent_next(a, epi, l_tile)
    if not SCHED["epi_none"]:   # (the "none" arm: DIAGNOSTIC, the main loop alone)
        if epi != "rope":
            epi_offsets(a, epi)
        {"plain": epilogue_plain, "swiglu_fwd": epilogue_swiglu_fwd, "swiglu_bwd": epilogue_swiglu_bwd,
         "rope": epilogue_rope, "delta": epilogue_delta, "resadd": epilogue_resadd}[epi](a)
    if trace or timing or SCHED["drain_end"]:
        a("s_waitcnt vmcnt(0)")
    # else: end with the epilogue's stores still in flight -- the wave's end
    # does not wait for them, so the next workgroup on this CU starts its
    # prologue while they drain (the hardware completes them)
    if timing:
        # record per (workgroup, wave): vm wait, X-free barrier, W-free barrier,
        # start -> loop end, epilogue, k-tiles, workgroup id, 0 (cycles)
        a(_stamp(1))
        a("s_waitcnt lgkmcnt(0)")
        a(f"s_sub_u32 {sr(S_TMT + 4)}, {sr(S_TMT)}, {sr(S_T_START)}")
        a(f"s_sub_u32 {sr(S_TMT + 5)}, {sr(S_TMT + 2)}, {sr(S_TMT)}")
        for ins in trace_setup(a):
            a(ins)
        for k, src in enumerate((sr(S_ACC), sr(S_ACC + 1), sr(S_ACC + 2), sr(S_TMT + 4), sr(S_TMT + 5), sr(S_KT),
                                 "s2", "0")):
            a(f"v_mov_b32 {vr(V_T + 2)}, {src}")
            a(f"buffer_store_dword {vr(V_T + 2)}, {vr(V_T + 3)}, {sr(SRD_S, 4)}, 0 offen offset:{4 * k}")
        a("s_waitcnt vmcnt(0)")
    if trace:
        for ins in trace_setup(a)[-3:] + trace_mark(9999):
            a(ins)
    a.label(a.abort)
    a("s_endpgm")
    if epi == "plain" and not trace and not variant:
        a.label(a.stage_exit)
        a("s_waitcnt vmcnt(0)")
        a("s_endpgm")
    a.raw(f".size {name}, .-{name}")
    body = "\n".join(a.out)
    # the delta epilogue's partial sums: 4 waves x 256 B of LDS past the stages
    desc, meta = _descriptor(name, lds_bytes=LDS_BYTES + 1024 if epi == "delta" else None)
    return body + "\n" + desc, meta


def prologue_dma(a: Asm):
    """k-tiles 0 and 1 of the tile -> stages 0 and 1 (M0 bases end at stage 0)."""
    for _ in range(2):
        for half in ("x", "w"):
            for j in range(8):
                for ins in dma(a, half, j):
                    a(ins)
            for ins in advance(half):
                a(ins)
        a(f"s_xor_b32 {sr(S_M0X)}, {sr(S_M0X)}, {sr(S_M0XT)}")
        a(f"s_xor_b32 {sr(S_M0W)}, {sr(S_M0W)}, {sr(S_M0WT)}")


def persistent_next(a: Asm, epi: str, l_tile: str):
    """Persistent arms: this workgroup's next tile is S_ITER + grid.  If there
    is one, its first two k-tiles are staged (every wave's reads of the
    current tile are done: barrier) BEFORE the current tile's epilogue, so
    their flight hides under the epilogue; then the epilogue, the next tile's
    C resource, zeroed accumulators, and back to the tile loop."""
    l_last, l_even, l_par = a.fresh("last"), a.fresh("even"), a.fresh("par")
    # stage parity back to 0: the M0 bases toggled KT times this tile, the read bases KT - 1
    a(f"s_bitcmp1_b32 {sr(S_KT)}, 0")
    a(f"s_cbranch_scc0 {l_even}")
    a(f"s_xor_b32 {sr(S_M0X)}, {sr(S_M0X)}, {sr(S_M0XT)}")
    a(f"s_xor_b32 {sr(S_M0W)}, {sr(S_M0W)}, {sr(S_M0WT)}")
    a(f"s_branch {l_par}")
    a.label(l_even)
    a(f"v_xor_b32 {vr(V_RX)}, {vr(V_RX)}, {vr(V_RXT)}")
    a(f"v_xor_b32 {vr(V_RW)}, {vr(V_RW)}, {vr(V_RWT)}")
    a.label(l_par)
    a(f"s_add_u32 {sr(S_ITER)}, {sr(S_ITER)}, {sr(S_GRID)}")
    a(f"s_mul_i32 {sr(S_T0)}, {sr(S_TM_N)}, {sr(S_TN_N)}")
    a(f"s_cmp_ge_u32 {sr(S_ITER)}, {sr(S_T0)}")
    a(f"s_cbranch_scc1 {l_last}")
    a("s_barrier")                                 # every wave done reading this tile's LDS
    tile_setup(a, epi, sr(S_ITER))                 # SRD_X / SRD_W / (S_TM, S_TN) of the next tile
    prologue_dma(a)
    epi_offsets(a, epi)
    n0 = len(a.out)
    {"plain": epilogue_plain, "swiglu_fwd": epilogue_swiglu_fwd, "swiglu_bwd": epilogue_swiglu_bwd}[epi](a)
    n_vm = sum(1 for ins in a.out[n0:] if ins.lstrip().startswith(("buffer_load", "buffer_store")))
    tile_c(a, epi)
    zero_acc(a)
    # the next tile's k-tile 0 landed: k-tile 1's 16 pieces and the epilogue's
    # loads / stores are younger (plain: 32 stores -> 48; the SwiGLU epilogues
    # issue more than the counter holds, and their own waits already retired
    # everything up to their last load: 63 is then no wait at all)
    a(f"s_waitcnt vmcnt({min(63, 16 + n_vm)})")
    a("s_barrier")
    a(f"s_branch {l_tile}")
    a.label(l_last)


TRACE_REC = 32   # bytes per (workgroup, wave) trace record


def trace_setup(a: Asm) -> list[str]:
    """Diagnostic trace kernel only: SRD over the host-coherent trace buffer
    (pointer in the S slot), V_T+3 = this wave's record offset."""
    return [f"s_mov_b32 {sr(SRD_S)}, {sr(S_S)}", f"s_mov_b32 {sr(SRD_S + 1)}, {sr(S_S + 1)}",
            f"s_mul_i32 {sr(SRD_S + 2)}, {sr(S_TM_N)}, {sr(S_TN_N)}",
            f"s_mul_i32 {sr(SRD_S + 2)}, {sr(SRD_S + 2)}, {4 * TRACE_REC}",
            f"s_mov_b32 {sr(SRD_S + 3)}, 0x20000", "s_mov_b32 s71, 0",
            f"v_lshrrev_b32 {vr(V_T + 3)}, 6, {vr(V_TID)}",
            f"v_lshl_add_u32 {vr(V_T + 3)}, s2, 2, {vr(V_T + 3)}",
            f"v_mul_u32_u24 {vr(V_T + 3)}, {TRACE_REC}, {vr(V_T + 3)}"]


def trace_mark(code: int) -> list[str]:
    """Record (code, loop counter, M0, SRD_X lo, SRD_W lo, M0 bases, seq) for
    this wave, system-coherent, drained: after a fault the host reads how far
    every wave got (scripts/asm_gemm_bench.py --trace)."""
    out = ["s_add_u32 s71, s71, 1"]
    for k, src in enumerate((str(code), sr(S_LOOP), "m0", sr(SRD_X), sr(SRD_W), sr(S_M0X), sr(S_M0W), "s71")):
        out.append(f"v_mov_b32 {vr(V_T + 2)}, {src}")
        out.append(f"buffer_store_dword {vr(V_T + 2)}, {vr(V_T + 3)}, {sr(SRD_S, 4)}, 0 offen offset:{4 * k} sc0 sc1")
    out.append("s_waitcnt vmcnt(0)")
    return out


def stage_exit(a: Asm, stage: int):
    """Diagnostic (plain kernel only, whose fc argument is otherwise unused):
    fc == stage ends the workgroup here, after draining its DMA -- bisects a
    hardware fault by how far the kernel gets (scripts/asm_gemm_bench.py)."""
    a(f"s_cmp_eq_u32 {sr(S_FC)}, {stage}")
    a(f"s_cbranch_scc1 {a.stage_exit}")


def _descriptor(name: str, lds_bytes: int | None = None, n_sgpr: int | None = None,
                karg_bytes: int | None = None) -> tuple[str, str]:
    LDS_BYTES = globals()["LDS_BYTES"] if lds_bytes is None else lds_bytes  # noqa: N806
    N_SGPR = globals()["N_SGPR"] if n_sgpr is None else n_sgpr  # noqa: N806
    KARG_BYTES = globals()["KARG_BYTES"] if karg_bytes is None else karg_bytes  # noqa: N806
    desc = f"""
.rodata
.p2align 6
.amdhsa_kernel {name}
  .amdhsa_group_segment_fixed_size {LDS_BYTES}
  .amdhsa_private_segment_fixed_size 0
  .amdhsa_kernarg_size {KARG_BYTES}
  .amdhsa_user_sgpr_count 2
  .amdhsa_user_sgpr_kernarg_segment_ptr 1
  .amdhsa_system_sgpr_workgroup_id_x 1
  .amdhsa_system_vgpr_workitem_id 0
  .amdhsa_next_free_vgpr 512
  .amdhsa_next_free_sgpr {N_SGPR}
  .amdhsa_accum_offset 256
  .amdhsa_reserve_vcc 1
  .amdhsa_float_denorm_mode_32 3
  .amdhsa_float_denorm_mode_16_64 3
  .amdhsa_dx10_clamp 1
  .amdhsa_ieee_mode 1
.end_amdhsa_kernel
.text
"""
    meta = f"""  - .args:
      - .offset: 0
        .size: {KARG_BYTES}
        .value_kind: by_value
    .group_segment_fixed_size: {LDS_BYTES}
    .kernarg_segment_align: 8
    .kernarg_segment_size: {KARG_BYTES}
    .max_flat_workgroup_size: 256
    .name: {name}
    .private_segment_fixed_size: 0
    .sgpr_count: {N_SGPR + 6}
    .sgpr_spill_count: 0
    .symbol: {name}.kd
    .vgpr_count: 512
    .agpr_count: 256
    .vgpr_spill_count: 0
    .wavefront_size: 64
    .uniform_work_group_size: 1
    .uses_dynamic_stack: false
    .language: OpenCL C
    .language_version:
      - 2
      - 0
"""
    return desc, meta


PROBE_SGPRS = 72   # s0..s71: what the plain prologue writes (the timing kernel's s72.. are not dumped)
PROBE_MAGIC = (0x626F7270, 0x31657461)   # "prob" "ate1" in the fw / fc argument slots


def probe_kernel() -> tuple[str, str]:
    """Diagnostic kernel: the plain kernel's prologue, then a dump of every
    SGPR s0..s71 and, per thread, the DMA / fragment / epilogue offsets to
    the buffer in the S argument slot -- ONLY when fw / fc hold PROBE_MAGIC
    (a kernarg block that did not arrive intact stores nothing).  Compared
    with the emulator's dump of the same prologue (tests/test_asm_gemm.py,
    scripts/asm_gemm_bench.py --probe)."""
    name = "toa_gemm_tn_asm_probe"
    a = Asm(prefix="probe_")
    a.raw(f".globl {name}")
    a.raw(".p2align 8")
    a.raw(f".type {name},@function")
    a.raw(f"{name}:")
    prologue(a, "plain")
    epi_offsets(a, "plain")
    end = a.fresh("end")
    a(f"s_cmp_eq_u32 {sr(S_FW)}, {PROBE_MAGIC[0]:#x}")
    a(f"s_cbranch_scc0 {end}")
    a(f"s_cmp_eq_u32 {sr(S_FC)}, {PROBE_MAGIC[1]:#x}")
    a(f"s_cbranch_scc0 {end}")
    # workgroup b dumps to S + b * PROBE_WORDS * 4
    a(f"s_mul_i32 {sr(S_E0)}, s2, {PROBE_WORDS * 4}")
    a(f"s_add_u32 {sr(SRD_S)}, {sr(S_S)}, {sr(S_E0)}")
    a(f"s_addc_u32 {sr(SRD_S + 1)}, {sr(S_S + 1)}, 0")
    a(f"s_mov_b32 {sr(SRD_S + 2)}, {PROBE_WORDS * 4}")
    a(f"s_mov_b32 {sr(SRD_S + 3)}, 0x20000")
    a(f"v_mov_b32 {vr(V_T + 1)}, 0")
    for r in range(PROBE_SGPRS):
        if r in (SRD_S, SRD_S + 1, SRD_S + 2, SRD_S + 3, S_E0):
            continue
        a(f"v_mov_b32 {vr(V_T)}, {sr(r)}")
        a(f"buffer_store_dword {vr(V_T)}, {vr(V_T + 1)}, {sr(SRD_S, 4)}, 0 offen offset:{4 * r}")
    a(f"v_mov_b32 {vr(V_T)}, m0")
    a(f"buffer_store_dword {vr(V_T)}, {vr(V_T + 1)}, {sr(SRD_S, 4)}, 0 offen offset:{4 * PROBE_SGPRS}")
    # per thread: 8 words at 4 * (PROBE_VBASE + 8 tid)
    a(f"v_lshlrev_b32 {vr(V_T + 1)}, 5, {vr(V_TID)}")
    for k, reg in enumerate((V_DX, V_DW, V_RX, V_RW, V_RXT, V_RWT, V_E, V_TID)):
        a(f"buffer_store_dword {vr(reg)}, {vr(V_T + 1)}, {sr(SRD_S, 4)}, 0 offen offset:{4 * (PROBE_VBASE + k)}")
    a("s_waitcnt vmcnt(0)")
    a.label(end)
    a.label(a.abort)
    a("s_endpgm")
    a.raw(f".size {name}, .-{name}")
    body = "\n".join(a.out)
    desc, meta = _descriptor(name)
    return body + "\n" + desc, meta


PROBE_VBASE = 128
PROBE_WORDS = PROBE_VBASE + 8 * 256


# A/B arms of the plain kernel, launched by index through toa_gemm_asm_variant
# (scripts/asm_gemm_bench.py --variants): layout / schedule knobs against the
# product kernel, measured in one process.  Index 0 is the product kernel.
PLAIN_VARIANTS = (
    ("v1", {"map": "spread", "zero_late": False}),   # the round-4 product kernel
    ("v2", {"zero_late": False}),           # accumulators zeroed ahead of the prologue DMA (round 4)
    ("v3", {"persist": True}),              # persistent: a workgroup per CU walks its tiles, next tile staged under the epilogue
    ("v4", {"nostore": True, "diag": True}),  # DIAGNOSTIC: no C stores (what the epilogue's stores cost); C is not written
    ("v5", {"dual": "lib1"}),               # the library's second loop body on odd SIMDs
    ("v6", {"store_same": True, "diag": True}),  # DIAGNOSTIC: every workgroup stores tile (0, 0) (L2-hot writes)
    ("v7", {"store_nt": False}),            # C stores without the non-temporal hint
    ("v8", {"persist": True, "store_nt": False}),
    ("v9", {"persist": True, "defer": True}),   # persistent, C stores deferred into the next tile's first k-tile
)
# measured (profiles/r4_asm_gemm/ab1..diag2): MFMAs on 8-byte boundaries, ending
# with the epilogue's stores in flight, two barriers per tile and the wait 16
# MFMAs earlier all within noise (+-1.5 %); LDS lines of 1040 B (same speed
# despite 2-way read conflicts), DMA pieces bunched after each barrier
# (-2..-4 %) and groups of 16 row tiles (-1..-7 %) rejected; groups of 4, the
# next-tile wait at MFMA 95 and the X-free barrier 16 MFMAs after the last X
# read taken into the product kernel (+1..+4 %); an L2 prefetch of the tile two
# beyond the DMA (one 4-B load per line, its own bounded resources) -16..-24 %
# (profiles/r4_asm_gemm/ab3): the extra loads share the counted vmcnt waits.
# Round 5 (profiles/r5_lib/forms.log): the "lib0" placement (barriers one MFMA
# after their waits, M0 / resource advances one MFMA after the pieces) +0.5..2 %
# over "spread" at every form, taken into the product kernel; the library's
# second loop body for odd SIMDs (with and without MFMA alignment) -1..-3 %.


# DIAGNOSTIC arms of the fused SwiGLU backward (wrong outputs by design),
# launched by index through toa_gemm_asm_swiglu_bwd_variant: where the fused
# epilogue's time goes (scripts/asm_gemm_bench.py --swiglu-variants).
# Persistent fused SwiGLU GEMMs (one workgroup per CU walks its tiles; the
# next tile's first two k-tiles are staged before the current tile's
# epilogue, so its gu loads / dgu stores overlap that DMA instead of a fresh
# workgroup's prologue): A/B arms with correct outputs, launched by
# toa_gemm_asm_set_swiglu_persist.
SWIGLU_PERSIST_VARIANTS = (("swiglu_fwd", "p1", {"persist": True}), ("swiglu_bwd", "p1", {"persist": True}))

SWIGLU_BWD_VARIANTS = (
    ("b1", {"epi_none": True}),          # the main loop alone
    ("b2", {"epi_noload": True}),        # math + stores, no gu loads
    ("b3", {"epi_novalu": True}),        # gu loads + dgu stores, no math
    ("b4", {"epi_nostore": True}),       # loads + math, no stores
    ("b5", {"epi_noload": True, "epi_nostore": True}),   # math alone
)


def _with_knobs(knobs: dict, fn):
    """Run fn() with the layout globals / SCHED entries in `knobs` overridden."""
    g = globals()
    saved = {k: g[k] for k in ("LINE", "HALF", "STAGE", "LDS_BYTES")}
    saved_sched = dict(SCHED)
    try:
        if "LINE" in knobs:
            g["LINE"] = knobs["LINE"]
            g["HALF"] = 32 * g["LINE"]
            g["STAGE"] = 2 * g["HALF"]
            g["LDS_BYTES"] = 2 * g["STAGE"]
        SCHED.update({k: v for k, v in knobs.items() if k in SCHED})
        return fn()
    finally:
        g.update(saved)
        SCHED.clear()
        SCHED.update(saved_sched)


def generate() -> str:
    parts = ['.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', ".amdhsa_code_object_version 5", ".text"]
    metas = []
    for epi in EPIS:
        body, meta = kernel(epi)
        parts.append(body)
        metas.append(meta)
    for epi in ("swiglu_fwd", "swiglu_bwd"):   # round-4 epilogues (per-round drains): in-model A/B arms
        body, meta = _with_knobs({"epi_pipe": False, "epi_pk": False, "epi_f32s": False},
                                 lambda: kernel(epi, variant="r4"))
        parts.append(body)
        metas.append(meta)
    for vname, knobs in PLAIN_VARIANTS:
        body, meta = _with_knobs(knobs, lambda: kernel("plain", variant=vname))
        parts.append(body)
        metas.append(meta)
    for vname, knobs in SWIGLU_BWD_VARIANTS:
        body, meta = _with_knobs(knobs, lambda: kernel("swiglu_bwd", variant=vname))
        parts.append(body)
        metas.append(meta)
    for epi, vname, knobs in SWIGLU_PERSIST_VARIANTS:
        body, meta = _with_knobs(knobs, lambda: kernel(epi, variant=vname))
        parts.append(body)
        metas.append(meta)
    import attn_gen   # the attention forward and the weight-gradient kernel share this code object
    import wgrad_gen  # (lazy: both import this module)

    def wgrad_round4():
        saved = dict(wgrad_gen.KNOBS)
        wgrad_gen.KNOBS.update(map="spread", zero_late=False)
        try:
            return wgrad_gen.kernel("v1")
        finally:
            wgrad_gen.KNOBS.clear()
            wgrad_gen.KNOBS.update(saved)

    import attn_bwd_gen  # the attention dK / dV backward, same code object

    for body, meta in (wgrad_gen.kernel(), wgrad_round4(), *attn_gen.all_kernels(), probe_kernel(), kernel("plain", trace=True),
                       _with_knobs({"timing": 1}, lambda: kernel("plain", variant="timing")),
                       _with_knobs({"timing": 2}, lambda: kernel("plain", variant="timing2")),
                       *attn_bwd_gen.all_kernels()):
        parts.append(body)
        metas.append(meta)
    # what hipcc emits after the last kernel: s_nop padding, so the
    # instruction prefetcher never runs off the end of the code object
    parts.append(".text\n.p2alignl 6, 3212836864\n.fill 256, 4, 3212836864")   # s_nop 0
    parts.append(".amdgpu_metadata\n---\namdhsa.version:\n  - 1\n  - 2\namdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.kernels:\n" + "".join(metas)
                 + "...\n.end_amdgpu_metadata")
    return "\n".join(parts) + "\n"


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else "gemm_tn_asm.s"
    with open(out, "w") as f:
        f.write(generate())
