#!/usr/bin/env python3
"""Generator of the hand-written gfx950 causal flash-attention dK / dV
backward (the dS form: every dS block is also stored for the dQ GEMM).

Emitted into the same code object as the GEMMs (gemm_gen.generate() calls
all_kernels() here); host side: toa_attn_dkdv_asm in csrc/hip/gemm_asm.hip,
which the dS-form backward (csrc/hip/attention.hip dkdv_ds_launch) calls for
the shapes it takes, in place of attn_bwd_dkdv_ds_kernel.

    P   = exp2(S * c - lse log2 e),  S = Q K^T          (c = scale log2 e)
    dS  = P * (dO V^T - delta)
    dV += P^T dO,   dK += scale dS^T Q     (summed over the rep query heads of
                                            the kv head and every query >= key)

bf16 Q [B, H, S, 128], K / V [B, Hk, S, 128], dO [B, H, S, 128] or
[B, S, H, 128] (flags bit 0); -lse log2 e and -delta fp32 [B, H, S] (the
delta pass, attn_delta_kernel); dS blocks in the dQ GEMM's packed layout
(attention.hip attn_bwd_dqg_kernel); dK / dV [B, Hk, S, 128], or with flags
bit 1 the k / v parts of d(qkv) rows [B S, H3 128] with RoPE's backward
rotation applied to dK (cos / sin [S, 64] fp32).  S % 256 == 0.

Why assembly (docs/kernels.md, round 5): the HIP kernel runs two waves per
SIMD with K / V in LDS, so every 32 x 32 sub-tile re-reads them and the
compiler serialises each sub-tile's softmax VALU between its MFMA halves:
48 % MFMA busy, ~3750 cycles per 64 MFMAs of a SIMD (docs/kernels.md round 4,
the ping-pong that would overlap the two waves spills under hipcc).  Here
one wave per SIMD owns the whole register file and every instruction is
placed by the list scheduler shared with the forward (attn_gen.schedule):

  workgroup  256 threads = 4 waves, 128 keys of one (batch, kv head); wave w
             owns keys 32 w .. + 31 (key on the MFMA lane); heaviest key
             blocks first (kb = 0 sees every query tile)
  registers  dV^T / dK^T accumulators a[0:127]; the wave's K and V rows as
             the B operands of S / dP, loaded once, a[128:191]
  step       one 64-query tile of one query head = two 32-query blocks n;
             per block: SD(n) = 8 S + 8 dP MFMAs (A = Q / dO rows from LDS,
             dP's accumulator initialised with -delta), E(n) = the VALU
             (P = exp2(S c - lse'), causal mask, dS = P dP', bf16 packs, the
             dS block store), KV(n) = 8 dV^T + 8 dK^T MFMAs (A = dO^T / Q^T
             by ds_read_b64_tr_b16, B = P / dS straight from the packs)
  pipeline   one loop iteration = one step it: MFMAs KV(2 it), SD(2 it + 2),
             KV(2 it + 1), SD(2 it + 3); fillers E(2 it + 1), E(2 it + 2),
             all fragment reads (rings of 6), the DMA of tile it + 2 and ONE
             barrier; E(n) runs while the matrix core does KV(n - 1) and
             SD(n + 1), so the exponentials never stand alone
  staging    Q / dO tiles (16 KiB each) and the -lse / -delta rows by LDS-DMA
             (buffer_load ... lds) into a ring of three tile buffers in the
             XOR-swizzled rt_off image of attention.hip (conflict-free row
             and transposed reads): tile it + 2 is issued right after the
             barrier of iteration it, a whole step ahead of its use
  causal     only the first two steps of every query-head pass touch the
             diagonal: their E(n) carry the mask (loop-body variants); a
             block wholly above the diagonal computes zeros and its dS store
             is dropped by a zero-size buffer resource

Reference anchor: SURVEY.md K5 (attention kernels of the flagship model;
the reference itself has no attention kernel).  Checked instruction by
instruction on the CPU by csrc/asm/emu.py (tests/test_asm_attn_bwd.py)
against an fp64 backward, and against the HIP kernel / fp32 on the GPU
(tests/test_ops_gpu.py).
"""
from __future__ import annotations

import sys

import attn_gen as AG
import gemm_gen as G
from attn_gen import Item, schedule
from gemm_gen import Asm, ar, sr, vr

NAME = "toa_attn_dkdv_asm"
D = 128
ROWB = 2 * D             # bytes per Q / dO / K / V row
TQ = 64                  # query rows per step (one tile)
TILEB = TQ * ROWB        # 16 KiB
OFF_DO = TILEB           # dO tile after the Q tile
OFF_L = 2 * TILEB        # -lse log2 e row (256 B), then -delta (256 B)
BUFB = 33 * 1024         # one tile buffer (1 KiB aligned)
NBUF = 3
LDS_BYTES = NBUF * BUFB
RING = 6
G_BAR = 10               # the iteration's barrier: after MFMA 10 (inside KV(2 it))
DL_DMA = 40              # every DMA piece issued by this gap
KARG_BYTES = 144
KARG = {"Q": 0, "K": 8, "V": 16, "dO": 24, "NLSE": 32, "NDELTA": 40, "dK": 48, "dV": 56, "dS": 64,
        "cos": 72, "sin": 80, "dbg": 88, "B": 96, "H": 100, "Hk": 104, "S": 108, "scale": 112, "c": 116,
        "flags": 120, "rep": 124, "nkb": 128, "H3": 132}

# ---------------------------------------------------------------- SGPRs
S_Q, S_K, S_V, S_DO, S_NL, S_ND, S_DK, S_DV, S_DS, S_COS, S_SIN, S_DBG = range(4, 28, 2)
S_B, S_H, S_HK, S_S, S_SC, S_C, S_FL, S_REP, S_NKB, S_H3 = range(28, 38)
S_W, S_KB, S_BB, S_HKV, S_NQT, S_TOT, S_IT, S_MOD = range(38, 46)
S_HEAD, S_NMOD, S_NHEAD, S_DIT, S_DMOD, S_DHEAD, S_HS256, S_QS64 = range(46, 54)
S_DSTR, S_TB, S_SOFF, S_NBLK, S_TSOFF, S_LSOFF, S_LB, S_S4 = range(54, 62)
S_4KB, S_KI, S_32W, S_HQ0, S_NREC, S_DSO0, S_DSO1, S_DD0 = range(62, 70)
S_DD1, S_TOTM1 = 70, 71
SRD_DMA, SRD_LD, SRD_DS0, SRD_DS1, SRD_X = 72, 76, 80, 84, 88
S_LM0 = SRD_X + 2         # the -lse / -delta row's LDS base in a buffer (SRD_X is prologue-only)
S_T0 = 92                 # s92..s95 scratch
S_U = 96                  # s96, s97: srd64's own scratch
S_TM = 98                 # s98, s99: the timing arm's loop-start stamp (loop end: s[SRD_X:+1])
N_SGPR = 100

# ---------------------------------------------------------------- VGPRs
# Tile-buffer read offsets: set A (base 0) serves buffers 0 and 1 through the
# instructions' 16-bit offsets, set B (base 2 BUFB) buffer 2.
V_RRO = 1                 # v1..v8: Q / dO row-read offsets per k-step
V_LO = 9                  # -lse / -delta read offset
V_TRO, V_TRO8 = 10, 14    # v10..v13, v14..v17: transposed-read offsets per d tile
V_RRO_B, V_LO_B, V_TRO_B = 82, 90, 91
V_TRO8_B = (95, 96, 97, 20)
V_C2 = 18                 # v18, v19: c = scale log2 e twice (packed-math operand)
V_L4 = 22                 # lane * 4 (the -lse / -delta row DMA)
V_DSO = 23                # dS store lane offset: key 16 + query half 8 (8-B stores) / + 512 (16-B stores)
V_MD0, V_MD = 24, 25      # mask: r - 4 hh, and + (first key - first query) of the block
V_T = 26                  # v26..v33 scratch
V_SF = 34                 # Q / dO fragment ring: 6 x 4
V_KF = 58                 # dO^T / Q^T fragment ring: 6 x 4
V_L = 98                  # -lse log2 e per block parity: 2 x 16
V_PW = 130                # P packs per parity: 2 x 8
V_SW = 146                # dS packs per parity: 2 x 8
V_SB = 162                # S (16) + dP (16) per parity: 2 x 32
V_DMA = 226               # v226..v233: DMA source offsets of the wave's 8 pieces
V_X = 234                 # v234..v255 scratch (prologue / epilogue; in the loop v234..v249 the 16-B dS store staging)

# AGPRs: dV^T a[0:63], dK^T a[64:127] ([d tile] x 16), K / V B-operand
# fragments a[128:159] / a[160:191] ([k-step] x 4)
A_DV, A_DK, A_K, A_V = 0, 64, 128, 160

# Schedule knobs; the DIAGNOSTIC arms (VARIANTS) switch one mechanism off to
# price it in-process (scripts/attn_dkdv_arms.py): their outputs are wrong by
# construction and only their time is read.
KNOBS = {"bar": True, "vmwait": True, "lgkm": True, "exp": True, "dma": True, "valu": True, "lds": True,
         "timing": False, "merge": True, "pk": False, "dsst": True, "dswide": False,
         "gbar": G_BAR, "dldma": DL_DMA, "lead": 3}   # schedule parameters (the s* arms sweep them)
VARIANTS = (
    ("d1", {"lgkm": False}),                     # MFMAs do not wait for their LDS fragments
    ("d2", {"bar": False, "vmwait": False}),     # no per-iteration barrier nor DMA wait
    ("d3", {"exp": False}),                      # v_exp_f32 -> v_mov_b32
    ("d4", {"dma": False, "vmwait": False}),     # no Q / dO staging in the loop
    ("d5", {"valu": False}),                     # no softmax / dS VALU (stores kept)
    ("d6", {"lds": False, "lgkm": False}),       # no LDS fragment reads
    ("d7", {"lds": False, "lgkm": False, "valu": False, "dma": False, "vmwait": False, "bar": False}),  # MFMAs + SALU
    ("t1", {"timing": True}),                    # the product kernel + s_memtime stamps (same outputs)
    # schedule-parameter arms (correct outputs; A/B by time)
    ("s1", {"gbar": 6}),
    ("s2", {"gbar": 14}),
    ("s3", {"dldma": 28}),
    ("s4", {"lead": 2}),
    ("s5", {"lead": 5}),
    ("s6", {"merge": False}),
    ("s7", {"pk": True}),                        # round 5: P / dS on packed v_pk_fma / v_pk_mul pairs
    ("d8", {"dsst": False}),                     # DIAGNOSTIC: no dS block stores (the dQ GEMM's input)
    ("s8", {"dswide": True}),                    # 16-B dS stores by permlane32 swaps (2 per block): measured
                                                 # 0.8 % slower than the four 8-B ones (profiles/r6_dkdv/arms3.log)
)

MASK_C = AG.MASK_C        # register r's row offset in a 32x32 accumulator: (r & 3) + 8 (r >> 2)


def sbuf(p):              # S accumulator of parity p
    return V_SB + 32 * p


def dpbuf(p):             # dP accumulator of parity p
    return V_SB + 32 * p + 16


def srd64(a: Asm, dst: int, base: int, row: int, row_bytes: int, nrec):
    """dst = buffer resource at s[base] + s[row] * row_bytes, num_records nrec
    (an SGPR name or a literal); scratch s[S_U:S_U+1] only."""
    a(f"s_mul_hi_u32 {sr(S_U + 1)}, {sr(row)}, {row_bytes}")
    a(f"s_mul_i32 {sr(S_U)}, {sr(row)}, {row_bytes}")
    a(f"s_add_u32 {sr(dst)}, {sr(base)}, {sr(S_U)}")
    a(f"s_addc_u32 {sr(dst + 1)}, {sr(base + 1)}, {sr(S_U + 1)}")
    a(f"s_mov_b32 {sr(dst + 2)}, {nrec}")
    a(f"s_mov_b32 {sr(dst + 3)}, 0x20000")


LAST_USE = {i % RING: i for i in range(16)}   # ring slot -> the last of 16 fragments using it


def slot_rel(i: int, base: int, base_prev: int | None) -> int:
    """Earliest gap for fragment i of a 16-fragment stream starting at MFMA
    `base`: after the MFMA that last used its ring slot (the previous
    stream's, at base_prev, for the first RING; None = slot free)."""
    if i >= RING:
        return base + i - RING
    return -1 if base_prev is None else base_prev + LAST_USE[i]


def sf(i):
    return V_SF + 4 * (i % RING)


def kf(i):
    return V_KF + 4 * (i % RING)


def rro(buf: int, s: int) -> tuple[int, int]:
    """(offset register, immediate base) of row reads in tile buffer `buf`."""
    return (V_RRO + s, buf * BUFB) if buf < 2 else (V_RRO_B + s, 0)


def lo(buf: int) -> tuple[int, int]:
    return (V_LO, buf * BUFB) if buf < 2 else (V_LO_B, 0)


def tro(buf: int, dt: int, eight: bool) -> tuple[int, int]:
    if buf < 2:
        return (V_TRO8 if eight else V_TRO) + dt, buf * BUFB
    return (V_TRO8_B[dt] if eight else V_TRO_B + dt), 0


# ---------------------------------------------------------------- pieces
def sd_frag(i: int, m: int, buf: int) -> str:
    """SD fragment i (S / dP interleaved: i = 2 s + (0 Q | 1 dO)) of block half m."""
    s, od = divmod(i, 2)
    reg, b0 = rro(buf, s)
    return f"ds_read_b128 {vr(sf(i), 4)}, {vr(reg)} offset:{b0 + od * OFF_DO + 8192 * m} ; SF{i}"


def sd_mfmas(p: int) -> list:
    out = []
    for i in range(16):
        s, od = divmod(i, 2)
        if od == 0:
            c = "0" if s == 0 else vr(sbuf(p), 16)
            # the last S MFMA also waits for the -lse rows (E reads them next)
            tags = [f"SF{i}"] + (["LL"] if i == 14 else [])
            out.append((f"v_mfma_f32_32x32x16_bf16 {vr(sbuf(p), 16)}, {vr(sf(i), 4)}, {ar(A_K + 4 * s, 4)}, {c}",
                        tags))
        else:
            tags = [f"SF{i}"] + (["DL"] if s == 0 else [])
            out.append((f"v_mfma_f32_32x32x16_bf16 {vr(dpbuf(p), 16)}, {vr(sf(i), 4)}, {ar(A_V + 4 * s, 4)}, "
                        f"{vr(dpbuf(p), 16)}", tags))
    return out


def lse_delta_reads(p: int, m: int, buf: int) -> list[str]:
    """-lse log2 e rows into V_L[p], -delta into dP's accumulator (its
    initial value, so the MFMAs leave dP - delta)."""
    reg, b0 = lo(buf)
    out = []
    for g in range(4):
        out.append(f"ds_read_b128 {vr(V_L + 16 * p + 4 * g, 4)}, {vr(reg)} offset:{b0 + 128 * m + 32 * g} ; LL")
    for g in range(4):
        out.append(f"ds_read_b128 {vr(dpbuf(p) + 4 * g, 4)}, {vr(reg)} offset:{b0 + 256 + 128 * m + 32 * g} ; DL")
    return out


def kv_frag(i: int, m: int, buf: int) -> list[str]:
    """KV fragment i (i = 2 (4 s2 + dt) + (0 dO^T | 1 Q^T)) of block half m:
    two transposed reads, 4 queries each (the P / dS pack's query order)."""
    j, q = divmod(i, 2)
    s2, dt = divmod(j, 4)
    base = (0 if q else OFF_DO) + (32 * m + 16 * s2) * ROWB
    r0, b0 = tro(buf, dt, False)
    r8, b8 = tro(buf, dt, True)
    return [f"ds_read_b64_tr_b16 {vr(kf(i), 2)}, {vr(r0)} offset:{b0 + base} ; KF{i}",
            f"ds_read_b64_tr_b16 {vr(kf(i) + 2, 2)}, {vr(r8)} offset:{b8 + base} ; KF{i}"]


def kv_mfmas(p: int) -> list:
    out = []
    for i in range(16):
        j, q = divmod(i, 2)
        s2, dt = divmod(j, 4)
        if q == 0:
            acc, b = ar(A_DV + 16 * dt, 16), vr(V_PW + 8 * p + 4 * s2, 4)
        else:
            acc, b = ar(A_DK + 16 * dt, 16), vr(V_SW + 8 * p + 4 * s2, 4)
        out.append((f"v_mfma_f32_32x32x16_bf16 {acc}, {vr(kf(i), 4)}, {b}, {acc}", [f"KF{i}"]))
    return out


def e_items(p: int, masked: bool, rel: int, dl: int, stream: str, st_rel: int | None = None) -> list[Item]:
    """E(n) of parity p: P, mask, dS, packs, and the dS block store (SRD of
    parity p, block offset S_DSO<p>, mask shift S_DD<p>); the stores no
    earlier than gap st_rel."""
    items = []
    S0, P0, L0 = sbuf(p), dpbuf(p), V_L + 16 * p
    if masked:
        items.append(Item([f"v_add_u32 {vr(V_MD)}, {sr(S_DD0 if p == 0 else S_DD1)}, {vr(V_MD0)}"], 4, rel, dl, stream))
    pk = KNOBS["pk"]
    for j0 in range(0, 16, 4):
        if pk:
            ins = [f"v_pk_fma_f32 {vr(S0 + j, 2)}, {vr(S0 + j, 2)}, {vr(V_C2, 2)}, {vr(L0 + j, 2)}"
                   for j in range(j0, j0 + 4, 2)]
        else:   # scalar: beside MFMAs a packed f32 op costs more than two scalar ones (MI355X_MICROARCH.md
                # 'price of one filler'; -3.5 % per call at the bench shape, profiles/r6_dkdv)
            ins = [f"v_fma_f32 {vr(S0 + j)}, {vr(S0 + j)}, {vr(V_C2)}, {vr(L0 + j)}" for j in range(j0, j0 + 4)]
        ins += [f"v_exp_f32 {vr(S0 + j)}, {vr(S0 + j)}" if KNOBS["exp"] else f"v_mov_b32 {vr(S0 + j)}, {vr(S0 + j)}"
                for j in range(j0, j0 + 4)]
        items.append(Item(ins, 0, rel, dl, stream))
        if masked:   # key > query -> 0; each vcc pair kept together
            for j in range(j0, j0 + 4):
                items.append(Item([f"v_cmp_lt_i32 vcc, {MASK_C[j]}, {vr(V_MD)}",
                                   f"v_cndmask_b32 {vr(S0 + j)}, {vr(S0 + j)}, 0, vcc"], 8, rel, dl, stream, split=False))
        ins = [f"v_cvt_pk_bf16_f32 {vr(V_PW + 8 * p + j // 2)}, {vr(S0 + j)}, {vr(S0 + j + 1)}" for j in range(j0, j0 + 4, 2)]
        if pk:
            ins += [f"v_pk_mul_f32 {vr(P0 + j, 2)}, {vr(S0 + j, 2)}, {vr(P0 + j, 2)}" for j in range(j0, j0 + 4, 2)]
        else:
            ins += [f"v_mul_f32 {vr(P0 + j)}, {vr(S0 + j)}, {vr(P0 + j)}" for j in range(j0, j0 + 4)]
        ins += [f"v_cvt_pk_bf16_f32 {vr(V_SW + 8 * p + j // 2)}, {vr(P0 + j)}, {vr(P0 + j + 1)}" for j in range(j0, j0 + 4, 2)]
        items.append(Item(ins, 0, rel, dl, stream))
    # dS block store: the lane's 4 queries 8 g + 4 hh .. + 3 of key r are the
    # packs 2 g, 2 g + 1 -> 8 B at (g, key r, query half hh) of the block's
    # [8-query group][key][8 queries] layout (512 contiguous bytes per store)
    srd = SRD_DS0 if p == 0 else SRD_DS1
    dso = S_DSO0 if p == 0 else S_DSO1
    srel = rel if st_rel is None else max(rel, st_rel)
    nst = 0
    if KNOBS["dswide"]:
        # 16-B stores: the packs of groups 2k and 2k + 1 copied to scratch
        # (the packs themselves are KV(n)'s B operands) and one
        # v_permlane32_swap per dword, so lanes < 32 hold the 8 queries of
        # group 2k and lanes >= 32 those of group 2k + 1 for their key (the
        # lane offset V_DSO then steps 512 B per lane half): 2 stores per
        # block instead of 4.  The stores cost 14 % of the kernel (arm d8),
        # but not through their count: this arm (s8) is 0.8 % slower than the
        # product's four 8-B stores (profiles/r6_dkdv/arms3.log).  The movs of
        # both pairs go first, so a swap reads scratch written >= 3
        # instructions earlier.
        tmp = [V_X + 8 * p + 4 * k for k in range(2)]
        for k in range(2):
            items.append(Item([f"v_mov_b32 {vr(tmp[k] + e)}, {vr(V_SW + 8 * p + 4 * k + e)}" for e in range(4)], 0,
                              max(srel, rel + 1), max(srel, dl), stream))
        for k in range(2):
            items.append(Item([f"v_permlane32_swap_b32 {vr(tmp[k])}, {vr(tmp[k] + 2)}",
                               f"v_permlane32_swap_b32 {vr(tmp[k] + 1)}, {vr(tmp[k] + 3)}",
                               f"buffer_store_dwordx4 {vr(tmp[k], 4)}, {vr(V_DSO)}, {sr(srd, 4)}, {sr(dso)} "
                               f"offen offset:{1024 * k} nt"], 16, max(srel, rel + 1), max(srel, dl), stream,
                              split=False))
        nst = 4
    else:
        for g in range(4):
            items.append(Item([f"buffer_store_dwordx2 {vr(V_SW + 8 * p + 2 * g, 2)}, {vr(V_DSO)}, {sr(srd, 4)}, "
                               f"{sr(dso)} offen offset:{512 * g} nt"], 8, max(srel, rel + 1), max(srel, dl), stream))
        nst = 4
    if not KNOBS["dsst"]:   # DIAGNOSTIC: no dS block stores
        items = items[:-nst]
    if not KNOBS["valu"]:
        items = items[-nst:] if KNOBS["dsst"] else []
    for it in items:
        if it.cost == 0:
            it.cost = sum(AG.issue_cost(x) for x in it.ins)
    return items


def dso_step(mod: int, head: int) -> list[str]:
    """Both blocks of step (mod, head) for this wave: dS block byte offsets
    ((hq0 + head) NBLK + qi (qi + 1) / 2 + ki) 2048 (qi = 4 kb + 2 mod + m,
    ki = 4 kb + w) into S_DSO0 / S_DSO1, the store resources' sizes (0 =
    dropped: block wholly above the diagonal, qi < ki), and the mask shifts
    kw - qs = 32 w - 64 mod - 32 m into S_DD0 / S_DD1."""
    t0, t1, t2, t3 = S_T0, S_T0 + 1, S_T0 + 2, S_T0 + 3
    return [f"s_lshl_b32 {sr(t0)}, {sr(mod)}, 1",                   # 2 mod
            f"s_add_u32 {sr(t1)}, {sr(t0)}, {sr(S_4KB)}",           # qi0
            f"s_add_u32 {sr(t2)}, {sr(t1)}, 1",
            f"s_mul_i32 {sr(t1)}, {sr(t1)}, {sr(t2)}",
            f"s_lshr_b32 {sr(t1)}, {sr(t1)}, 1",                    # qi0 (qi0 + 1) / 2
            f"s_add_u32 {sr(t3)}, {sr(S_HQ0)}, {sr(head)}",
            f"s_mul_i32 {sr(t3)}, {sr(t3)}, {sr(S_NBLK)}",
            f"s_add_u32 {sr(t3)}, {sr(t3)}, {sr(S_KI)}",
            f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(t3)}",
            f"s_lshl_b32 {sr(S_DSO0)}, {sr(t1)}, 11",
            f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(t2)}",              # + qi0 + 1: block (qi0 + 1, ki)
            f"s_lshl_b32 {sr(S_DSO1)}, {sr(t1)}, 11",
            f"s_cmp_ge_u32 {sr(t0)}, {sr(S_W)}",
            f"s_cselect_b32 {sr(SRD_DS0 + 2)}, {sr(S_NREC)}, 0",
            f"s_add_u32 {sr(t0)}, {sr(t0)}, 1",
            f"s_cmp_ge_u32 {sr(t0)}, {sr(S_W)}",
            f"s_cselect_b32 {sr(SRD_DS1 + 2)}, {sr(S_NREC)}, 0",
            f"s_lshl_b32 {sr(t0)}, {sr(mod)}, 6",
            f"s_sub_u32 {sr(S_DD0)}, {sr(S_32W)}, {sr(t0)}",
            f"s_sub_u32 {sr(S_DD1)}, {sr(S_DD0)}, 32"]


def advance(mod: int, head: int) -> list[str]:
    """(mod, head) -> the next step's: mod + 1, wrapping to the next head
    (the compare's SCC is the head's carry)."""
    return [f"s_add_u32 {sr(mod)}, {sr(mod)}, 1",
            f"s_cmp_eq_u32 {sr(mod)}, {sr(S_NQT)}",
            f"s_cselect_b32 {sr(mod)}, 0, {sr(mod)}",
            f"s_addc_u32 {sr(head)}, {sr(head)}, 0"]


def dma_advance() -> list[str]:
    """The DMA step (S_DIT; coordinates S_DMOD / S_DHEAD) moves on unless it
    is the last step already (past the end the last tile is re-fetched into
    a buffer nobody reads: a constant DMA count per iteration)."""
    t = S_T0 + 2
    return [f"s_add_u32 {sr(t)}, {sr(S_DIT)}, 1",
            f"s_cmp_lt_u32 {sr(t)}, {sr(S_TOT)}",
            f"s_cselect_b32 {sr(S_DIT)}, {sr(t)}, {sr(S_DIT)}",
            f"s_cselect_b32 {sr(t)}, 1, 0",
            f"s_add_u32 {sr(S_DMOD)}, {sr(S_DMOD)}, {sr(t)}",
            f"s_cmp_eq_u32 {sr(S_DMOD)}, {sr(S_NQT)}",
            f"s_cselect_b32 {sr(S_DMOD)}, 0, {sr(S_DMOD)}",
            f"s_addc_u32 {sr(S_DHEAD)}, {sr(S_DHEAD)}, 0"]


def dma_setup() -> list[str]:
    """Tile (S_DMOD, S_DHEAD): source offset of this wave's pieces (S_TSOFF;
    the row part of each piece is in its VGPR offset) and of the -lse /
    -delta row (S_LSOFF)."""
    t0, t1 = S_T0, S_T0 + 1
    return [f"s_mul_i32 {sr(t0)}, {sr(S_DMOD)}, {sr(S_QS64)}",
            f"s_mul_i32 {sr(t1)}, {sr(S_DHEAD)}, {sr(S_HS256)}",
            f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(t1)}",
            f"s_add_u32 {sr(S_TSOFF)}, {sr(t0)}, {sr(S_TB)}",
            f"s_lshl_b32 {sr(t0)}, {sr(S_DMOD)}, 8",
            f"s_mul_i32 {sr(t1)}, {sr(S_DHEAD)}, {sr(S_S4)}",
            f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(t1)}",
            f"s_add_u32 {sr(S_LSOFF)}, {sr(t0)}, {sr(S_LB)}"]


def dma_pieces(buf: int) -> list[list[str]]:
    """This wave's 8 pieces of the Q (waves 0, 1) or dO (2, 3) tile into tile
    buffer `buf`, then its -lse (even waves) / -delta (odd) row."""
    out = []
    for u in range(8):
        out.append([f"s_add_u32 m0, {sr(S_SOFF)}, {buf * BUFB + 1024 * u}",
                    "s_nop 0",
                    f"buffer_load_dwordx4 {vr(V_DMA + u)}, {sr(SRD_DMA, 4)}, {sr(S_TSOFF)} offen lds"])
    out.append([f"s_add_u32 m0, {sr(S_LM0)}, {buf * BUFB}",
                "s_nop 0",
                f"buffer_load_dword {vr(V_L4)}, {sr(SRD_LD, 4)}, {sr(S_LSOFF)} offen lds"])
    return out


NPRE = 2                  # KV fragments of the next body read at the end of this one


def kv_read_items(base: int, m: int, buf: int, base_prev: int | None, pre: bool, stream: str) -> list[Item]:
    """KV fragment reads for MFMAs base .. base + 15 (fragments 0 .. NPRE - 1
    already read when pre)."""
    items = []
    for i in range(NPRE if pre else 0, 16):
        rel = slot_rel(i, base, base_prev)
        items.append(Item(kv_frag(i, m, buf), 8, rel, max(rel, base + i - KNOBS["lead"]), stream))
    return items


def kv_prefetch_items(rel: int, dl: int, m: int, buf: int) -> list[Item]:
    """Fragments 0 .. NPRE - 1 of the next body's KV, read in this body's
    last gaps (rel: after the MFMAs that last used their ring slots)."""
    return [Item(kv_frag(i, m, buf), 8, rel, dl, "kvpre") for i in range(NPRE)]


def sd_read_items(base: int, m: int, p: int, buf: int, rel0: int, base_prev: int | None, ld_rel: int,
                  stream: str) -> list[Item]:
    """SD(n) reads for MFMAs base .. base + 15: the -lse rows (by the last S
    MFMA) and -delta rows (into dP, by the first dP MFMA) no earlier than gap
    ld_rel, the Q / dO fragments no earlier than rel0."""
    lr = lse_delta_reads(p, m, buf)
    items = [Item(lr[4:], 16, ld_rel, max(ld_rel, base - 1), stream + "d"),
             Item(lr[:4], 16, ld_rel, max(ld_rel, base + 11), stream + "l")]
    for i in range(16):
        rel = max(rel0, slot_rel(i, base, base_prev))
        items.append(Item([sd_frag(i, m, buf)], 4, rel, max(rel, base + i - KNOBS["lead"]), stream))
    return items


def schedule_merged(a: Asm, mfmas: list, items: list, tail=None, pre=()):
    """attn_gen.schedule, with each lgkmcnt wait also covering the next
    MFMA's fragments when they are already in flight (one wait per two
    MFMAs: each wait costs an issue slot, and one wave per SIMD issues at
    most one instruction per 4 cycles)."""
    if not KNOBS["merge"]:
        return schedule(a, mfmas, items, tail, pre=pre)
    out = []

    class Cap:          # collect schedule()'s output, then rewrite its waits
        def __call__(self, txt):
            out.append(txt)
    saved = dict(AG.KNOBS)
    AG.KNOBS["lgkm"] = False
    try:
        schedule(Cap(), mfmas, items, tail, pre=())
    finally:
        AG.KNOBS.clear()
        AG.KNOBS.update(saved)
    if not KNOBS["lgkm"]:
        for t in out:
            a(t)
        return
    # replay: lds = tags of issued reads in order; before MFMA g wait for
    # the tags of g (and of g + 1 when all of them were read already)
    lds: list = list(pre)
    done = 0
    mf_idx = [i for i, t in enumerate(out) if t.startswith("v_mfma")]
    need_tags = {i: mfmas[k][1] for k, i in enumerate(mf_idx)}
    nxt = {mf_idx[k]: mf_idx[k + 1] for k in range(len(mf_idx) - 1)}

    def idx_of(t):
        return max((i for i, x in enumerate(lds) if x == t), default=-1)

    for i, t in enumerate(out):
        if i in need_tags:
            need = 0
            for tag in need_tags[i]:
                j = idx_of(tag)
                assert j >= 0, f"MFMA needs {tag} before any read of it"
                need = max(need, j + 1)
            if need > done:
                j2 = nxt.get(i)
                if j2 is not None:
                    idx2 = [idx_of(tag) for tag in need_tags[j2]]
                    if idx2 and min(idx2) >= 0:
                        need = max(need, max(idx2) + 1)
                cnt = min(15, len(lds) - need)
                a(f"s_waitcnt lgkmcnt({cnt})")
                done = len(lds) - cnt
        a(t)
        if t.startswith("ds_read"):
            lds.append(t.split(";")[1].strip() if ";" in t else None)


def sched(a: Asm, mf: list, items: list, tail=None, pre=()):
    """The list schedule with this kernel's knobs (lgkm waits, LDS reads)."""
    items = [it for it in items if it.ins]
    if not KNOBS["lds"]:
        items = [it for it in items if not it.ins[0].startswith("ds_read")]
        mf = [(t, []) for t, _ in mf]
        pre = ()
    schedule_merged(a, mf, items, tail, pre=pre)


# ---------------------------------------------------------------- loop bodies
def iteration(a: Asm, m1: bool, m2: bool, ph: int, nxt: str):
    """One step it (not the last), it % 3 == ph: MFMAs KV(2 it) [0..15],
    SD(2 it + 2) [16..31], KV(2 it + 1) [32..47], SD(2 it + 3) [48..63].
    Tile it sits in buffer ph, tile it + 1 in ph + 1, tile it + 2 goes to ph + 2."""
    kbuf, sbuf_, dbuf = ph, (ph + 1) % 3, (ph + 2) % 3
    G_BAR, DL_DMA = KNOBS["gbar"], KNOBS["dldma"]   # noqa: N806 -- the sweep arms' values
    mf = kv_mfmas(0) + sd_mfmas(0) + kv_mfmas(1) + sd_mfmas(1)
    n = len(mf)
    items: list[Item] = []
    # KV reads (tile it); KV(2 it)'s first NPRE fragments came with the previous body
    items += kv_read_items(0, 0, kbuf, None, True, "kr")
    items += kv_read_items(32, 1, kbuf, 0, False, "kr2")
    # the barrier: every wave's pieces of tile it + 1 landed (vmcnt: only the
    # dS stores of E(2 it) -- issued after every DMA piece, two 16-B or four
    # 8-B ones -- and any since may be outstanding), every wave done with tile it - 1
    vm = 2 if KNOBS["dswide"] else 4
    items.append(Item(([f"s_waitcnt vmcnt({vm})"] if KNOBS["vmwait"] else []) + (["s_barrier"] if KNOBS["bar"] else []),
                      8, G_BAR, G_BAR, "bar", split=False))
    # SD reads (tile it + 1): SD(2 it + 2) after the barrier; SD(2 it + 3)'s
    # -lse / -delta rows after E(2 it + 1) let go of the parity-1 registers
    items += sd_read_items(16, 0, 0, sbuf_, G_BAR, None, G_BAR, "sr")
    items += sd_read_items(48, 1, 1, sbuf_, -1, 16, 30, "sr2")
    # E(2 it + 1) (parity 1: step it, half 1) uses S_DSO1 / S_DD1 / SRD_DS1 of
    # step it; then both halves' of step it + 1 for E(2 it + 2) (now) and E(2 it + 3)
    items += e_items(1, m1, 1, 29, "e1")
    items.append(Item(dso_step(S_NMOD, S_NHEAD), 40, 30, 33, "e2", split=False))
    items += e_items(0, m2, 33, 61, "e2", st_rel=DL_DMA + 1)
    # DMA of tile min(it + 2, last) into buffer ph + 2, after the barrier
    items.append(Item(dma_setup(), 16, -1, G_BAR, "dma", split=False))
    for ins in dma_pieces(dbuf) if KNOBS["dma"] else []:
        items.append(Item(ins, 48, G_BAR, DL_DMA, "dma", split=False))
    # bookkeeping for the next iteration, and KV(2 it + 2)'s first fragments
    # (tile it + 1; their ring slots last used by MFMAs 44, 45)
    book = [[f"s_add_u32 {sr(S_IT)}, {sr(S_IT)}, 1",
             f"s_mov_b32 {sr(S_MOD)}, {sr(S_NMOD)}",
             f"s_mov_b32 {sr(S_HEAD)}, {sr(S_NHEAD)}"], advance(S_NMOD, S_NHEAD), dma_advance()]
    for ins in book:   # each group SCC-self-contained
        items.append(Item(ins, 2 * len(ins), DL_DMA + 1, 44, "book", split=False))
    items += kv_prefetch_items(46, n - 1, 0, sbuf_)
    sched(a, mf, items, [f"s_branch {nxt}"], pre=("KF0", "KF0", "KF1", "KF1"))


def tail(a: Asm, m1: bool, ph: int):
    """The last step: KV(N - 2) [0..15] with E(N - 1), then KV(N - 1)."""
    mf = kv_mfmas(0) + kv_mfmas(1)
    items: list[Item] = []
    items += kv_read_items(0, 0, ph, None, True, "kr")
    items += kv_read_items(16, 1, ph, 0, False, "kr2")
    items += e_items(1, m1, 1, 13, "e1")
    sched(a, mf, items, pre=("KF0", "KF0", "KF1", "KF1"))


# ---------------------------------------------------------------- prologue
def prologue(a: Asm):
    a(f"s_load_dwordx16 {sr(4, 16)}, s[0:1], 0x0")
    a(f"s_load_dwordx8 {sr(20, 8)}, s[0:1], 0x40")
    a(f"s_load_dwordx8 {sr(28, 8)}, s[0:1], 0x60")
    a(f"s_load_dwordx2 {sr(36, 2)}, s[0:1], 0x80")
    a(f"v_lshrrev_b32 {vr(V_X + 20)}, 6, v0")            # wave id
    a("s_waitcnt lgkmcnt(0)")
    t0, t1, t2, t3 = S_T0, S_T0 + 1, S_T0 + 2, S_T0 + 3
    # defensive checks (the host launcher validates the same): S = 128 nkb,
    # H = rep Hk, workgroup id < nkb B Hk
    a(f"s_cmp_eq_u32 {sr(S_NKB)}, 0")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_lshl_b32 {sr(t0)}, {sr(S_NKB)}, 7")
    a(f"s_cmp_lg_u32 {sr(t0)}, {sr(S_S)}")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_mul_i32 {sr(t0)}, {sr(S_REP)}, {sr(S_HK)}")
    a(f"s_cmp_lg_u32 {sr(t0)}, {sr(S_H)}")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_mul_i32 {sr(t1)}, {sr(S_B)}, {sr(S_HK)}")     # B Hk
    a(f"s_mul_i32 {sr(t0)}, {sr(t1)}, {sr(S_NKB)}")
    a(f"s_cmp_ge_u32 s2, {sr(t0)}")
    a(f"s_cbranch_scc1 {a.abort}")
    # kb = id / (B Hk) (heaviest first), b = (id % (B Hk)) / Hk, hk = id % Hk
    AG.udiv(a, S_KB, t2, 2, t1)
    AG.udiv(a, S_BB, S_HKV, t2, S_HK)
    a("s_nop 4")
    a(f"v_readfirstlane_b32 {sr(S_W)}, {vr(V_X + 20)}")
    a("s_nop 4")
    # steps per head pass nqt = S / 64 - 2 kb, total = nqt rep
    a(f"s_lshr_b32 {sr(S_NQT)}, {sr(S_S)}, 6")
    a(f"s_lshl_b32 {sr(t0)}, {sr(S_KB)}, 1")
    a(f"s_sub_u32 {sr(S_NQT)}, {sr(S_NQT)}, {sr(t0)}")
    a(f"s_mul_i32 {sr(S_TOT)}, {sr(S_NQT)}, {sr(S_REP)}")
    a(f"s_sub_u32 {sr(S_TOTM1)}, {sr(S_TOT)}, 1")
    a(f"s_mul_i32 {sr(S_HQ0)}, {sr(S_HKV)}, {sr(S_REP)}")
    # dS blocks per (batch, head): nb (nb + 1) / 2, nb = S / 32
    a(f"s_lshr_b32 {sr(t0)}, {sr(S_S)}, 5")
    a(f"s_add_u32 {sr(t1)}, {sr(t0)}, 1")
    a(f"s_mul_i32 {sr(t0)}, {sr(t0)}, {sr(t1)}")
    a(f"s_lshr_b32 {sr(S_NBLK)}, {sr(t0)}, 1")
    # --- per-wave DMA role: waves 0, 1 the Q tile (rows 32 (w & 1) ..), 2, 3 dO
    lq, ld = a.fresh("role_q"), a.fresh("role_done")
    a(f"s_mul_i32 {sr(t0)}, {sr(S_BB)}, {sr(S_H)}")
    a(f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(S_HQ0)}")
    a(f"s_mul_i32 {sr(t0)}, {sr(t0)}, {sr(S_S)}")                 # (b H + hq0) S
    a(f"s_mul_i32 {sr(t1)}, {sr(S_REP)}, {sr(S_S)}")
    a(f"s_lshl_b32 {sr(t1)}, {sr(t1)}, 8")                       # rep S rows
    a(f"s_mov_b32 {sr(S_HS256)}, {sr(S_S)}")          # head stride in rows (scaled below)
    a(f"s_mov_b32 {sr(S_QS64)}, 1")                   # query stride in rows
    a(f"s_mov_b32 {sr(S_DSTR)}, {ROWB}")
    a(f"s_cmp_lt_u32 {sr(S_W)}, 2")
    a(f"s_cbranch_scc1 {lq}")
    a(f"s_bitcmp1_b32 {sr(S_FL)}, 0")
    a(f"s_cbranch_scc0 {ld}_do")
    # dO as [B, S, H, D]: row (b S + q) H + h
    a(f"s_mul_i32 {sr(t0)}, {sr(S_BB)}, {sr(S_S)}")
    a(f"s_mul_i32 {sr(t0)}, {sr(t0)}, {sr(S_H)}")
    a(f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(S_HQ0)}")
    a(f"s_mul_i32 {sr(t1)}, {sr(S_S)}, {sr(S_H)}")
    a(f"s_sub_u32 {sr(t1)}, {sr(t1)}, {sr(S_HQ0)}")
    a(f"s_lshl_b32 {sr(t1)}, {sr(t1)}, 8")
    a(f"s_mov_b32 {sr(S_HS256)}, 1")
    a(f"s_mov_b32 {sr(S_QS64)}, {sr(S_H)}")
    a(f"s_lshl_b32 {sr(S_DSTR)}, {sr(S_H)}, 8")
    a.label(ld + "_do")
    srd64(a, SRD_DMA, S_DO, t0, ROWB, sr(t1))
    a(f"s_branch {ld}")
    a.label(lq)
    srd64(a, SRD_DMA, S_Q, t0, ROWB, sr(t1))
    a.label(ld)
    # tile offsets: TSOFF = mod QS64 + head HS256 + TB, with QS64 = 64 QS 256,
    # HS256 = HS 256, TB = 2 kb 64 QS 256 + 32 (w & 1) DSTR (the wave's rows)
    t0_, t1_ = S_T0, S_T0 + 1
    a(f"s_lshl_b32 {sr(S_QS64)}, {sr(S_QS64)}, 14")
    a(f"s_lshl_b32 {sr(S_HS256)}, {sr(S_HS256)}, 8")
    a(f"s_mul_i32 {sr(S_TB)}, {sr(S_KB)}, {sr(S_QS64)}")
    a(f"s_lshl_b32 {sr(S_TB)}, {sr(S_TB)}, 1")
    a(f"s_and_b32 {sr(t0_)}, {sr(S_W)}, 1")
    a(f"s_mul_i32 {sr(t0_)}, {sr(t0_)}, {sr(S_DSTR)}")
    a(f"s_lshl_b32 {sr(t0_)}, {sr(t0_)}, 5")
    a(f"s_add_u32 {sr(S_TB)}, {sr(S_TB)}, {sr(t0_)}")
    # -lse / -delta row offsets: LSOFF = mod 256 + head S4 + LB (LB = 2 kb 64 4)
    a(f"s_lshl_b32 {sr(S_S4)}, {sr(S_S)}, 2")
    a(f"s_lshl_b32 {sr(S_LB)}, {sr(S_KB)}, 9")
    # piece region / base inside a tile buffer: Q or dO region + 8 (w & 1) pieces
    a(f"s_and_b32 {sr(t0)}, {sr(S_W)}, 1")
    a(f"s_lshl_b32 {sr(S_SOFF)}, {sr(t0)}, 13")
    a(f"s_cmp_ge_u32 {sr(S_W)}, 2")
    a(f"s_cselect_b32 {sr(t0)}, {OFF_DO}, 0")
    a(f"s_add_u32 {sr(S_SOFF)}, {sr(S_SOFF)}, {sr(t0)}")
    # dS block coordinates: 4 kb, ki = 4 kb + w, 32 w
    a(f"s_lshl_b32 {sr(S_4KB)}, {sr(S_KB)}, 2")
    a(f"s_add_u32 {sr(S_KI)}, {sr(S_4KB)}, {sr(S_W)}")
    a(f"s_lshl_b32 {sr(S_32W)}, {sr(S_W)}, 5")
    # -lse (even waves) / -delta (odd) rows: (b H + hq0) S + .., rep S floats
    a(f"s_mul_i32 {sr(t0)}, {sr(S_BB)}, {sr(S_H)}")
    a(f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(S_HQ0)}")
    a(f"s_mul_i32 {sr(t0)}, {sr(t0)}, {sr(S_S)}")
    a(f"s_mul_i32 {sr(t1)}, {sr(S_REP)}, {sr(S_S)}")
    a(f"s_lshl_b32 {sr(t1)}, {sr(t1)}, 2")
    a(f"s_bitcmp1_b32 {sr(S_W)}, 0")
    a(f"s_cselect_b32 {sr(t2)}, {sr(S_ND)}, {sr(S_NL)}")
    a(f"s_cselect_b32 {sr(t3)}, {sr(S_ND + 1)}, {sr(S_NL + 1)}")
    a(f"s_mov_b32 {sr(SRD_X)}, {sr(t2)}")
    a(f"s_mov_b32 {sr(SRD_X + 1)}, {sr(t3)}")
    srd64(a, SRD_LD, SRD_X, t0, 4, sr(t1))
    # dS blocks of batch b: base dS + b H NBLK 2048, H NBLK 2048 bytes
    a(f"s_mul_i32 {sr(t0)}, {sr(S_BB)}, {sr(S_H)}")
    a(f"s_mul_i32 {sr(t0)}, {sr(t0)}, {sr(S_NBLK)}")
    a(f"s_mul_i32 {sr(S_NREC)}, {sr(S_H)}, {sr(S_NBLK)}")
    a(f"s_lshl_b32 {sr(S_NREC)}, {sr(S_NREC)}, 11")
    srd64(a, SRD_DS0, S_DS, t0, 2048, sr(S_NREC))
    for x in range(4):
        a(f"s_mov_b32 {sr(SRD_DS1 + x)}, {sr(SRD_DS0 + x)}")
    # --- lane constants
    l, g, qq, pp, hh, r, tt = (V_X + i for i in range(7))
    t = V_T
    a(f"v_and_b32 {vr(l)}, 63, v0")
    a(f"v_lshrrev_b32 {vr(g)}, 4, {vr(l)}")
    a(f"v_bfe_u32 {vr(qq)}, {vr(l)}, 2, 2")
    a(f"v_and_b32 {vr(pp)}, 3, {vr(l)}")
    a(f"v_lshrrev_b32 {vr(hh)}, 5, {vr(l)}")
    a(f"v_and_b32 {vr(r)}, 31, {vr(l)}")
    # row reads: rro[s] = r 256 + (((2 s + hh) ^ swz(r)) << 4), swz(r) = ((r & 3) << 2) | ((r >> 2) & 3)
    a(f"v_and_b32 {vr(t)}, 3, {vr(r)}")
    a(f"v_lshlrev_b32 {vr(t)}, 2, {vr(t)}")
    a(f"v_bfe_u32 {vr(t + 1)}, {vr(r)}, 2, 2")
    a(f"v_or_b32 {vr(t)}, {vr(t)}, {vr(t + 1)}")               # swz(r)
    a(f"v_lshlrev_b32 {vr(t + 2)}, 8, {vr(r)}")                # r 256
    for s_ in range(8):
        a(f"v_add_u32 {vr(t + 1)}, {2 * s_}, {vr(hh)}")
        a(f"v_xor_b32 {vr(t + 1)}, {vr(t + 1)}, {vr(t)}")
        a(f"v_lshl_add_u32 {vr(V_RRO + s_)}, {vr(t + 1)}, 4, {vr(t + 2)}")
    # -lse / -delta rows: OFF_L + 16 hh
    a(f"v_lshlrev_b32 {vr(V_LO)}, 4, {vr(hh)}")
    a(f"v_add_u32 {vr(V_LO)}, {OFF_L}, {vr(V_LO)}")
    # transposed reads: row0 = 4 hh + qq (swz 4 qq + hh), row8 = row0 + 8 (swz 4 qq + hh + 2),
    # chunk c = 4 dt + 2 (g & 1) + (pp >> 1), + 8 (pp & 1) bytes
    a(f"v_lshl_add_u32 {vr(tt)}, {vr(hh)}, 2, {vr(qq)}")       # row0
    a(f"v_lshlrev_b32 {vr(tt)}, 8, {vr(tt)}")                  # row0 256
    a(f"v_and_b32 {vr(t)}, 1, {vr(g)}")
    a(f"v_lshlrev_b32 {vr(t)}, 1, {vr(t)}")
    a(f"v_lshrrev_b32 {vr(t + 1)}, 1, {vr(pp)}")
    a(f"v_add_u32 {vr(t)}, {vr(t)}, {vr(t + 1)}")              # cb
    a(f"v_lshl_add_u32 {vr(t + 1)}, {vr(qq)}, 2, {vr(hh)}")    # swz0
    a(f"v_add_u32 {vr(t + 2)}, 2, {vr(t + 1)}")                # swz8
    a(f"v_and_b32 {vr(t + 3)}, 1, {vr(pp)}")
    a(f"v_lshlrev_b32 {vr(t + 3)}, 3, {vr(t + 3)}")            # 8 (pp & 1)
    a(f"v_add_u32 {vr(t + 3)}, {vr(t + 3)}, {vr(tt)}")
    for dt in range(4):
        a(f"v_add_u32 {vr(t + 4)}, {4 * dt}, {vr(t)}")         # c
        a(f"v_xor_b32 {vr(t + 5)}, {vr(t + 4)}, {vr(t + 1)}")
        a(f"v_lshl_add_u32 {vr(V_TRO + dt)}, {vr(t + 5)}, 4, {vr(t + 3)}")
        a(f"v_xor_b32 {vr(t + 5)}, {vr(t + 4)}, {vr(t + 2)}")
        a(f"v_lshl_add_u32 {vr(V_TRO8 + dt)}, {vr(t + 5)}, 4, {vr(t + 3)}")
        a(f"v_add_u32 {vr(V_TRO8 + dt)}, {8 * ROWB}, {vr(V_TRO8 + dt)}")
    # set B: the same offsets into buffer 2
    for x in range(8):
        a(f"v_add_u32 {vr(V_RRO_B + x)}, {2 * BUFB}, {vr(V_RRO + x)}")
    a(f"v_add_u32 {vr(V_LO_B)}, {2 * BUFB}, {vr(V_LO)}")
    for dt in range(4):
        a(f"v_add_u32 {vr(V_TRO_B + dt)}, {2 * BUFB}, {vr(V_TRO + dt)}")
        a(f"v_add_u32 {vr(V_TRO8_B[dt])}, {2 * BUFB}, {vr(V_TRO8 + dt)}")
    # DMA sources: piece u = rows 4 u + (l >> 4) of the wave's 32, chunk
    # (l & 15) ^ ((l >> 4) << 2) ^ (u & 3) of the swizzled image
    a(f"v_lshlrev_b32 {vr(t)}, 2, {vr(g)}")
    a(f"v_and_b32 {vr(t + 1)}, 15, {vr(l)}")
    a(f"v_xor_b32 {vr(t)}, {vr(t)}, {vr(t + 1)}")
    a(f"v_mul_u32_u24 {vr(t + 2)}, {sr(S_DSTR)}, {vr(g)}")
    for u in range(8):
        a(f"s_mul_i32 {sr(t0)}, {sr(S_DSTR)}, {4 * u}")
        a(f"v_xor_b32 {vr(t + 1)}, {u & 3}, {vr(t)}")
        a(f"v_lshl_add_u32 {vr(V_DMA + u)}, {vr(t + 1)}, 4, {vr(t + 2)}")
        a(f"v_add_u32 {vr(V_DMA + u)}, {sr(t0)}, {vr(V_DMA + u)}")
    a(f"v_lshlrev_b32 {vr(V_L4)}, 2, {vr(l)}")
    a(f"v_mov_b32 {vr(V_C2)}, {sr(S_C)}")
    a(f"v_mov_b32 {vr(V_C2 + 1)}, {sr(S_C)}")
    # dS store: key 16 + hh 8; mask base r - 4 hh
    a(f"v_lshlrev_b32 {vr(V_DSO)}, 4, {vr(r)}")
    # lane half hh: + 8 B (4 of the group's 8 queries) for the 8-B stores, + 512 B
    # (the next query group) for the 16-B ones (e_items)
    a(f"v_lshl_add_u32 {vr(V_DSO)}, {vr(hh)}, {9 if KNOBS['dswide'] else 3}, {vr(V_DSO)}")
    a(f"v_lshlrev_b32 {vr(t)}, 2, {vr(hh)}")
    a(f"v_sub_u32 {vr(V_MD0)}, {vr(r)}, {vr(t)}")
    # --- K / V rows of this wave's keys -> B-operand fragments (AGPRs)
    a(f"s_lshl_b32 {sr(t0)}, {sr(S_KB)}, 7")
    a(f"s_lshl_b32 {sr(t1)}, {sr(S_W)}, 5")
    a(f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(t1)}")                  # kw
    a(f"s_mul_i32 {sr(t1)}, {sr(S_BB)}, {sr(S_HK)}")
    a(f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(S_HKV)}")
    a(f"s_mul_i32 {sr(t1)}, {sr(t1)}, {sr(S_S)}")
    a(f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(t0)}")                  # (b Hk + hk) S + kw
    srd64(a, SRD_X, S_K, t1, ROWB, 32 * ROWB)
    a(f"v_lshlrev_b32 {vr(t)}, 8, {vr(r)}")
    a(f"v_lshl_add_u32 {vr(t)}, {vr(hh)}, 4, {vr(t)}")           # r 256 + 16 hh
    for s_ in range(8):
        a(f"buffer_load_dwordx4 {vr(V_SB + 4 * s_, 4)}, {vr(t)}, {sr(SRD_X, 4)}, 0 offen offset:{32 * s_}")
    srd64(a, SRD_X, S_V, t1, ROWB, 32 * ROWB)
    for s_ in range(8):
        a(f"buffer_load_dwordx4 {vr(V_SB + 32 + 4 * s_, 4)}, {vr(t)}, {sr(SRD_X, 4)}, 0 offen offset:{32 * s_}")
    # the -lse / -delta row's LDS base (SRD_X is free from here on)
    a(f"s_and_b32 {sr(t0)}, {sr(S_W)}, 1")
    a(f"s_lshl_b32 {sr(t0)}, {sr(t0)}, 8")
    a(f"s_add_u32 {sr(S_LM0)}, {sr(t0)}, {OFF_L}")
    # --- tiles 0 and 1 -> buffers 0 and 1
    a(f"s_mov_b32 {sr(S_DMOD)}, 0")
    a(f"s_mov_b32 {sr(S_DHEAD)}, 0")
    for tile in range(2):
        for x in dma_setup():
            a(x)
        for ins in dma_pieces(tile):
            for x in ins:
                a(x)
        if tile == 0:
            for x in advance(S_DMOD, S_DHEAD):
                a(x)
    # the next DMA: step 2 clamped to the last (total >= 2)
    a(f"s_mov_b32 {sr(S_DIT)}, 1")
    for x in dma_advance():
        a(x)
    for x in range(128):
        a(f"v_accvgpr_write_b32 {ar(A_DV + x)}, 0")
    a("s_waitcnt vmcnt(0)")
    for x in range(64):
        a(f"v_accvgpr_write_b32 {ar(A_K + x)}, {vr(V_SB + x)}")
    a("s_barrier")
    # counters: step 0 = (mod 0, head 0), the next (1 % nqt, ..); step 0's dS
    # offsets / masks for E(0) and E(1)
    a(f"s_mov_b32 {sr(S_IT)}, 0")
    a(f"s_mov_b32 {sr(S_MOD)}, 0")
    a(f"s_mov_b32 {sr(S_HEAD)}, 0")
    a(f"s_mov_b32 {sr(S_NMOD)}, 0")
    a(f"s_mov_b32 {sr(S_NHEAD)}, 0")
    for x in dso_step(S_MOD, S_HEAD):
        a(x)
    for x in advance(S_NMOD, S_NHEAD):
        a(x)
    a("s_nop 1")
    if KNOBS["timing"]:
        a(f"s_memtime {sr(S_TM, 2)}")
        a("s_waitcnt lgkmcnt(0)")
    # --- fill: SD(0), then SD(1) with E(0) (step 0: masked) and KV(0)'s first
    # fragments (all of tile 0, buffer 0)
    mf = sd_mfmas(0) + sd_mfmas(1)
    items = sd_read_items(0, 0, 0, 0, -1, None, -1, "sr")
    items += sd_read_items(16, 1, 1, 0, -1, 0, -1, "sr2")
    items += e_items(0, True, 17, 29, "e0")
    items += kv_prefetch_items(20, 31, 0, 0)
    sched(a, mf, items)


# ---------------------------------------------------------------- epilogue
def timing_store(a: Asm):
    """Timing arm: 8 dwords per (workgroup, wave) at dbg + 32 (4 wg + wave):
    cycles from the end of the fill to the end of the loop (lo, hi), steps,
    key block, 0..."""
    if not KNOBS["timing"]:
        return
    a(f"s_memtime {sr(SRD_X, 2)}")
    a("s_waitcnt lgkmcnt(0)")
    t = S_T0
    a(f"s_sub_u32 {sr(SRD_X)}, {sr(SRD_X)}, {sr(S_TM)}")
    a(f"s_subb_u32 {sr(SRD_X + 1)}, {sr(SRD_X + 1)}, {sr(S_TM + 1)}")
    a(f"s_lshl_b32 {sr(t)}, s2, 2")
    a(f"s_add_u32 {sr(t)}, {sr(t)}, {sr(S_W)}")
    a(f"s_lshl_b32 {sr(t)}, {sr(t)}, 5")
    a(f"s_add_u32 {sr(SRD_LD)}, {sr(S_DBG)}, {sr(t)}")
    a(f"s_addc_u32 {sr(SRD_LD + 1)}, {sr(S_DBG + 1)}, 0")
    a(f"s_mov_b32 {sr(SRD_LD + 2)}, 32")
    a(f"s_mov_b32 {sr(SRD_LD + 3)}, 0x20000")
    a(f"v_mov_b32 {vr(V_T + 1)}, 0")
    for k, x in enumerate((SRD_X, SRD_X + 1, S_TOT, S_KB)):
        a(f"v_mov_b32 {vr(V_T)}, {sr(x)}")
        a(f"buffer_store_dword {vr(V_T)}, {vr(V_T + 1)}, {sr(SRD_LD, 4)}, 0 offen offset:{4 * k}")
        a("s_nop 1")
    a("s_waitcnt vmcnt(0)")


def epilogue(a: Asm):
    timing_store(a)
    a("s_waitcnt vmcnt(0)")
    a("s_nop 7")
    a("s_nop 7")
    a("s_nop 7")
    t0, t1 = S_T0, S_T0 + 1
    r, hh = V_X, V_X + 1
    a(f"v_and_b32 {vr(r)}, 31, v0")
    a(f"v_bfe_u32 {vr(hh)}, v0, 5, 1")
    a(f"s_lshl_b32 {sr(t0)}, {sr(S_KB)}, 7")
    a(f"s_lshl_b32 {sr(t1)}, {sr(S_W)}, 5")
    a(f"s_add_u32 {sr(S_T0 + 2)}, {sr(t0)}, {sr(t1)}")            # kw
    lr, ld = a.fresh("epi_rope"), a.fresh("epi_go")
    a(f"s_bitcmp1_b32 {sr(S_FL)}, 1")
    a(f"s_cbranch_scc1 {lr}")
    # dK / dV [B, Hk, S, D]: rows (b Hk + hk) S + kw ..; dK scaled by `scale`
    a(f"s_mul_i32 {sr(t1)}, {sr(S_BB)}, {sr(S_HK)}")
    a(f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(S_HKV)}")
    a(f"s_mul_i32 {sr(t1)}, {sr(t1)}, {sr(S_S)}")
    a(f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(S_T0 + 2)}")
    srd64(a, SRD_DMA, S_DK, t1, ROWB, 32 * ROWB)
    srd64(a, SRD_LD, S_DV, t1, ROWB, 32 * ROWB)
    a(f"s_mov_b32 {sr(S_DSTR)}, {ROWB}")
    a(f"s_mov_b32 {sr(S_T0 + 3)}, {sr(S_SC)}")                    # dK scale
    a(f"s_branch {ld}")
    a.label(lr)
    # RoPE: d(qkv) rows (b S + key) H3 + [H + hk | H + Hk + hk]; dK rotated
    # back with cos / sin [key][d] (d = 32 dt + 8 g + 4 hh + e, dt < 2, pairs d + 64)
    a(f"s_mul_i32 {sr(t1)}, {sr(S_BB)}, {sr(S_S)}")
    a(f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(S_T0 + 2)}")
    a(f"s_mul_i32 {sr(t1)}, {sr(t1)}, {sr(S_H3)}")
    a(f"s_add_u32 {sr(t0)}, {sr(t1)}, {sr(S_H)}")
    a(f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(S_HKV)}")
    a(f"s_mul_i32 {sr(S_DSTR)}, {sr(S_H3)}, {ROWB}")
    a(f"s_lshl_b32 {sr(S_T0 + 3)}, {sr(S_DSTR)}, 5")             # 32 rows
    srd64(a, SRD_DMA, S_DK, t0, ROWB, sr(S_T0 + 3))
    a(f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(S_HK)}")
    srd64(a, SRD_LD, S_DK, t0, ROWB, sr(S_T0 + 3))
    # cos / sin rows of this wave's keys: [S, 64] fp32
    srd64(a, SRD_DS0, S_COS, S_T0 + 2, 256, 32 * 256)
    srd64(a, SRD_DS1, S_SIN, S_T0 + 2, 256, 32 * 256)
    cb, sb = V_SB, V_SB + 32
    a(f"v_lshlrev_b32 {vr(V_T)}, 8, {vr(r)}")
    a(f"v_lshl_add_u32 {vr(V_T)}, {vr(hh)}, 4, {vr(V_T)}")      # key 256 + 16 hh
    for dt in range(2):
        for g in range(4):
            o = 128 * dt + 32 * g
            a(f"buffer_load_dwordx4 {vr(cb + 16 * dt + 4 * g, 4)}, {vr(V_T)}, {sr(SRD_DS0, 4)}, 0 offen offset:{o}")
            a(f"buffer_load_dwordx4 {vr(sb + 16 * dt + 4 * g, 4)}, {vr(V_T)}, {sr(SRD_DS1, 4)}, 0 offen offset:{o}")
    a("s_waitcnt vmcnt(0)")
    y1, y2 = V_T, V_T + 1
    for dt in range(2):
        for j in range(16):
            a1, a2 = A_DK + 16 * dt + j, A_DK + 16 * (dt + 2) + j
            c, s_ = cb + 16 * dt + j, sb + 16 * dt + j
            a(f"v_accvgpr_read_b32 {vr(y1)}, {ar(a1)}")
            a(f"v_accvgpr_read_b32 {vr(y2)}, {ar(a2)}")
            a(f"v_mul_f32 {vr(y1)}, {sr(S_SC)}, {vr(y1)}")
            a(f"v_mul_f32 {vr(y2)}, {sr(S_SC)}, {vr(y2)}")
            a(f"v_mul_f32 {vr(V_T + 2)}, {vr(y1)}, {vr(c)}")
            a(f"v_fma_f32 {vr(V_T + 2)}, {vr(y2)}, {vr(s_)}, {vr(V_T + 2)}")
            a(f"v_mul_f32 {vr(V_T + 3)}, {vr(y2)}, {vr(c)}")
            a(f"v_fma_f32 {vr(V_T + 3)}, -{vr(y1)}, {vr(s_)}, {vr(V_T + 3)}")
            a(f"v_accvgpr_write_b32 {ar(a1)}, {vr(V_T + 2)}")
            a(f"v_accvgpr_write_b32 {ar(a2)}, {vr(V_T + 3)}")
    a(f"s_mov_b32 {sr(S_T0 + 3)}, 1.0")
    a.label(ld)
    a("s_nop 1")
    oo = V_X + 2
    a(f"v_mul_lo_u32 {vr(oo)}, {vr(r)}, {sr(S_DSTR)}")
    a(f"v_lshl_add_u32 {vr(oo)}, {vr(hh)}, 4, {vr(oo)}")
    for which, acc0, srd, scl in (("dK", A_DK, SRD_DMA, sr(S_T0 + 3)), ("dV", A_DV, SRD_LD, None)):
        for dt in range(4):
            for k in range(2):
                tmp, data = V_X + 4, V_X + 12
                base = acc0 + 16 * dt + 8 * k
                for e in range(8):
                    a(f"v_accvgpr_read_b32 {vr(tmp + e)}, {ar(base + e)}")
                if scl:
                    for e in range(8):
                        a(f"v_mul_f32 {vr(tmp + e)}, {scl}, {vr(tmp + e)}")
                for e in range(4):
                    a(f"v_cvt_pk_bf16_f32 {vr(data + e)}, {vr(tmp + 2 * e)}, {vr(tmp + 2 * e + 1)}")
                a("s_nop 1")
                a(f"v_permlane32_swap_b32 {vr(data)}, {vr(data + 2)}")
                a(f"v_permlane32_swap_b32 {vr(data + 1)}, {vr(data + 3)}")
                a(f"buffer_store_dwordx4 {vr(data, 4)}, {vr(oo)}, {sr(srd, 4)}, 0 offen offset:{64 * dt + 32 * k}")
                a("s_nop 1")


# ---------------------------------------------------------------- kernel
def kernel(variant: str = "") -> tuple[str, str]:
    name = NAME + (f"_{variant}" if variant else "")
    a = Asm(prefix=f"dkdv{variant}_")
    a.raw(f".globl {name}")
    a.raw(".p2align 8")
    a.raw(f".type {name},@function")
    a.raw(f"{name}:")
    prologue(a)
    epi = a.fresh("epi")
    top = [a.fresh(f"top{ph}") for ph in range(3)]
    # iteration dispatch per phase it % 3 (the tile buffers): the last step ->
    # the tail; else by whether E(2 it + 1) (step it) and E(2 it + 2) (step
    # it + 1) touch the diagonal (mod < 2)
    for ph in range(3):
        lab = {k: a.fresh(f"{k}{ph}") for k in ("uu", "um", "mu", "mm", "m", "t", "tm")}
        a.label(top[ph])
        a(f"s_cmp_eq_u32 {sr(S_IT)}, {sr(S_TOTM1)}")
        a(f"s_cbranch_scc1 {lab['t']}")
        a(f"s_cmp_lt_u32 {sr(S_MOD)}, 2")
        a(f"s_cbranch_scc1 {lab['m']}")
        a(f"s_cmp_lt_u32 {sr(S_NMOD)}, 2")
        a(f"s_cbranch_scc1 {lab['um']}")
        a(f"s_branch {lab['uu']}")
        a.label(lab["m"])
        a(f"s_cmp_lt_u32 {sr(S_NMOD)}, 2")
        a(f"s_cbranch_scc1 {lab['mm']}")
        a(f"s_branch {lab['mu']}")
        for key, m1, m2 in (("uu", False, False), ("um", False, True), ("mu", True, False), ("mm", True, True)):
            a.label(lab[key])
            iteration(a, m1, m2, ph, top[(ph + 1) % 3])
        a.label(lab["t"])
        a(f"s_cmp_lt_u32 {sr(S_MOD)}, 2")
        a(f"s_cbranch_scc1 {lab['tm']}")
        tail(a, False, ph)
        a(f"s_branch {epi}")
        a.label(lab["tm"])
        tail(a, True, ph)
        a(f"s_branch {epi}")
    lab = {"epi": epi}
    a.label(lab["epi"])
    epilogue(a)
    a.label(a.abort)
    a("s_waitcnt vmcnt(0)")
    a("s_endpgm")
    a.raw(f".size {name}, .-{name}")
    desc, meta = G._descriptor(name, lds_bytes=LDS_BYTES, n_sgpr=N_SGPR, karg_bytes=KARG_BYTES)
    return "\n".join(a.out) + "\n" + desc, meta


def variant_kernel(vname: str, knobs: dict) -> tuple[str, str]:
    saved = dict(KNOBS)
    KNOBS.update(knobs)
    try:
        return kernel(vname)
    finally:
        KNOBS.clear()
        KNOBS.update(saved)


def all_kernels() -> list[tuple[str, str]]:
    """The product kernel, then the diagnostic arms (host table order)."""
    return [kernel()] + [variant_kernel(v, k) for v, k in VARIANTS]


def generate(kernels=None) -> str:
    """This kernel alone in a code object (tests; the build embeds it through
    gemm_gen.generate())."""
    kernels = kernels or [kernel()]
    return "\n".join(['.amdgcn_target "amdgcn-amd-amdhsa--gfx950"', ".amdhsa_code_object_version 5", ".text",
                      *(b for b, _ in kernels),
                      ".amdgpu_metadata\n---\namdhsa.version:\n  - 1\n  - 2\namdhsa.target: amdgcn-amd-amdhsa--gfx950\n"
                      "amdhsa.kernels:\n" + "".join(m for _, m in kernels) + "...\n.end_amdgpu_metadata"]) + "\n"


if __name__ == "__main__":
    with open(sys.argv[1] if len(sys.argv) > 1 else "attn_dkdv_asm.s", "w") as f:
        f.write(generate())
