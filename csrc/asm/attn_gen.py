#!/usr/bin/env python3
"""Generator of the hand-written gfx950 causal flash-attention forward.

Emitted into the same code object as the GEMMs (gemm_gen.generate() calls
kernel() here); host side: toa_attn_fwd_asm in csrc/hip/gemm_asm.hip, which
toa_attn_fwd (csrc/hip/attention.hip) calls for the shapes it takes.

    O[b, q, h] = softmax_k<=q(Q[b, h, q] . K[b, h / rep, k] * scale) V[b, h / rep, k]
    LSE[b, h, q] = ln sum_k<=q exp(Q . K * scale)

bf16 Q / K / V [B, H(k), S, 128], O [B, S, H, 128] (flags bit 1) or
[B, H, S, 128], LSE fp32; S % 256 == 0.

Why assembly (docs/kernels.md, round 5): the HIP kernel (attn_fwd_gl_kernel,
8 waves x 32 query rows, two waves per SIMD) spends 53 % of its cycles with
the matrix cores idle -- the compiler neither spreads the softmax VALU evenly
between the MFMAs nor keeps the LDS reads ahead of them.  The vector issue
port, not the matrix core, is the binding resource: per 64-key tile a wave's
MFMAs occupy 2048 cycles of the matrix pipe but their softmax (64 scores per
lane: fma, exp, cvt, max) costs ~1500 cycles of issue, and every MFMA holds
the issue port for 8 of its 32 cycles.  This kernel places every instruction
(an earliest-deadline list schedule over the MFMA gaps, schedule() below):

  workgroup  256 threads = 4 waves (one per SIMD), 256 query rows of one
             (batch, head): wave w rows 64 w .. + 63, as two 32-row blocks
  scores     S^T = K Q^T with v_mfma_f32_32x32x16_bf16: A = K rows from LDS
             (ds_read_b128), B = Q^T fragments held in AGPRs for the whole
             block; the lane owns a query column, so the row max / exp / bf16
             pack are lane-local (one permlane32 swap per row max)
  P V        O^T += V^T P^T: A = V^T via ds_read_b64_tr_b16 from the same LDS
             image, B = P straight from the exp's v_cvt_pk_bf16_f32; the row
             sums l come from the matrix core too (an all-ones A operand:
             8 MFMAs per tile instead of 64 VALU adds -- the issue port is
             the bottleneck, the matrix pipe has room)
  softmax    log2 domain (scale * log2 e folded into the exp's fma), deferred
             rescale (T13, threshold 8): O and l are rescaled out of line only
             when a row max grows by more than 2^8, at the end of a tile, after
             all of its P V MFMAs (the textbook-safe order)
  staging    K and V tiles of 64 keys by LDS-DMA (buffer_load_dwordx4 ... lds,
             4 + 4 pieces of 1 KiB per wave per tile) in the XOR-swizzled image
             attention.hip uses (k_off / v_off); K double-buffered two tiles
             ahead, V triple-buffered one tile ahead, ONE barrier per tile
  pipeline   tile i's loop body: 32 QK MFMAs of tile i + 1, then 40 MFMAs of
             P_i V_i + l_i; fillers: exp of S_i (deadlines = the P V k-step that
             reads them), mask + row max of S_{i+1}, K / V fragment reads
             (rings of 6), DMA of K_{i+2} / V_{i+1}, the barrier mid-P V
  causal     only the last 4 tiles of a block touch the diagonal: a masked
             loop body for them, an unmasked one for the rest
  grid       one workgroup per (query block, head, batch), XCD-aware (whole
             (batch, kv head) groups per XCD, heaviest query blocks first), as
             attention.hip fwd_block_coords

Reference anchor: SURVEY.md K5 (attention kernels of the flagship model;
the reference itself has no attention kernel).  Checked instruction by
instruction on the CPU by csrc/asm/emu.py (tests/test_asm_attn.py) and
against the HIP kernel / fp32 on the GPU (tests/test_ops_gpu.py).
"""
from __future__ import annotations

import sys

import gemm_gen as G
from gemm_gen import Asm, ar, sr, vr

NAME = "toa_attn_fwd_asm"
D = 128
ROWB = 2 * D             # bytes per K / V / Q row
TK = 64                  # keys per tile
QB = 256                 # query rows per workgroup
TILE = TK * ROWB         # 16 KiB: one K or V tile in LDS
VBUF0 = 2 * TILE         # K tiles at 0 / TILE, V tiles at VBUF0 + n TILE (n = 0..2)
LDS_BYTES = 5 * TILE
THR = 8.0                # deferred-rescale threshold (log2 units)
KARG_BYTES = 88
KARG = {"Q": 0, "K": 8, "V": 16, "O": 24, "LSE": 32, "B": 40, "H": 44, "Hk": 48, "S": 52, "c": 56,
        "flags": 60, "nqb": 64, "rep": 68, "g8": 72, "dbg": 80}

# ---------------------------------------------------------------- SGPRs
S_Q, S_K, S_V, S_O, S_L = 4, 6, 8, 10, 12
S_B, S_H, S_HK, S_S, S_C, S_FLAGS = 14, 15, 16, 17, 18, 19
S_NQB, S_REP, S_G8 = 20, 21, 22
S_W, S_QB, S_HH, S_BB, S_HKV, S_T, S_NU, S_TM1 = 24, 25, 26, 27, 28, 29, 30, 31
S_I, S_KT, S_VT, S_M0V, S_VDEL, S_VR, S_W1K, S_QSO = 32, 33, 34, 35, 36, 37, 38, 39
SRD_Q, SRD_K, SRD_V, SRD_O, SRD_L = 40, 44, 48, 52, 56
S_T0 = 60                 # s60..s67 scratch
S_DQ, S_DR = 68, 69
S_FA, S_FB, S_F = 70, 72, 74   # rescale flags (pairs)
S_OSTR, S_OQB, S_SOFF, S_Q0 = 76, 77, 78, 79
S_TM = 80                 # timing arm: s80..s87 four s_memtime stamps, s88 rescale count, s[90:91] dbg pointer
N_SGPR = 96

# ---------------------------------------------------------------- VGPRs
V_KOFF = 1                # v1..v8: K fragment read offsets per 16-d k-step (+ buffer)
V_VOFF = 9                # v9..v12: V^T read offsets per 32-d output tile (+ buffer)
V_DK, V_DV = 13, 14       # DMA lane offsets
V_M = 15                  # v15, v16: running max (log2 units) per 32-row block
V_E0, V_E, V_NEGINF = 17, 18, 19
V_MC = 20                 # v20, v21: this tile's max candidate per block
V_DP, V_DM = 22, 23       # mask: e + 32, e - 32
V_ONES = 24               # v24..v27: bf16 1.0 (the row-sum MFMA's A operand)
V_T = 28                  # v28..v31 scratch
V_KR = 32                 # K fragment ring: 6 x 4
V_VR = 56                 # V^T fragment ring: 6 x 4
V_P = 80                  # P (bf16 pairs): [block][k-step] x 4
V_SB = (112, 176)         # score buffers (64 each): [block][key half] x 16
V_X = 240                 # v240..v255 scratch (row max, rescale, epilogue)
RING = 6

# Schedule knobs; the DIAGNOSTIC arms (VARIANTS) switch one mechanism off to
# price it in-process (scripts/attn_fwd_ab.py --variants): their outputs are
# wrong by construction and only their time is read.
KNOBS = {"bar": True, "vmwait": True, "lgkm": True, "exp": True, "dma": True, "timing": False, "fine": True}
VARIANTS = (
    ("d1", {"bar": False, "vmwait": False}),   # no per-tile barrier nor DMA wait
    ("d2", {"vmwait": False}),                 # barrier, but not for the DMA to land
    ("d3", {"lgkm": False}),                   # MFMAs do not wait for their LDS fragments
    ("d4", {"exp": False}),                    # v_exp_f32 -> v_mov_b32 (transcendental issue cost)
    ("d5", {"dma": False, "vmwait": False}),   # no K / V staging in the loop
    ("t1", {"timing": True}),                  # the product kernel + s_memtime stamps (bit-identical outputs)
    ("c1", {"fine": False}),                   # fillers placed as whole groups (the first schedule)
    ("t2", {"timing": True, "fine": False}),   # its timing arm
)

# AGPRs: O^T a[0:127] ([block][d tile] x 16), Q^T fragments a[128:191]
# ([block][k-step] x 4), row sums a[192:223] ([block] x 16)
A_O, A_Q, A_L = 0, 128, 192


def kreg(f):
    return V_KR + 4 * (f % RING)


def vreg(u):
    return V_VR + 4 * (u % RING)


def sreg(buf, qb2, kh, r):
    return V_SB[buf] + 32 * qb2 + 16 * kh + r


def preg(qb2, ks):
    return V_P + 16 * qb2 + 4 * ks


# ---------------------------------------------------------------- helpers
def udiv(a: Asm, q: int, r: int, num: int, den: int):
    """s_q = s_num / s_den, s_r = s_num % s_den (unsigned, < 2^24), as
    gemm_gen.udiv with this kernel's scratch VGPRs."""
    t = V_T
    a(f"v_cvt_f32_u32 {vr(t)}, {sr(den)}")
    a(f"v_cvt_f32_u32 {vr(t + 1)}, {sr(num)}")
    a("s_nop 4")
    a(f"v_rcp_iflag_f32 {vr(t)}, {vr(t)}")
    a("s_nop 4")
    a(f"v_mul_f32 {vr(t)}, {vr(t)}, {vr(t + 1)}")
    a("s_nop 4")
    a(f"v_cvt_u32_f32 {vr(t)}, {vr(t)}")
    a("s_nop 4")
    a(f"v_readfirstlane_b32 {sr(q)}, {vr(t)}")
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


def srd64(a: Asm, dst: int, base: int, row: int, row_bytes: int, nrec):
    """dst = buffer resource at s[base] + s[row] * row_bytes, num_records nrec
    (an SGPR index or a literal)."""
    a(f"s_mul_hi_u32 {sr(S_T0 + 7)}, {sr(row)}, {row_bytes}")
    a(f"s_mul_i32 {sr(S_T0 + 6)}, {sr(row)}, {row_bytes}")
    a(f"s_add_u32 {sr(dst)}, {sr(base)}, {sr(S_T0 + 6)}")
    a(f"s_addc_u32 {sr(dst + 1)}, {sr(base + 1)}, {sr(S_T0 + 7)}")
    a(f"s_mov_b32 {sr(dst + 2)}, {nrec if isinstance(nrec, str) else nrec}")
    a(f"s_mov_b32 {sr(dst + 3)}, 0x20000")


# ---------------------------------------------------------------- scheduler
class Item:
    """A group of filler instructions.  Gap g = after MFMA g (-1: before the
    first).  rel / dl: earliest / latest gap of every instruction of the
    group.  Items of one stream keep their order; schedule() places their
    instructions one by one (split=False: as one unit)."""

    __slots__ = ("ins", "cost", "rel", "dl", "stream", "split")

    def __init__(self, ins, cost, rel, dl, stream, split=True):
        self.ins, self.cost, self.rel, self.dl, self.stream, self.split = ins, cost, rel, dl, stream, split


def issue_cost(ins: str) -> int:
    """Vector-issue cycles of one filler beside MFMAs, one wave per SIMD
    (MI355X_MICROARCH.md constants: transcendental 8, other VALU 4, an
    MFMA holds the port 8 of its 32; an LDS-DMA piece ~40-60)."""
    op = ins.split()[0]
    if op.startswith("buffer_load") and ins.rstrip().endswith("lds"):
        return 40
    if op in ("v_exp_f32", "v_log_f32", "v_rcp_f32"):
        return 8
    if op.startswith(("v_", "ds_", "buffer_")):
        return 4
    if op == "s_nop":
        return 4 * (int(ins.split()[1]) + 1)
    return 1


GAP_BUDGET = 24     # filler issue cycles one 32x32x16 MFMA gap hides


def schedule(a: Asm, mfmas: list, items: list, tail: list | None = None, pre=()):
    """Emit MFMAs (text, needed LDS tags) with the items spread over the gaps:
    earliest deadline first, against an even cumulative issue-cost line.
    LDS reads are tagged by a trailing "; tag" comment in their text; before
    an MFMA the lgkmcnt wait its tags need is inserted (LDS completes in
    order, so older outstanding reads do not change the count).  `pre`: tags
    read before this schedule (the previous loop body's prefetch), taken as
    the most recent LDS ops at its start."""
    n = len(mfmas)
    streams: dict = {}
    for it in items:
        assert -1 <= it.rel <= n - 1 and it.dl >= it.rel, (it.ins[:1], it.rel, it.dl)
        if it.split and KNOBS["fine"]:
            for ins in it.ins:
                streams.setdefault(it.stream, []).append(Item([ins], issue_cost(ins), it.rel, it.dl, it.stream))
        else:
            streams.setdefault(it.stream, []).append(it)
    total = sum(it.cost for lst in streams.values() for it in lst)
    place = {g: [] for g in range(-1, n)}
    heads = {s: 0 for s in streams}
    cum = 0.0
    for g in range(-1, n):
        target = total * (g + 2) / (n + 1)
        while True:
            cands = [(streams[s][heads[s]].dl, str(s), s) for s in streams
                     if heads[s] < len(streams[s]) and streams[s][heads[s]].rel <= g]
            if not cands:
                break
            dl, _, s = min(cands)
            if cum >= target and dl > g:
                break
            it = streams[s][heads[s]]
            heads[s] += 1
            place[g].append(it)
            cum += it.cost
    for s, lst in streams.items():
        assert heads[s] == len(lst), f"stream {s}: {len(lst) - heads[s]} items unplaced"
    for g, lst in place.items():
        for it in lst:
            if g > it.dl:
                raise AssertionError(f"item {it.ins[:1]} (stream {it.stream}) placed at gap {g} > deadline {it.dl}")
    lds: list = list(pre)   # tags of issued LDS ops, in order
    done = [0]              # LDS ops known complete

    def emit(txt):
        a(txt)
        if txt.startswith("ds_read"):
            lds.append(txt.split(";")[1].strip() if ";" in txt else None)

    def wait_for(tags):
        if not KNOBS["lgkm"]:
            return
        need = 0
        for t in tags:
            idx = max((i for i, x in enumerate(lds) if x == t), default=-1)
            assert idx >= 0, f"MFMA needs {t} before any read of it"
            need = max(need, idx + 1)
        if need > done[0]:
            cnt = min(15, len(lds) - need)
            a(f"s_waitcnt lgkmcnt({cnt})")
            done[0] = len(lds) - cnt

    for it in place[-1]:
        for t in it.ins:
            emit(t)
    for g in range(n):
        txt, tags = mfmas[g]
        wait_for(tags)
        a(txt)
        for it in place[g]:
            for t in it.ins:
                emit(t)
    for t in tail or []:
        emit(t)


# ---------------------------------------------------------------- pieces
def kread(f: int) -> str:
    kh, ds = divmod(f, 8)
    return f"ds_read_b128 {vr(kreg(f), 4)}, {vr(V_KOFF + ds)} offset:{kh * 8192} ; K{f}"


def vread(u: int) -> list[str]:
    ks, dt = divmod(u, 4)
    kb0 = 4096 * ks
    return [f"ds_read_b64_tr_b16 {vr(vreg(u), 2)}, {vr(V_VOFF + dt)} offset:{kb0} ; V{u}",
            f"ds_read_b64_tr_b16 {vr(vreg(u) + 2, 2)}, {vr(V_VOFF + dt)} offset:{kb0 + 2048} ; V{u}"]


def qk_mfmas(dst_buf: int, first_zero: bool = True) -> list:
    out = []
    for f in range(16):
        kh, ds = divmod(f, 8)
        for qb2 in range(2):
            d = sreg(dst_buf, qb2, kh, 0)
            c = "0" if (ds == 0 and first_zero) else vr(d, 16)
            out.append((f"v_mfma_f32_32x32x16_bf16 {vr(d, 16)}, {vr(kreg(f), 4)}, {ar(A_Q + 32 * qb2 + 4 * ds, 4)}, {c}",
                        [f"K{f}"]))
    return out


def pv_mfmas() -> list:
    """P V in k-step order: per k-step 4 d tiles x 2 blocks, then the two
    row-sum MFMAs (A = ones).  Group of k-step ks starts at 10 ks."""
    out = []
    for ks in range(4):
        for dt in range(4):
            u = 4 * ks + dt
            for qb2 in range(2):
                acc = ar(A_O + 64 * qb2 + 16 * dt, 16)
                out.append((f"v_mfma_f32_32x32x16_bf16 {acc}, {vr(vreg(u), 4)}, {vr(preg(qb2, ks), 4)}, {acc}",
                            [f"V{u}"]))
        for qb2 in range(2):
            acc = ar(A_L + 16 * qb2, 16)
            out.append((f"v_mfma_f32_32x32x16_bf16 {acc}, {vr(V_ONES, 4)}, {vr(preg(qb2, ks), 4)}, {acc}", []))
    return out


def pv_index(u: int) -> int:
    ks, dt = divmod(u, 4)
    return 10 * ks + 2 * dt


def exp_items(buf: int, base: int, stream="exp") -> list[Item]:
    """P = bf16(exp2(S * c - m)) for score buffer `buf`; deadlines: two gaps
    ahead of the P V k-step reading them (PV MFMAs start at index `base`)."""
    items = []
    for ks in range(4):
        kh, half = divmod(ks, 2)
        dl = max(-1, base + 10 * ks - 2)
        for qb2 in range(2):
            for part in range(2):
                r0 = 8 * half + 4 * part
                regs = [sreg(buf, qb2, kh, r0 + e) for e in range(4)]
                p = preg(qb2, ks) + 2 * part
                ins = [f"v_fma_f32 {vr(x)}, {vr(x)}, {sr(S_C)}, -{vr(V_M + qb2)}" for x in regs]
                ins += [f"v_exp_f32 {vr(x)}, {vr(x)}" if KNOBS["exp"] else f"v_mov_b32 {vr(x)}, {vr(x)}" for x in regs]
                ins += [f"v_cvt_pk_bf16_f32 {vr(p)}, {vr(regs[0])}, {vr(regs[1])}",
                        f"v_cvt_pk_bf16_f32 {vr(p + 1)}, {vr(regs[2])}, {vr(regs[3])}"]
                items.append(Item(ins, 58, -1, dl, stream))
    return items


MASK_C = [(r & 3) + 8 * (r >> 2) for r in range(16)]


def mask_ins(buf: int, qb2: int, kh: int, rs) -> list[str]:
    """key > query -> -inf for registers rs of (block, key half).  Lane
    value d = q - (first key of the half) - 4 hh; register r's key offset is
    MASK_C[r]: masked iff MASK_C[r] > d."""
    dreg = V_E if qb2 == kh else (V_DP if qb2 > kh else V_DM)
    out = []
    for r in rs:
        x = sreg(buf, qb2, kh, r)
        out += [f"v_cmp_gt_i32 vcc, {MASK_C[r]}, {vr(dreg)}", f"v_cndmask_b32 {vr(x)}, {vr(x)}, {vr(V_NEGINF)}, vcc"]
    return out


def max_ops(buf: int, qb2: int) -> tuple[list[str], list[str]]:
    """Row-max chain over the 32 scores of a block: ops touching key half 0
    only, and the rest (from key half 1's MFMAs on)."""
    vals = [sreg(buf, qb2, 0, r) for r in range(16)] + [sreg(buf, qb2, 1, r) for r in range(16)]
    t = V_X + qb2
    ops = [(f"v_max3_f32 {vr(t)}, {vr(vals[0])}, {vr(vals[1])}, {vr(vals[2])}", 2)]
    i = 3
    while i + 1 < 32:
        ops.append((f"v_max3_f32 {vr(t)}, {vr(t)}, {vr(vals[i])}, {vr(vals[i + 1])}", i + 1))
        i += 2
    ops.append((f"v_max_f32 {vr(t)}, {vr(t)}, {vr(vals[31])}", 31))
    a_ops = [o for o, last in ops if last < 16]
    b_ops = [o for o, last in ops if last >= 16]
    return a_ops, b_ops


def max_final(qb2: int) -> list[str]:
    """Both halves' maxima -> V_MC (log2 units); flag rows whose max grew by
    more than THR into s[S_FA / S_FB]."""
    t, u = V_X + qb2, V_X + 2 + qb2
    return [f"v_mov_b32 {vr(u)}, {vr(t)}",
            "s_nop 1",
            f"v_permlane32_swap_b32 {vr(t)}, {vr(u)}",
            f"v_max_f32 {vr(t)}, {vr(t)}, {vr(u)}",
            f"v_mul_f32 {vr(V_MC + qb2)}, {sr(S_C)}, {vr(t)}",
            f"v_add_f32 {vr(u)}, {THR}, {vr(V_M + qb2)}",
            f"v_cmp_gt_f32 {sr(S_FA if qb2 == 0 else S_FB, 2)}, {vr(V_MC + qb2)}, {vr(u)}"]


def dma_piece(kind: str, j: int, p: int) -> list[str]:
    """Piece j of this wave's share of the K (into K buffer p) or V tile."""
    if kind == "K":
        so, m0 = S_KT, f"s_add_u32 m0, {sr(S_W1K)}, {p * TILE + j * 4096}"
        vo, srd_ = V_DK, SRD_K
    else:
        so, m0 = S_VT, f"s_add_u32 m0, {sr(S_M0V)}, {j * 4096}"
        vo, srd_ = V_DV, SRD_V
    out = []
    if j:
        out.append(f"s_add_u32 {sr(S_SOFF)}, {sr(so)}, {j * 4096}")
    out += [m0, "s_nop 0", f"buffer_load_dwordx4 {vr(vo)}, {sr(srd_, 4)}, {sr(S_SOFF if j else so)} offen lds"]
    return out


def mask_setup(tile_sgpr_expr: list[str]) -> list[str]:
    """V_E = V_E0 - 64 t (t from the SALU lines), V_DP / V_DM = V_E +- 32."""
    return tile_sgpr_expr + [f"v_subrev_u32 {vr(V_E)}, {sr(S_T0 + 2)}, {vr(V_E0)}",
                             f"v_add_u32 {vr(V_DP)}, 32, {vr(V_E)}",
                             f"v_subrev_u32 {vr(V_DM)}, 32, {vr(V_E)}"]


def koff_toggle() -> list[str]:
    return [f"v_xor_b32 {vr(V_KOFF + ds)}, {TILE}, {vr(V_KOFF + ds)}" for ds in range(8)]


# ---------------------------------------------------------------- loop bodies
G_BAR = 47          # the barrier: after QK MFMA 32 + 15 (mid P V)
DL_DMA = 30         # DMA pieces issued by this gap (>= ~10 gaps of flight before the barrier)


def body(a: Asm, kind: str, p: int, resc_label: str, back_label: str):
    """Loop body for tile i (S_i in score buffer p): kind "U" (tile i + 1
    unmasked), "M" (tile i + 1 touches the diagonal) or "T" (the last tile:
    no QK, no DMA)."""
    items: list[Item] = []
    if kind == "T":
        mf = pv_mfmas()
        items += exp_items(p, 0)
        for u in range(16):
            rel = -1 if u < RING else pv_index(u - RING) + 1
            items.append(Item(vread(u), 12, rel, max(rel, pv_index(u) - 4), "vr"))
        schedule(a, mf, items)
        return
    mf = qk_mfmas(p ^ 1) + pv_mfmas()
    n = len(mf)
    # --- DMA: K_{min(i+2, T-1)} -> K buffer p, V_{i+1} -> V buffer (i+1) % 3
    setup = [f"s_add_u32 {sr(S_T0)}, {sr(S_I)}, 2",
             f"s_min_u32 {sr(S_T0)}, {sr(S_T0)}, {sr(S_TM1)}",
             f"s_lshl_b32 {sr(S_KT)}, {sr(S_T0)}, 14",
             f"s_add_u32 {sr(S_T0)}, {sr(S_I)}, 1",
             f"s_lshl_b32 {sr(S_VT)}, {sr(S_T0)}, 14"]
    items.append(Item(setup, 10, -1, DL_DMA, "dma"))
    for j in range(4 if KNOBS["dma"] else 0):
        items.append(Item(dma_piece("K", j, p), 40, -1, DL_DMA, "dma"))
        items.append(Item(dma_piece("V", j, p), 40, -1, DL_DMA, "dma"))
    items.append(Item([f"s_add_u32 {sr(S_M0V)}, {sr(S_M0V)}, {TILE}",
                       f"s_cmp_ge_u32 {sr(S_M0V)}, {VBUF0 + 3 * TILE}",
                       f"s_cselect_b32 {sr(S_T0 + 1)}, {3 * TILE}, 0",
                       f"s_sub_u32 {sr(S_M0V)}, {sr(S_M0V)}, {sr(S_T0 + 1)}"], 8, -1, n - 1, "dma"))
    # --- the barrier: everyone's K_{i+2} / V_{i+1} landed; then the next
    # tile's K offsets and its first fragments
    items.append(Item((["s_waitcnt vmcnt(0)"] if KNOBS["vmwait"] else []) + (["s_barrier"] if KNOBS["bar"] else []),
                      8, G_BAR, G_BAR, "bar", split=False))
    items.append(Item(koff_toggle(), 32, G_BAR, n - 1, "bar"))
    for f in range(3):
        items.append(Item([kread(f)], 6, G_BAR, n - 1, "bar"))
    # --- K fragment reads of QK(i+1): frags 0..2 prefetched by the previous body
    for f in range(3, 16):
        rel = -1 if f < RING else 2 * (f - RING) + 1
        items.append(Item([kread(f)], 6, rel, max(rel, 2 * f - 4), "kr"))
    # --- V^T reads of P_i V_i
    for u in range(16):
        idx = 32 + pv_index(u)
        rel = -1 if u < RING else 32 + pv_index(u - RING) + 1
        items.append(Item(vread(u), 12, rel, max(rel, idx - 4), "vr"))
    # V read offsets -> the next tile's buffer (after the last V^T read)
    items.append(Item([f"s_add_u32 {sr(S_T0 + 3)}, {sr(S_VR)}, 1",
                       f"s_mov_b32 {sr(S_VDEL)}, {TILE}",
                       f"s_cmp_eq_u32 {sr(S_VR)}, 2",
                       f"s_cselect_b32 {sr(S_VDEL)}, {-2 * TILE & 0xFFFFFFFF:#x}, {sr(S_VDEL)}",
                       f"s_cselect_b32 {sr(S_VR)}, 0, {sr(S_T0 + 3)}"]
                      + [f"v_add_u32 {vr(V_VOFF + dt)}, {sr(S_VDEL)}, {vr(V_VOFF + dt)}" for dt in range(4)],
                      24, -1, n - 1, "vr"))
    # --- softmax of S_i
    items += exp_items(p, 32)
    # --- mask + row max of S_{i+1} (buffer p ^ 1)
    q = p ^ 1
    for qb2 in range(2):
        st = f"max{qb2}"
        rel0 = 2 * 7 + qb2 + 3      # last MFMA of (block, key half 0) + 3
        rel1 = 2 * 15 + qb2 + 3
        if kind == "M":
            if qb2 == 0:
                items.append(Item(mask_setup([f"s_add_u32 {sr(S_T0 + 2)}, {sr(S_I)}, 1",
                                              f"s_lshl_b32 {sr(S_T0 + 2)}, {sr(S_T0 + 2)}, 6"]), 16, -1, rel0, st))
            items.append(Item(mask_ins(q, qb2, 0, range(8)), 64, rel0, n - 1, st))
            items.append(Item(mask_ins(q, qb2, 0, range(8, 16)), 64, rel0, n - 1, st))
        a_ops, b_ops = max_ops(q, qb2)
        items.append(Item(a_ops, 4 * len(a_ops), rel0, n - 1, st))
        if kind == "M":
            items.append(Item(mask_ins(q, qb2, 1, range(8)), 64, rel1, n - 1, st))
            items.append(Item(mask_ins(q, qb2, 1, range(8, 16)), 64, rel1, n - 1, st))
        items.append(Item(b_ops, 4 * len(b_ops), rel1, n - 1, st))
        items.append(Item(max_final(qb2), 30, rel1, n - 1, st))
    items = [it for it in items if it.ins]
    tail = [f"s_add_u32 {sr(S_I)}, {sr(S_I)}, 1",
            f"s_or_b64 {sr(S_F, 2)}, {sr(S_FA, 2)}, {sr(S_FB, 2)}",      # SCC: some row's max grew past THR
            f"s_cbranch_scc1 {resc_label}"]
    schedule(a, mf, items, tail, pre=("K0", "K1", "K2"))
    a.label(back_label)


def rescale_block(a: Asm, label: str, back: str):
    """Out of line: m_new = max(m, mc), alpha = 2^(m - m_new); O, l *= alpha.
    Runs after every P V MFMA of the tile was issued: drain them first."""
    a.label(label)
    if KNOBS["timing"]:
        a(f"s_add_u32 {sr(S_TM + 8)}, {sr(S_TM + 8)}, 1")
    a("s_nop 7")
    a("s_nop 7")
    a("s_nop 7")
    al = V_T                 # v28, v29: alpha per block
    for qb2 in range(2):
        a(f"v_max_f32 {vr(V_T + 2)}, {vr(V_M + qb2)}, {vr(V_MC + qb2)}")
        a(f"v_sub_f32 {vr(al + qb2)}, {vr(V_M + qb2)}, {vr(V_T + 2)}")
        a(f"v_mov_b32 {vr(V_M + qb2)}, {vr(V_T + 2)}")
        a(f"v_exp_f32 {vr(al + qb2)}, {vr(al + qb2)}")
    a("s_nop 1")
    for qb2 in range(2):
        regs = [A_O + 64 * qb2 + r for r in range(64)] + [A_L + 16 * qb2 + r for r in range(16)]
        for k in range(0, len(regs), 8):
            grp = regs[k:k + 8]
            for e, x in enumerate(grp):
                a(f"v_accvgpr_read_b32 {vr(V_X + 4 + e)}, {ar(x)}")
            for e in range(len(grp)):
                a(f"v_mul_f32 {vr(V_X + 4 + e)}, {vr(al + qb2)}, {vr(V_X + 4 + e)}")
            for e, x in enumerate(grp):
                a(f"v_accvgpr_write_b32 {ar(x)}, {vr(V_X + 4 + e)}")
    a(f"s_branch {back}")


# ---------------------------------------------------------------- prologue
def stamp(a: Asm, k: int):
    """Timing arm: shader-clock stamp k (0 start, 1 loop, 2 epilogue, 3 end).
    s_memtime returns through lgkmcnt: the wait also drains LDS reads."""
    if KNOBS["timing"]:
        a(f"s_memtime {sr(S_TM + 2 * k, 2)}")
        a("s_waitcnt lgkmcnt(0)")


def prologue(a: Asm):
    stamp(a, 0)
    if KNOBS["timing"]:
        a(f"s_mov_b32 {sr(S_TM + 8)}, 0")
        a(f"s_load_dwordx2 {sr(S_TM + 10, 2)}, s[0:1], 0x50")
    a(f"s_load_dwordx16 {sr(4, 16)}, s[0:1], 0x0")
    a(f"s_load_dwordx4 {sr(20, 4)}, s[0:1], 0x40")
    a(f"v_lshrrev_b32 {vr(V_X + 15)}, 6, v0")          # wave id (v255: untouched until the epilogue)
    a("s_waitcnt lgkmcnt(0)")
    # defensive checks (the host launcher validates the same): S = 256 nqb,
    # H = rep Hk, g8 only when B Hk % 8 == 0, workgroup id in range
    t0, t1 = S_T0, S_T0 + 1
    a(f"s_cmp_eq_u32 {sr(S_NQB)}, 0")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_lshl_b32 {sr(t0)}, {sr(S_NQB)}, 8")
    a(f"s_cmp_lg_u32 {sr(t0)}, {sr(S_S)}")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_mul_i32 {sr(t0)}, {sr(S_REP)}, {sr(S_HK)}")
    a(f"s_cmp_lg_u32 {sr(t0)}, {sr(S_H)}")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_mul_i32 {sr(t0)}, {sr(S_NQB)}, {sr(S_H)}")
    a(f"s_mul_i32 {sr(t0)}, {sr(t0)}, {sr(S_B)}")
    a(f"s_cmp_ge_u32 s2, {sr(t0)}")
    a(f"s_cbranch_scc1 {a.abort}")
    a(f"s_mul_i32 {sr(t1)}, {sr(S_B)}, {sr(S_HK)}")     # G = B Hk
    lgen, lcoord = a.fresh("coords_generic"), a.fresh("coords_done")
    a(f"s_cmp_eq_u32 {sr(S_G8)}, 0")
    a(f"s_cbranch_scc1 {lgen}")
    a(f"s_and_b32 {sr(t0 + 2)}, {sr(t1)}, 7")
    a(f"s_cmp_lg_u32 {sr(t0 + 2)}, 0")
    a(f"s_cbranch_scc1 {a.abort}")
    # XCD-grouped: xcd = id & 7, slot = id >> 3, gper = G / 8, per_rank = gper rep
    a(f"s_and_b32 {sr(S_T0 + 2)}, s2, 7")                  # xcd
    a(f"s_lshr_b32 {sr(S_T0 + 3)}, s2, 3")                 # slot
    a(f"s_lshr_b32 {sr(S_T0 + 4)}, {sr(t1)}, 3")           # gper
    a(f"s_mul_i32 {sr(S_T0 + 5)}, {sr(S_T0 + 4)}, {sr(S_REP)}")   # per_rank
    udiv(a, S_DQ, S_DR, S_T0 + 3, S_T0 + 5)                # rank, w2
    a(f"s_sub_u32 {sr(S_QB)}, {sr(S_NQB)}, 1")
    a(f"s_sub_u32 {sr(S_QB)}, {sr(S_QB)}, {sr(S_DQ)}")     # qb = nqb - 1 - rank
    a(f"s_mov_b32 {sr(S_T0 + 3)}, {sr(S_DR)}")
    udiv(a, S_DQ, S_DR, S_T0 + 3, S_REP)                   # gi, hr
    a(f"s_mul_i32 {sr(S_T0 + 2)}, {sr(S_T0 + 2)}, {sr(S_T0 + 4)}")
    a(f"s_add_u32 {sr(S_T0 + 2)}, {sr(S_T0 + 2)}, {sr(S_DQ)}")    # grp
    a(f"s_mov_b32 {sr(S_T0 + 5)}, {sr(S_DR)}")                    # hr
    udiv(a, S_DQ, S_DR, S_T0 + 2, S_HK)                    # b, grp % Hk
    a(f"s_mov_b32 {sr(S_BB)}, {sr(S_DQ)}")
    a(f"s_mul_i32 {sr(S_HH)}, {sr(S_DR)}, {sr(S_REP)}")
    a(f"s_add_u32 {sr(S_HH)}, {sr(S_HH)}, {sr(S_T0 + 5)}")
    a(f"s_branch {lcoord}")
    a.label(lgen)
    a(f"s_mul_i32 {sr(S_T0 + 2)}, {sr(S_H)}, {sr(S_B)}")
    udiv(a, S_DQ, S_DR, 2, S_T0 + 2)                       # rank, w2
    a(f"s_sub_u32 {sr(S_QB)}, {sr(S_NQB)}, 1")
    a(f"s_sub_u32 {sr(S_QB)}, {sr(S_QB)}, {sr(S_DQ)}")
    a(f"s_mov_b32 {sr(S_T0 + 3)}, {sr(S_DR)}")
    udiv(a, S_DQ, S_DR, S_T0 + 3, S_H)                     # b, h
    a(f"s_mov_b32 {sr(S_BB)}, {sr(S_DQ)}")
    a(f"s_mov_b32 {sr(S_HH)}, {sr(S_DR)}")
    a.label(lcoord)
    udiv(a, S_DQ, S_DR, S_HH, S_REP)
    a(f"s_mov_b32 {sr(S_HKV)}, {sr(S_DQ)}")
    # tiles T = 4 (qb + 1), unmasked bodies NU = max(4 qb - 1, 0)
    a(f"s_add_u32 {sr(S_T)}, {sr(S_QB)}, 1")
    a(f"s_lshl_b32 {sr(S_T)}, {sr(S_T)}, 2")
    a(f"s_sub_u32 {sr(S_TM1)}, {sr(S_T)}, 1")
    a(f"s_lshl_b32 {sr(S_NU)}, {sr(S_QB)}, 2")
    a(f"s_cmp_eq_u32 {sr(S_NU)}, 0")
    a(f"s_cselect_b32 {sr(t0)}, 0, 1")
    a(f"s_sub_u32 {sr(S_NU)}, {sr(S_NU)}, {sr(t0)}")
    # wave id, first query row of the wave
    a("s_nop 4")
    a(f"v_readfirstlane_b32 {sr(S_W)}, {vr(V_X + 15)}")
    a("s_nop 4")
    a(f"s_lshl_b32 {sr(S_Q0)}, {sr(S_QB)}, 8")
    a(f"s_lshl_b32 {sr(t0)}, {sr(S_W)}, 6")
    a(f"s_add_u32 {sr(S_Q0)}, {sr(S_Q0)}, {sr(t0)}")      # q0w = 256 qb + 64 w
    a(f"s_lshl_b32 {sr(S_W1K)}, {sr(S_W)}, 10")
    a(f"s_mov_b32 {sr(S_QSO)}, 8192")
    # --- buffer resources
    a(f"s_mul_i32 {sr(t0)}, {sr(S_BB)}, {sr(S_H)}")
    a(f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(S_HH)}")
    a(f"s_mul_i32 {sr(t0)}, {sr(t0)}, {sr(S_S)}")
    a(f"s_add_u32 {sr(t0)}, {sr(t0)}, {sr(S_Q0)}")        # (b H + h) S + q0w
    srd64(a, SRD_Q, S_Q, t0, ROWB, 64 * ROWB)
    srd64(a, SRD_L, S_L, t0, 4, 256)
    a(f"s_mul_i32 {sr(t1)}, {sr(S_BB)}, {sr(S_HK)}")
    a(f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(S_HKV)}")
    a(f"s_mul_i32 {sr(t1)}, {sr(t1)}, {sr(S_S)}")         # (b Hk + hk) S
    a(f"s_lshl_b32 {sr(S_T0 + 2)}, {sr(S_S)}, 8")         # S * 256 bytes
    srd64(a, SRD_K, S_K, t1, ROWB, sr(S_T0 + 2))
    srd64(a, SRD_V, S_V, t1, ROWB, sr(S_T0 + 2))
    lo_n, lo_d = a.fresh("o_bhsd"), a.fresh("o_done")
    a(f"s_bitcmp1_b32 {sr(S_FLAGS)}, 1")
    a(f"s_cbranch_scc0 {lo_n}")
    a(f"s_mul_i32 {sr(t1)}, {sr(S_BB)}, {sr(S_S)}")
    a(f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(S_Q0)}")
    a(f"s_mul_i32 {sr(t1)}, {sr(t1)}, {sr(S_H)}")
    a(f"s_add_u32 {sr(t1)}, {sr(t1)}, {sr(S_HH)}")        # (b S + q0w) H + h
    a(f"s_lshl_b32 {sr(S_OSTR)}, {sr(S_H)}, 8")
    a(f"s_branch {lo_d}")
    a.label(lo_n)
    a(f"s_mov_b32 {sr(t1)}, {sr(t0)}")
    a(f"s_mov_b32 {sr(S_OSTR)}, {ROWB}")
    a.label(lo_d)
    a(f"s_lshl_b32 {sr(S_OQB)}, {sr(S_OSTR)}, 5")         # 32 rows
    a(f"s_lshl_b32 {sr(S_T0 + 2)}, {sr(S_OSTR)}, 6")
    srd64(a, SRD_O, S_O, t1, ROWB, sr(S_T0 + 2))
    # --- lane constants
    l, g, pos, hh, r32, qq, pp = (V_X + i for i in range(7))
    a(f"v_and_b32 {vr(l)}, 63, v0")
    a(f"v_lshrrev_b32 {vr(g)}, 4, {vr(l)}")               # l >> 4
    a(f"v_and_b32 {vr(pos)}, 15, {vr(l)}")
    a(f"v_lshrrev_b32 {vr(hh)}, 5, {vr(l)}")
    a(f"v_and_b32 {vr(r32)}, 31, {vr(l)}")
    a(f"v_lshrrev_b32 {vr(qq)}, 2, {vr(pos)}")
    a(f"v_and_b32 {vr(pp)}, 3, {vr(l)}")
    t = V_T
    # DMA: K chunk pos ^ (4 w + (l >> 4)), V chunk pos ^ ((l >> 4) << 2)
    a(f"v_lshl_add_u32 {vr(t)}, {sr(S_W)}, 2, {vr(g)}")
    a(f"v_xor_b32 {vr(t)}, {vr(t)}, {vr(pos)}")
    a(f"v_lshlrev_b32 {vr(t)}, 4, {vr(t)}")
    a(f"v_lshl_add_u32 {vr(V_DK)}, {vr(g)}, 8, {vr(t)}")
    a(f"v_add_u32 {vr(V_DK)}, {sr(S_W1K)}, {vr(V_DK)}")
    a(f"v_lshlrev_b32 {vr(t)}, 2, {vr(g)}")
    a(f"v_xor_b32 {vr(t)}, {vr(t)}, {vr(pos)}")
    a(f"v_lshlrev_b32 {vr(t)}, 4, {vr(t)}")
    a(f"v_lshl_add_u32 {vr(V_DV)}, {vr(g)}, 8, {vr(t)}")
    a(f"v_add_u32 {vr(V_DV)}, {sr(S_W1K)}, {vr(V_DV)}")
    # K fragment reads: row r32, chunk (2 ds + hh) ^ pos (K buffer 0)
    for ds in range(8):
        a(f"v_add_u32 {vr(t)}, {2 * ds}, {vr(hh)}")
        a(f"v_xor_b32 {vr(t)}, {vr(t)}, {vr(pos)}")
        a(f"v_lshlrev_b32 {vr(t)}, 4, {vr(t)}")
        a(f"v_lshl_add_u32 {vr(V_KOFF + ds)}, {vr(r32)}, 8, {vr(t)}")
    # V^T reads: key 4 hh + qq, chunk 4 (dt ^ qq) + 2 (g & 1) + (pp >> 1), + 8 (pp & 1)
    a(f"v_lshl_add_u32 {vr(t + 1)}, {vr(hh)}, 2, {vr(qq)}")
    a(f"v_lshlrev_b32 {vr(t + 1)}, 8, {vr(t + 1)}")       # key * 256
    a(f"v_and_b32 {vr(t + 2)}, 1, {vr(g)}")
    a(f"v_lshlrev_b32 {vr(t + 2)}, 1, {vr(t + 2)}")
    a(f"v_lshrrev_b32 {vr(t + 3)}, 1, {vr(pp)}")
    a(f"v_add_u32 {vr(t + 2)}, {vr(t + 2)}, {vr(t + 3)}")  # 2 (g & 1) + (pp >> 1)
    a(f"v_and_b32 {vr(t + 3)}, 1, {vr(pp)}")
    a(f"v_lshlrev_b32 {vr(t + 3)}, 3, {vr(t + 3)}")        # 8 (pp & 1)
    a(f"v_add_u32 {vr(t + 1)}, {vr(t + 1)}, {vr(t + 3)}")
    a(f"v_add_u32 {vr(t + 1)}, {VBUF0}, {vr(t + 1)}")
    for dt in range(4):
        a(f"v_xor_b32 {vr(t)}, {dt}, {vr(qq)}")
        a(f"v_lshl_add_u32 {vr(t)}, {vr(t)}, 2, {vr(t + 2)}")
        a(f"v_lshl_add_u32 {vr(V_VOFF + dt)}, {vr(t)}, 4, {vr(t + 1)}")
    # mask base: q0w + r32 - 4 hh
    a(f"v_add_u32 {vr(V_E0)}, {sr(S_Q0)}, {vr(r32)}")
    a(f"v_lshlrev_b32 {vr(t)}, 2, {vr(hh)}")
    a(f"v_sub_u32 {vr(V_E0)}, {vr(V_E0)}, {vr(t)}")
    a(f"v_mov_b32 {vr(V_NEGINF)}, 0xff800000")
    for e in range(4):
        a(f"v_mov_b32 {vr(V_ONES + e)}, 0x3f803f80")
    # --- Q fragments (into score buffer 1 for now), K_0, V_0, K_1
    a(f"v_lshlrev_b32 {vr(t)}, 4, {vr(hh)}")
    a(f"v_lshl_add_u32 {vr(t)}, {vr(r32)}, 8, {vr(t)}")   # r32 * 256 + 16 hh
    for qb2 in range(2):
        for ds in range(8):
            a(f"buffer_load_dwordx4 {vr(V_SB[1] + 32 * qb2 + 4 * ds, 4)}, {vr(t)}, {sr(SRD_Q, 4)}, "
              f"{sr(S_QSO) if qb2 else '0'} offen offset:{32 * ds}")
    for kind, tile, buf in (("K", 0, 0), ("V", 0, None), ("K", 1, 1)):
        for j in range(4):
            a(f"s_mov_b32 {sr(S_SOFF)}, {tile * TILE + j * 4096}")
            if kind == "K":
                a(f"s_add_u32 m0, {sr(S_W1K)}, {buf * TILE + j * 4096}")
            else:
                a(f"s_add_u32 m0, {sr(S_W1K)}, {VBUF0 + j * 4096}")
            a("s_nop 0")
            a(f"buffer_load_dwordx4 {vr(V_DK if kind == 'K' else V_DV)}, {sr(SRD_K if kind == 'K' else SRD_V, 4)}, "
              f"{sr(S_SOFF)} offen lds")
    for x in range(128 + 32):
        a(f"v_accvgpr_write_b32 {ar(A_O + x if x < 128 else A_L + x - 128)}, 0")
    a("s_waitcnt vmcnt(0)")
    a("s_barrier")
    for qb2 in range(2):
        for x in range(32):
            a(f"v_accvgpr_write_b32 {ar(A_Q + 32 * qb2 + x)}, {vr(V_SB[1] + 32 * qb2 + x)}")
    a("s_nop 1")
    # --- S_0 = K_0 Q^T into score buffer 0
    items = [Item([kread(f)], 6, -1 if f < RING else 2 * (f - RING) + 1, max(-1, 2 * f - 4), "kr") for f in range(16)]
    schedule(a, qk_mfmas(0), items)
    a("s_nop 7")
    a("s_nop 7")
    a("s_nop 7")
    lskip = a.fresh("nomask0")
    a(f"s_cmp_lg_u32 {sr(S_QB)}, 0")
    a(f"s_cbranch_scc1 {lskip}")
    for x in mask_setup([f"s_mov_b32 {sr(S_T0 + 2)}, 0"]):
        a(x)
    for qb2 in range(2):
        for kh in range(2):
            for x in mask_ins(0, qb2, kh, range(16)):
                a(x)
    a.label(lskip)
    for qb2 in range(2):
        a_ops, b_ops = max_ops(0, qb2)
        for x in a_ops + b_ops + max_final(qb2):
            a(x)
        a(f"v_mov_b32 {vr(V_M + qb2)}, {vr(V_MC + qb2)}")
    # every wave done with K_0 (iteration 0 restages its buffer); K_1's first fragments
    a("s_barrier")
    for x in koff_toggle():
        a(x)
    for f in range(3):
        a(kread(f).split(";")[0])
    a(f"s_mov_b32 {sr(S_I)}, 0")
    a(f"s_mov_b32 {sr(S_VR)}, 0")
    a(f"s_add_u32 {sr(S_M0V)}, {sr(S_W1K)}, {VBUF0 + TILE}")
    stamp(a, 1)


# ---------------------------------------------------------------- epilogue
def timing_store(a: Asm):
    """Timing arm: 8 dwords per (workgroup, wave) at dbg + 32 (4 wg + wave):
    prologue, loop and epilogue cycles, tiles, query block, rescales, 0, 0."""
    if not KNOBS["timing"]:
        return
    stamp(a, 3)
    t = S_T0
    a(f"s_lshl_b32 {sr(t)}, s2, 2")
    a(f"s_add_u32 {sr(t)}, {sr(t)}, {sr(S_W)}")
    a(f"s_lshl_b32 {sr(t)}, {sr(t)}, 5")
    a(f"s_add_u32 {sr(SRD_Q)}, {sr(S_TM + 10)}, {sr(t)}")
    a(f"s_addc_u32 {sr(SRD_Q + 1)}, {sr(S_TM + 11)}, 0")
    a(f"s_mov_b32 {sr(SRD_Q + 2)}, 32")
    a(f"s_mov_b32 {sr(SRD_Q + 3)}, 0x20000")
    vals = [f"s_sub_u32 {sr(t)}, {sr(S_TM + 2)}, {sr(S_TM)}", f"s_sub_u32 {sr(t)}, {sr(S_TM + 4)}, {sr(S_TM + 2)}",
            f"s_sub_u32 {sr(t)}, {sr(S_TM + 6)}, {sr(S_TM + 4)}", f"s_mov_b32 {sr(t)}, {sr(S_T)}",
            f"s_mov_b32 {sr(t)}, {sr(S_QB)}", f"s_mov_b32 {sr(t)}, {sr(S_TM + 8)}"]
    a(f"v_mov_b32 {vr(V_T + 1)}, 0")
    for k, ins in enumerate(vals):
        a(ins)
        a(f"v_mov_b32 {vr(V_T)}, {sr(t)}")
        a(f"buffer_store_dword {vr(V_T)}, {vr(V_T + 1)}, {sr(SRD_Q, 4)}, 0 offen offset:{4 * k}")
    a("s_waitcnt vmcnt(0)")


def epilogue(a: Asm):
    stamp(a, 2)
    a("s_nop 7")
    a("s_nop 7")
    a("s_nop 7")
    lsum, inv, lv, oo = V_T, V_T + 1, V_T + 2, V_T + 3
    # lane offsets: O row r32 (stride S_OSTR) + 16 hh; LSE row r32
    hh, r32 = V_X, V_X + 1
    a(f"v_and_b32 {vr(r32)}, 31, v0")
    a(f"v_bfe_u32 {vr(hh)}, v0, 5, 1")
    a(f"v_mul_lo_u32 {vr(oo)}, {vr(r32)}, {sr(S_OSTR)}")
    a(f"v_lshl_add_u32 {vr(oo)}, {vr(hh)}, 4, {vr(oo)}")
    a(f"v_lshlrev_b32 {vr(lv)}, 2, {vr(r32)}")
    for qb2 in range(2):
        a(f"v_accvgpr_read_b32 {vr(lsum)}, {ar(A_L + 16 * qb2)}")
        a("s_nop 1")
        a(f"v_rcp_f32 {vr(inv)}, {vr(lsum)}")
        a("s_nop 4")
        for dt in range(4):
            for k in range(2):
                tmp = V_X + 2
                data = V_SB[0] + 4 * ((2 * (4 * qb2 + dt) + k) % 16)
                base = A_O + 64 * qb2 + 16 * dt + 8 * k      # groups g = 2k, 2k+1: regs 8k .. 8k+7
                for e in range(8):
                    a(f"v_accvgpr_read_b32 {vr(tmp + e)}, {ar(base + e)}")
                for e in range(8):
                    a(f"v_mul_f32 {vr(tmp + e)}, {vr(inv)}, {vr(tmp + e)}")
                for e in range(4):
                    a(f"v_cvt_pk_bf16_f32 {vr(data + e)}, {vr(tmp + 2 * e)}, {vr(tmp + 2 * e + 1)}")
                a("s_nop 1")
                a(f"v_permlane32_swap_b32 {vr(data)}, {vr(data + 2)}")
                a(f"v_permlane32_swap_b32 {vr(data + 1)}, {vr(data + 3)}")
                so = sr(S_OQB) if qb2 else "0"
                a(f"buffer_store_dwordx4 {vr(data, 4)}, {vr(oo)}, {sr(SRD_O, 4)}, {so} offen offset:{64 * dt + 32 * k}")
        # LSE = (m + log2 l) ln 2
        x = V_X + 10
        a(f"v_log_f32 {vr(x)}, {vr(lsum)}")
        a("s_nop 1")
        a(f"v_add_f32 {vr(x)}, {vr(V_M + qb2)}, {vr(x)}")
        a(f"v_mul_f32 {vr(x)}, 0x3f317218, {vr(x)}")
        a(f"buffer_store_dword {vr(x)}, {vr(lv)}, {sr(SRD_L, 4)}, 0 offen offset:{128 * qb2}")
    timing_store(a)


# ---------------------------------------------------------------- kernel
def kernel(variant: str = "") -> tuple[str, str]:
    name = NAME + (f"_{variant}" if variant else "")
    a = Asm(prefix=f"attn{variant}_")
    a.raw(f".globl {name}")
    a.raw(".p2align 8")
    a.raw(f".type {name},@function")
    a.raw(f"{name}:")
    prologue(a)
    lab = {k: a.fresh(k) for k in ("u0", "m0", "m1", "t0", "t1", "epi")}
    resc = {}
    # unmasked bodies, unrolled by two (i even, i odd)
    a.label(lab["u0"])
    a(f"s_cmp_ge_u32 {sr(S_I)}, {sr(S_NU)}")
    a(f"s_cbranch_scc1 {lab['m0']}")
    for p in (0, 1):
        resc[("U", p)] = (a.fresh(f"resc_u{p}"), a.fresh(f"back_u{p}"))
        body(a, "U", p, *resc[("U", p)])
        if p == 0:
            a(f"s_cmp_ge_u32 {sr(S_I)}, {sr(S_NU)}")
            a(f"s_cbranch_scc1 {lab['m1']}")
    a(f"s_branch {lab['u0']}")
    # masked bodies (the last 3-4 QK tiles), then the tail
    for p in (0, 1):
        a.label(lab[f"m{p}"])
        a(f"s_cmp_ge_u32 {sr(S_I)}, {sr(S_TM1)}")
        a(f"s_cbranch_scc1 {lab[f't{p}']}")
        resc[("M", p)] = (a.fresh(f"resc_m{p}"), a.fresh(f"back_m{p}"))
        body(a, "M", p, *resc[("M", p)])
        if p == 1:
            a(f"s_branch {lab['m0']}")
    for p in (0, 1):
        a.label(lab[f"t{p}"])
        body(a, "T", p, "", "")
        a(f"s_branch {lab['epi']}")
    a.label(lab["epi"])
    epilogue(a)
    a.label(a.abort)
    a("s_endpgm")
    for lbl, back in resc.values():
        rescale_block(a, lbl, back)
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


def generate_all() -> str:
    return generate(all_kernels())


if __name__ == "__main__":
    with open(sys.argv[1] if len(sys.argv) > 1 else "attn_fwd_asm.s", "w") as f:
        f.write(generate())
