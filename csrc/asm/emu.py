"""Functional emulator for the gfx950 instruction subset the assembly
generators in this directory emit (csrc/asm/gemm_gen.py).

It runs ONE workgroup of a generated kernel on the CPU: 4 wave64s in
lockstep between barriers, scalar/vector register files, the 160 KiB LDS,
buffer resources over numpy "global memory", LDS-DMA, ds_read_b128 and
v_mfma_f32_16x16x32_bf16 with the CDNA4 fragment layout.  Memory operations
complete immediately, so it checks ADDRESSING and data flow (every byte that
lands in LDS, every fragment a lane reads, every output element) -- not the
timing of waits, which the schedule's vmcnt / barrier placement is reasoned
about in the generator's docstring.  Any buffer access outside its
resource's num_records raises, so a bounds bug fails the CPU test instead of
being silently zero-filled on the GPU.

Used by tests/test_asm_gemm.py; no GPU, no assembler needed.
"""
from __future__ import annotations

import re
import struct

import numpy as np

M32 = 0xFFFFFFFF


def f2u(x):
    return np.asarray(x, dtype=np.float32).view(np.uint32)


def u2f(x):
    return np.asarray(x, dtype=np.uint32).view(np.float32)


def bf16_rne(f32: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 bits (uint32 holding 16 bits), round to nearest even."""
    u = f2u(f32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    return r.astype(np.uint32)


class Memory:
    """Flat 64-bit address space made of named numpy byte buffers."""

    def __init__(self):
        self.bufs: list[tuple[int, np.ndarray]] = []
        self.next = 1 << 32

    def add(self, arr: np.ndarray) -> int:
        b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        base = self.next
        self.bufs.append((base, b))
        self.next += ((b.size + (1 << 20)) >> 20 << 20) + (1 << 20)
        return base

    def add_at(self, base: int, arr: np.ndarray) -> int:
        """Map `arr` at a given address (mirror a real device pointer)."""
        b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        self.bufs.append((int(base), b))
        return int(base)

    def locate(self, addr: np.ndarray, nbytes: int):
        for base, b in self.bufs:
            if base <= int(addr.min()) and int(addr.max()) + nbytes <= base + b.size:
                return base, b
        raise IndexError(f"address range {hex(int(addr.min()))}..{hex(int(addr.max()))} outside every buffer")


# v_mfma_f32_32x32x16_bf16 D layout: register r of lane l holds row
# (r & 3) + 8 (r >> 2) + 4 (l >> 5), column l & 31
_LANES = np.arange(64)
_ROW32 = np.array([(r & 3) + 8 * (r >> 2) + 4 * (_LANES >> 5) for r in range(16)])
_COL32 = np.broadcast_to(_LANES & 31, (16, 64))
# ds_read_b64_tr_b16: lane 16 G + i takes element i & 3 of lane 16 G + 4 q + (i >> 2)
_TR_SRC = np.array([[16 * (l >> 4) + 4 * q + ((l & 15) >> 2) for q in range(4)] for l in range(64)])
_TR_ELT = np.broadcast_to((_LANES & 3)[:, None], (64, 4))

_REG = re.compile(r"^([vsa])(?:\[(\d+):(\d+)\]|(\d+))$")


class Wave:
    def __init__(self, wid: int, nvgpr=512):
        self.s = np.zeros(110, dtype=np.uint64)      # held as u64, masked to 32
        self.v = np.zeros((nvgpr, 64), dtype=np.uint32)   # v0..255, a0..255 at 256..
        self.scc = 0
        self.m0 = 0
        self.vcc = 0
        self.pc = 0
        self.done = False
        self.wid = wid
        self.vmq = []          # outstanding VMEM ops, oldest first (Emu.strict_vm)


class Emu:
    """strict_vm (default): a VMEM load lands -- in LDS for an LDS-DMA, in
    its VGPRs otherwise -- only when the issuing wave's s_waitcnt vmcnt(N)
    retires it (in issue order, stores counted too, as on gfx950) or the wave
    ends; its global data are read at issue.  A wait that counts too few
    outstanding ops therefore leaves stale LDS / VGPRs behind and the kernel's
    output wrong, as it would be on the hardware.  With strict_vm False every
    load lands at issue (the round-5 model)."""

    def __init__(self, asm_text: str, kernel: str, strict_vm: bool = True):
        self.prog, self.labels = self._parse(asm_text, kernel)
        self.strict_vm = strict_vm

    def _vm_issue(self, w, effect):
        """Queue a VMEM op's effect (None for a store: its memory write is
        made at issue; it only occupies a vmcnt slot)."""
        if self.strict_vm:
            w.vmq.append(effect)
        elif effect is not None:
            effect()

    def _vm_retire(self, w, keep: int):
        while len(w.vmq) > keep:
            eff = w.vmq.pop(0)
            if eff is not None:
                eff()

    # ------------------------------------------------------------ parsing
    @staticmethod
    def _parse(text: str, kernel: str):
        lines = text.splitlines()
        start = lines.index(f"{kernel}:")
        prog, labels = [], {}
        for ln in lines[start + 1:]:
            t = ln.split(";")[0].strip()
            if not t:
                continue
            if t.startswith(".size"):
                break
            if t.endswith(":"):
                labels[t[:-1]] = len(prog)
                continue
            if t.startswith("."):
                continue
            op, _, rest = t.partition(" ")
            args = [x.strip() for x in rest.split(",")] if rest else []
            # trailing modifiers ("offen lds", "offset:32") live in the last arg
            mods = []
            if args:
                parts = args[-1].split()
                args[-1] = parts[0]
                mods = parts[1:]
            prog.append((op, args, mods))
        return prog, labels

    # ------------------------------------------------------------ operands
    def _reg(self, w: Wave, tok: str):
        m = _REG.match(tok)
        if not m:
            return None
        kind = m.group(1)
        lo = int(m.group(2) if m.group(2) is not None else m.group(4))
        hi = int(m.group(3)) if m.group(3) is not None else lo
        return kind, lo, hi

    def sget(self, w: Wave, tok: str) -> int:
        if tok == "m0":
            return w.m0
        r = self._reg(w, tok)
        if r is not None:
            assert r[0] == "s" and r[1] == r[2], tok
            return int(w.s[r[1]]) & M32
        return self._lit(tok)

    @staticmethod
    def _lit(tok: str) -> int:
        if re.match(r"^-?\d+\.\d*(e-?\d+)?$", tok):
            return int(f2u(np.float32(float(tok))))
        v = int(tok, 0)
        return v & M32

    def sset(self, w: Wave, tok: str, val: int):
        if tok == "m0":
            w.m0 = val & M32
            return
        r = self._reg(w, tok)
        assert r and r[0] == "s" and r[1] == r[2], tok
        w.s[r[1]] = val & M32

    def vget(self, w: Wave, tok: str) -> np.ndarray:
        r = self._reg(w, tok)
        if r is None:
            return np.full(64, self.sget(w, tok), dtype=np.uint32) if not tok.startswith(("v", "a")) else None
        kind, lo, hi = r
        if kind == "s":
            return np.full(64, int(w.s[lo]) & M32, dtype=np.uint32)
        base = 256 if kind == "a" else 0
        assert lo == hi, tok
        return w.v[base + lo].copy()

    def vrange(self, w: Wave, tok: str):
        kind, lo, hi = self._reg(w, tok)
        base = 256 if kind == "a" else 0
        return base + lo, base + hi + 1

    def vset(self, w: Wave, tok: str, val):
        lo, hi = self.vrange(w, tok)
        assert hi == lo + 1, tok
        w.v[lo] = np.asarray(val).astype(np.uint32) & M32

    # ------------------------------------------------------------ run
    def run(self, kernarg: bytes, wg_id: int, mem: Memory, nthreads=256, lds_bytes=160 * 1024):
        self.mem = mem
        self.lds = np.zeros(lds_bytes, dtype=np.uint8)
        self.kernarg = kernarg
        waves = [Wave(i) for i in range(nthreads // 64)]
        for w in waves:
            w.s[2] = wg_id
            w.v[0] = np.arange(64, dtype=np.uint32) + 64 * w.wid
        steps = 0
        while not all(w.done for w in waves):
            for w in waves:           # each wave to its next barrier (or the end)
                while not w.done:
                    steps += 1
                    if steps > 50_000_000:
                        raise RuntimeError("emulator step limit")
                    if self.step(w) == "barrier":
                        break
        return steps

    def step(self, w: Wave):
        op, args, mods = self.prog[w.pc]
        w.pc += 1
        h = getattr(self, "op_" + op, None)
        if h is None:
            raise NotImplementedError(op)
        return h(w, args, mods)

    # ------------------------------------------------------------ SALU
    def op_s_load_dwordx16(self, w, a, m):
        self._sload(w, a, 16)

    def op_s_load_dwordx8(self, w, a, m):
        self._sload(w, a, 8)

    def op_s_load_dwordx4(self, w, a, m):
        self._sload(w, a, 4)

    def op_s_load_dwordx2(self, w, a, m):
        self._sload(w, a, 2)

    def op_s_load_dword(self, w, a, m):
        self._sload(w, a, 1)

    def op_s_sleep(self, w, a, m):
        """A wait with no architectural effect (the emulator has no clock)."""
        w.slept = getattr(w, "slept", 0) + 64 * self._lit(a[0])

    def op_s_memtime(self, w, a, m):
        """A monotonically increasing stand-in for the shader clock: this
        wave's instruction count (the timing kernel's records stay ordered)."""
        kind, lo, hi = self._reg(w, a[0])
        w.ticks = getattr(w, "ticks", 0) + 1000
        t = w.ticks + w.pc
        w.s[lo], w.s[lo + 1] = t & M32, t >> 32

    def _sload(self, w, a, n):
        kind, lo, hi = self._reg(w, a[0])
        off = self._lit(a[2])
        vals = struct.unpack_from(f"<{n}I", self.kernarg, off)
        for i, x in enumerate(vals):
            w.s[lo + i] = x

    def op_s_mov_b32(self, w, a, m):
        self.sset(w, a[0], self.sget(w, a[1]))

    def op_s_add_u32(self, w, a, m):
        r = self.sget(w, a[1]) + self.sget(w, a[2])
        w.scc = int(r > M32)
        self.sset(w, a[0], r)

    def op_s_addc_u32(self, w, a, m):
        r = self.sget(w, a[1]) + self.sget(w, a[2]) + w.scc
        w.scc = int(r > M32)
        self.sset(w, a[0], r)

    def op_s_sub_u32(self, w, a, m):
        x, y = self.sget(w, a[1]), self.sget(w, a[2])
        w.scc = int(y > x)
        self.sset(w, a[0], x - y)

    def op_s_subb_u32(self, w, a, m):
        x, y = self.sget(w, a[1]), self.sget(w, a[2]) + w.scc
        w.scc = int(y > x)
        self.sset(w, a[0], x - y)

    def op_s_sub_i32(self, w, a, m):
        self.sset(w, a[0], self.sget(w, a[1]) - self.sget(w, a[2]))

    def op_s_mul_i32(self, w, a, m):
        self.sset(w, a[0], self.sget(w, a[1]) * self.sget(w, a[2]))

    def op_s_mul_hi_u32(self, w, a, m):
        self.sset(w, a[0], (self.sget(w, a[1]) * self.sget(w, a[2])) >> 32)

    def op_s_lshl_b32(self, w, a, m):
        r = (self.sget(w, a[1]) << (self.sget(w, a[2]) & 31)) & M32
        w.scc = int(r != 0)
        self.sset(w, a[0], r)

    def op_s_lshr_b32(self, w, a, m):
        r = self.sget(w, a[1]) >> (self.sget(w, a[2]) & 31)
        w.scc = int(r != 0)
        self.sset(w, a[0], r)

    def op_s_and_b32(self, w, a, m):
        r = self.sget(w, a[1]) & self.sget(w, a[2])
        w.scc = int(r != 0)
        self.sset(w, a[0], r)

    def op_s_xor_b32(self, w, a, m):
        r = self.sget(w, a[1]) ^ self.sget(w, a[2])
        w.scc = int(r != 0)
        self.sset(w, a[0], r)

    def op_s_bitcmp1_b32(self, w, a, m):
        w.scc = int((self.sget(w, a[0]) >> (self.sget(w, a[1]) & 31)) & 1)

    def op_s_min_u32(self, w, a, m):
        x, y = self.sget(w, a[1]), self.sget(w, a[2])
        w.scc = int(x < y)
        self.sset(w, a[0], min(x, y))

    @staticmethod
    def _i32(x):
        return x - (1 << 32) if x & 0x80000000 else x

    def op_s_cmp_eq_u32(self, w, a, m):
        w.scc = int(self.sget(w, a[0]) == self.sget(w, a[1]))

    def op_s_cmp_lg_u32(self, w, a, m):
        w.scc = int(self.sget(w, a[0]) != self.sget(w, a[1]))

    def op_s_cmp_gt_u32(self, w, a, m):
        w.scc = int(self.sget(w, a[0]) > self.sget(w, a[1]))

    def op_s_cmp_lt_u32(self, w, a, m):
        w.scc = int(self.sget(w, a[0]) < self.sget(w, a[1]))

    def op_s_cmp_ge_u32(self, w, a, m):
        w.scc = int(self.sget(w, a[0]) >= self.sget(w, a[1]))

    def op_s_cmp_lt_i32(self, w, a, m):
        w.scc = int(self._i32(self.sget(w, a[0])) < self._i32(self.sget(w, a[1])))

    def op_s_cselect_b32(self, w, a, m):
        self.sset(w, a[0], self.sget(w, a[1]) if w.scc else self.sget(w, a[2]))

    def op_s_cbranch_scc0(self, w, a, m):
        if not w.scc:
            w.pc = self.labels[a[0]]

    def op_s_cbranch_scc1(self, w, a, m):
        if w.scc:
            w.pc = self.labels[a[0]]

    def op_s_branch(self, w, a, m):
        w.pc = self.labels[a[0]]

    def op_s_getreg_b32(self, w, a, m):
        """hwreg(HW_REG_HW_ID, offset, size) only: wave id in [3:0], SIMD id
        in [5:4].  Waves 0..3 sit on SIMDs 0, 2, 1, 3 (the hardware's cyclic
        placement from SIMD 0), so both SIMD-parity paths of a kernel run."""
        assert a[1].replace(" ", "") == "hwreg(HW_REG_HW_ID", a
        off, size = int(a[2]), int(a[3].rstrip(")"))
        hw_id = ([0, 2, 1, 3][w.wid % 4] << 4) | w.wid
        self.sset(w, a[0], (hw_id >> off) & ((1 << size) - 1))

    def op_s_waitcnt(self, w, a, m):
        for tok in list(a) + list(m):
            for part in str(tok).split():
                if part.startswith("vmcnt("):
                    self._vm_retire(w, int(part[6:].rstrip(")")))

    def op_s_nop(self, w, a, m):
        pass

    def op_s_setprio(self, w, a, m):
        pass

    def op_s_barrier(self, w, a, m):
        return "barrier"

    def op_s_endpgm(self, w, a, m):
        self._vm_retire(w, 0)
        w.done = True
        return "barrier"

    # ------------------------------------------------------------ VALU
    def _vbin(self, w, a, fn):
        self.vset(w, a[0], fn(self.vget(w, a[1]), self.vget(w, a[2])))

    def op_v_mov_b32(self, w, a, m):
        self.vset(w, a[0], self.vget(w, a[1]))

    def op_v_cvt_f32_u32(self, w, a, m):
        self.vset(w, a[0], f2u(self.vget(w, a[1]).astype(np.float32)))

    def op_v_cvt_u32_f32(self, w, a, m):
        f = u2f(self.vget(w, a[1]))
        self.vset(w, a[0], np.clip(np.trunc(f), 0, M32).astype(np.uint64).astype(np.uint32))

    def op_v_rcp_iflag_f32(self, w, a, m):
        with np.errstate(divide="ignore"):
            self.vset(w, a[0], f2u(np.float32(1.0) / u2f(self.vget(w, a[1]))))

    op_v_rcp_f32 = op_v_rcp_iflag_f32

    def op_v_mul_f32(self, w, a, m):
        self._vbin(w, a, lambda x, y: f2u(u2f(x) * u2f(y)))

    def op_v_add_f32(self, w, a, m):
        self._vbin(w, a, lambda x, y: f2u(u2f(x) + u2f(y)))

    def op_v_sub_f32(self, w, a, m):
        self._vbin(w, a, lambda x, y: f2u(u2f(x) - u2f(y)))

    def op_v_exp_f32(self, w, a, m):
        self.vset(w, a[0], f2u(np.exp2(u2f(self.vget(w, a[1]))).astype(np.float32)))

    def op_v_readfirstlane_b32(self, w, a, m):
        self.sset(w, a[0], int(self.vget(w, a[1])[0]))

    def op_v_lshrrev_b32(self, w, a, m):
        self._vbin(w, a, lambda s, x: x >> (s & 31))

    def op_v_lshlrev_b32(self, w, a, m):
        self._vbin(w, a, lambda s, x: (x.astype(np.uint64) << (s & 31)).astype(np.uint64) & M32)

    def op_v_and_b32(self, w, a, m):
        self._vbin(w, a, lambda x, y: x & y)

    def op_v_xor_b32(self, w, a, m):
        self._vbin(w, a, lambda x, y: x ^ y)

    def op_v_add_u32(self, w, a, m):
        self._vbin(w, a, lambda x, y: (x.astype(np.uint64) + y) & M32)

    def op_v_mul_lo_u32(self, w, a, m):
        self._vbin(w, a, lambda x, y: (x.astype(np.uint64) * y) & M32)

    def op_v_bfe_u32(self, w, a, m):
        x, off, width = (self.vget(w, t) for t in a[1:4])
        self.vset(w, a[0], (x >> (off & 31)) & ((1 << (width & 31)) - 1))

    def op_v_mul_u32_u24(self, w, a, m):
        self._vbin(w, a, lambda x, y: ((x & 0xFFFFFF).astype(np.uint64) * (y & 0xFFFFFF)) & M32)

    def op_v_lshl_add_u32(self, w, a, m):
        x, s, y = (self.vget(w, t) for t in a[1:4])
        self.vset(w, a[0], ((x.astype(np.uint64) << (s & 31)) + y) & M32)

    # --- attention-forward subset (csrc/asm/attn_gen.py)
    def op_v_max_f32(self, w, a, m):
        self._vbin(w, a, lambda x, y: f2u(np.maximum(u2f(x), u2f(y))))

    def op_v_max3_f32(self, w, a, m):
        x, y, z = (u2f(self.vget(w, t)) for t in a[1:4])
        self.vset(w, a[0], f2u(np.maximum(np.maximum(x, y), z)))

    def op_v_log_f32(self, w, a, m):
        with np.errstate(divide="ignore"):
            self.vset(w, a[0], f2u(np.log2(u2f(self.vget(w, a[1]))).astype(np.float32)))

    def _fop(self, w, tok):
        """A float operand with an optional leading '-' (VOP3 neg modifier)."""
        if tok.startswith("-") and self._reg(w, tok[1:]) is not None:
            return -u2f(self.vget(w, tok[1:]))
        return u2f(self.vget(w, tok))

    def op_v_fma_f32(self, w, a, m):
        x, y, z = (self._fop(w, t).astype(np.float64) for t in a[1:4])
        self.vset(w, a[0], f2u((x * y + z).astype(np.float32)))

    def _pair(self, w, tok) -> np.ndarray:
        lo, hi = self.vrange(w, tok)
        assert hi == lo + 2 and lo % 2 == 0, tok   # 64-bit operands: even-aligned pairs
        return u2f(w.v[lo:hi]).astype(np.float64)

    def op_v_pk_fma_f32(self, w, a, m):
        """Two fp32 FMAs on register pairs (op_sel defaults: low with low)."""
        x, y, z = (self._pair(w, t) for t in a[1:4])
        lo, hi = self.vrange(w, a[0])
        w.v[lo:hi] = f2u((x * y + z).astype(np.float32))

    def op_v_pk_add_f32(self, w, a, m):
        x, y = (self._pair(w, t) for t in a[1:3])
        lo, hi = self.vrange(w, a[0])
        w.v[lo:hi] = f2u((x + y).astype(np.float32))

    def op_v_pk_mul_f32(self, w, a, m):
        x, y = (self._pair(w, t) for t in a[1:3])
        lo, hi = self.vrange(w, a[0])
        w.v[lo:hi] = f2u((x * y).astype(np.float32))

    def op_v_sub_u32(self, w, a, m):
        self._vbin(w, a, lambda x, y: (x.astype(np.int64) - y.astype(np.int64)) & M32)

    def op_v_subrev_u32(self, w, a, m):
        self._vbin(w, a, lambda x, y: (y.astype(np.int64) - x.astype(np.int64)) & M32)

    def op_v_or_b32(self, w, a, m):
        self._vbin(w, a, lambda x, y: x | y)

    def op_v_permlane32_swap_b32(self, w, a, m):
        """lanes 32..63 of vdst <-> lanes 0..31 of vsrc."""
        d0, _ = self.vrange(w, a[0])
        s0, _ = self.vrange(w, a[1])
        hi = w.v[d0, 32:].copy()
        w.v[d0, 32:] = w.v[s0, :32]
        w.v[s0, :32] = hi

    def _mask(self, w, tok) -> np.ndarray:
        if tok == "vcc":
            v = w.vcc
        else:
            kind, lo, hi = self._reg(w, tok)
            v = (int(w.s[lo]) & M32) | ((int(w.s[lo + 1]) & M32) << 32)
        return np.array([(v >> l) & 1 for l in range(64)], dtype=bool)

    def _set_mask(self, w, tok, bits: np.ndarray):
        v = int(sum(1 << l for l in range(64) if bits[l]))
        if tok == "vcc":
            w.vcc = v
        else:
            kind, lo, hi = self._reg(w, tok)
            w.s[lo], w.s[lo + 1] = v & M32, v >> 32

    def op_v_cmp_gt_f32(self, w, a, m):
        self._set_mask(w, a[0], u2f(self.vget(w, a[1])) > u2f(self.vget(w, a[2])))

    def op_v_cmp_gt_i32(self, w, a, m):
        x = self.vget(w, a[1]).view(np.int32)
        y = self.vget(w, a[2]).view(np.int32)
        self._set_mask(w, a[0], x > y)

    def op_v_cmp_lt_i32(self, w, a, m):
        x = self.vget(w, a[1]).view(np.int32)
        y = self.vget(w, a[2]).view(np.int32)
        self._set_mask(w, a[0], x < y)

    def op_v_cndmask_b32(self, w, a, m):
        """vdst = mask ? src1 : src0"""
        sel = self._mask(w, a[3])
        self.vset(w, a[0], np.where(sel, self.vget(w, a[2]), self.vget(w, a[1])))

    def op_s_or_b64(self, w, a, m):
        bits = self._mask(w, a[1]) | self._mask(w, a[2])
        self._set_mask(w, a[0], bits)
        w.scc = int(bits.any())

    def op_s_mov_b64(self, w, a, m):
        if a[1] == "vcc" or a[1].startswith("s["):
            bits = self._mask(w, a[1])
        else:
            v = int(a[1], 0) & ((1 << 64) - 1)
            bits = np.array([(v >> l) & 1 for l in range(64)], dtype=bool)
        self._set_mask(w, a[0], bits)

    def op_s_cmp_eq_u64(self, w, a, m):
        x = self._mask(w, a[0])
        v = int(a[1], 0)
        y = np.array([(v >> l) & 1 for l in range(64)], dtype=bool)
        w.scc = int((x == y).all())

    def op_s_cbranch_vccz(self, w, a, m):
        if w.vcc == 0:
            w.pc = self.labels[a[0]]

    def op_v_mfma_f32_32x32x16_bf16(self, w, a, m):
        """D[32x32] = A[32x16] B[16x32] + C.  Lane l: A row l&31, k 8(l>>5)..+7;
        B k 8(l>>5)..+7, column l&31; D/C register r: row (r&3) + 8(r>>2) +
        4(l>>5), column l&31.  srcC may be the inline constant 0."""
        d0, d1 = self.vrange(w, a[0])
        a0, a1 = self.vrange(w, a[1])
        b0, b1 = self.vrange(w, a[2])
        assert d1 - d0 == 16 and a1 - a0 == 4 and b1 - b0 == 4

        def elems(r0):
            regs = w.v[r0:r0 + 4].T
            out = np.empty((64, 8), dtype=np.uint32)
            out[:, 0::2] = (regs & 0xFFFF) << 16
            out[:, 1::2] = regs & 0xFFFF0000
            return u2f(out)

        ea, eb = elems(a0).astype(np.float64), elems(b0).astype(np.float64)
        A = np.concatenate([ea[:32], ea[32:]], axis=1)        # [32 rows, 16 k]
        B = np.concatenate([eb[:32], eb[32:]], axis=1).T      # [16 k, 32 cols]
        D = A @ B
        if a[3] == "0":
            C = np.zeros((16, 64), np.float64)
        else:
            c0, c1 = self.vrange(w, a[3])
            assert c1 - c0 == 16
            C = u2f(w.v[c0:c0 + 16]).astype(np.float64)
        out = C + D[_ROW32, _COL32]
        w.v[d0:d0 + 16] = f2u(out.astype(np.float32))

    def op_v_accvgpr_write_b32(self, w, a, m):
        self.vset(w, a[0], self.vget(w, a[1]))

    def op_v_accvgpr_read_b32(self, w, a, m):
        self.vset(w, a[0], self.vget(w, a[1]))

    def op_v_cvt_pk_bf16_f32(self, w, a, m):
        lo = bf16_rne(u2f(self.vget(w, a[1])))
        hi = bf16_rne(u2f(self.vget(w, a[2])))
        self.vset(w, a[0], lo | (hi << 16))

    def op_v_mfma_f32_16x16x32_bf16(self, w, a, m):
        d0, d1 = self.vrange(w, a[0])
        a0, a1 = self.vrange(w, a[1])
        b0, b1 = self.vrange(w, a[2])
        c_zero = a[3] == "0"          # srcC may be the inline constant 0
        c0, c1 = (0, 4) if c_zero else self.vrange(w, a[3])
        assert d1 - d0 == 4 and a1 - a0 == 4 and b1 - b0 == 4 and c1 - c0 == 4

        def elems(r0):  # [64 lanes, 8] bf16 -> f32
            regs = w.v[r0:r0 + 4].T  # [64, 4] u32
            lo = (regs & 0xFFFF) << 16
            hi = regs & 0xFFFF0000
            out = np.empty((64, 8), dtype=np.uint32)
            out[:, 0::2] = lo
            out[:, 1::2] = hi
            return u2f(out)

        ea, eb = elems(a0), elems(b0)
        A = np.zeros((16, 32), np.float32)
        B = np.zeros((32, 16), np.float32)
        for l in range(64):
            A[l & 15, 8 * (l >> 4): 8 * (l >> 4) + 8] = ea[l]
            B[8 * (l >> 4): 8 * (l >> 4) + 8, l & 15] = eb[l]
        D = A.astype(np.float64) @ B.astype(np.float64)
        C = np.zeros((4, 64)) if c_zero else u2f(w.v[c0:c0 + 4]).astype(np.float64)     # [4, 64]
        out = np.empty((4, 64), np.float64)
        for l in range(64):
            for r in range(4):
                out[r, l] = C[r, l] + D[(l >> 4) * 4 + r, l & 15]
        w.v[d0:d0 + 4] = f2u(out.astype(np.float32))

    # ------------------------------------------------------------ memory
    def _buffer_addr(self, w, a, mods, nbytes):
        voff = self.vget(w, a[0]).astype(np.uint64)
        kind, lo, hi = self._reg(w, a[1])
        srd = [int(w.s[lo + i]) & M32 for i in range(4)]
        base = srd[0] | ((srd[1] & 0xFFFF) << 32)
        nrec = srd[2]
        soff = self.sget(w, a[2])
        ioff = 0
        for md in mods:
            if md.startswith("offset:"):
                ioff = int(md.split(":")[1])
        off = voff + soff + ioff
        if int(off.max()) + nbytes > nrec:
            raise IndexError(f"buffer access past num_records ({int(off.max())} + {nbytes} > {nrec})")
        return base + off

    def _gread(self, addr, nbytes):
        base, buf = self.mem.locate(addr, nbytes)
        rel = (addr - base).astype(np.int64)
        return np.stack([buf[rel + i] for i in range(nbytes)], axis=1)  # [64, nbytes]

    def _gwrite(self, addr, data):
        nbytes = data.shape[1]
        base, buf = self.mem.locate(addr, nbytes)
        rel = (addr - base).astype(np.int64)
        for i in range(nbytes):
            buf[rel + i] = data[:, i]

    def op_buffer_load_dwordx4(self, w, a, mods):
        if "lds" not in mods:
            addr = self._buffer_addr(w, a[1:], mods, 16)
            data = self._gread(addr, 16).view(np.uint32).reshape(64, 4)
            lo, hi = self.vrange(w, a[0])

            def land(lo=lo, hi=hi, data=data):
                w.v[lo:hi] = data.T
            self._vm_issue(w, land)
            return
        assert "offen" in mods
        addr = self._buffer_addr(w, a, mods, 16)
        data = self._gread(addr, 16)
        dst = w.m0 + 16 * np.arange(64)
        if dst.max() + 16 > self.lds.size:
            raise IndexError("LDS-DMA past the LDS")

        def land(dst=dst, data=data):
            for l in range(64):
                self.lds[dst[l]:dst[l] + 16] = data[l]
        self._vm_issue(w, land)

    def op_buffer_load_dword(self, w, a, mods):
        """4-B load into a VGPR.  Lanes past num_records read 0, as on the
        hardware (kept for prefetch-style loads whose result is discarded;
        the product kernels do not issue this form).  Every other buffer
        access past num_records raises."""
        if "lds" in mods:        # LDS-DMA, 4 B per lane to M0 + 4 lane
            assert "offen" in mods
            addr = self._buffer_addr(w, a, mods, 4)
            data = self._gread(addr, 4)
            dst = w.m0 + 4 * np.arange(64)
            if dst.max() + 4 > self.lds.size:
                raise IndexError("LDS-DMA past the LDS")

            def land(dst=dst, data=data):
                for l in range(64):
                    self.lds[dst[l]:dst[l] + 4] = data[l]
            self._vm_issue(w, land)
            return
        voff = self.vget(w, a[1]).astype(np.uint64)
        kind, lo_, hi_ = self._reg(w, a[2])
        srd = [int(w.s[lo_ + i]) & M32 for i in range(4)]
        base, nrec = srd[0] | ((srd[1] & 0xFFFF) << 32), srd[2]
        ioff = 0
        for md in mods:
            if md.startswith("offset:"):
                ioff = int(md.split(":")[1])
        off = voff + self.sget(w, a[3]) + ioff
        out = np.zeros(64, np.uint32)
        ok = off + 4 <= nrec
        if ok.any():
            addr = base + off[ok]
            b0, buf = self.mem.locate(addr, 4)
            rel = (addr - b0).astype(np.int64)
            out[ok] = np.stack([buf[rel + i] for i in range(4)], axis=1).view(np.uint32).reshape(-1)
        lo, hi = self.vrange(w, a[0])

        def land(lo=lo, out=out):
            w.v[lo] = out
        self._vm_issue(w, land)

    def op_buffer_load_dwordx2(self, w, a, mods):
        addr = self._buffer_addr(w, a[1:], mods, 8)
        data = self._gread(addr, 8).view(np.uint32).reshape(64, 2)
        lo, hi = self.vrange(w, a[0])

        def land(lo=lo, hi=hi, data=data):
            w.v[lo:hi] = data.T
        self._vm_issue(w, land)

    def _dropped(self, w, a) -> bool:
        """A store through a resource of num_records 0 writes nothing (the
        hardware's range check; attn_bwd_gen.py drops the dS stores of
        blocks above the diagonal this way).  Counted in self.dropped."""
        kind, lo, hi = self._reg(w, a[2])
        if int(w.s[lo + 2]) & M32 == 0:
            self.dropped = getattr(self, "dropped", 0) + 1
            return True
        return False

    def op_buffer_store_dword(self, w, a, mods):
        self._vm_issue(w, None)
        if self._dropped(w, a):
            return
        addr = self._buffer_addr(w, a[1:], mods, 4)
        lo, hi = self.vrange(w, a[0])
        self._gwrite(addr, np.ascontiguousarray(w.v[lo]).view(np.uint8).reshape(64, 4))

    def op_buffer_store_dwordx4(self, w, a, mods):
        self._vm_issue(w, None)
        if self._dropped(w, a):
            return
        addr = self._buffer_addr(w, a[1:], mods, 16)
        lo, hi = self.vrange(w, a[0])
        self._gwrite(addr, np.ascontiguousarray(w.v[lo:hi].T).view(np.uint8).reshape(64, 16))

    def op_buffer_store_dwordx2(self, w, a, mods):
        self._vm_issue(w, None)
        if self._dropped(w, a):
            return
        addr = self._buffer_addr(w, a[1:], mods, 8)
        lo, hi = self.vrange(w, a[0])
        data = np.ascontiguousarray(w.v[lo:hi].T).view(np.uint8).reshape(64, 8)
        self._gwrite(addr, data)

    def op_ds_read_b64_tr_b16(self, w, a, mods):
        """Transposed 64-bit read: lane 16 G + 4 q + p reads four bf16 at its
        address; lane 16 G + i receives element i & 3 of lane 16 G + 4 q +
        (i >> 2) for q = 0..3 (its column, four rows)."""
        addr = self.vget(w, a[1]).astype(np.int64)
        for md in mods:
            if md.startswith("offset:"):
                addr = addr + int(md.split(":")[1])
        if addr.max() + 8 > self.lds.size:
            raise IndexError("ds_read past the LDS")
        src = np.stack([self.lds[x:x + 8] for x in addr]).view(np.uint16).reshape(64, 4)
        out = np.ascontiguousarray(src[_TR_SRC, _TR_ELT])
        lo, hi = self.vrange(w, a[0])
        w.v[lo:hi] = out.view(np.uint32).reshape(64, 2).T

    def _ds_addr(self, w, tok, mods, nbytes):
        addr = self.vget(w, tok).astype(np.int64)
        for md in mods:
            if md.startswith("offset:"):
                addr = addr + int(md.split(":")[1])
        if addr.min() < 0 or addr.max() + nbytes > self.lds.size:
            raise IndexError("ds access past the LDS")
        return addr

    def op_ds_write_b32(self, w, a, mods):
        addr = self._ds_addr(w, a[0], mods, 4)
        data = self.vget(w, a[1]).astype(np.uint32)
        for l in range(64):
            self.lds[addr[l]:addr[l] + 4] = np.frombuffer(np.uint32(data[l]).tobytes(), np.uint8)

    def op_ds_read_b32(self, w, a, mods):
        addr = self._ds_addr(w, a[1], mods, 4)
        lo, hi = self.vrange(w, a[0])
        w.v[lo] = np.array([self.lds[x:x + 4].view(np.uint32)[0] for x in addr], dtype=np.uint32)

    def op_ds_read_b128(self, w, a, mods):
        addr = self.vget(w, a[1]).astype(np.int64)
        for md in mods:
            if md.startswith("offset:"):
                addr = addr + int(md.split(":")[1])
        if addr.max() + 16 > self.lds.size:
            raise IndexError("ds_read past the LDS")
        lo, hi = self.vrange(w, a[0])
        data = np.stack([self.lds[x:x + 16] for x in addr]).view(np.uint32).reshape(64, 4)
        w.v[lo:hi] = data.T
