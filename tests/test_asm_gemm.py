"""CPU tests of the hand-written gfx950 assembly GEMMs (csrc/asm/gemm_gen.py).

The generated kernels run one workgroup at a time in the functional emulator
(csrc/asm/emu.py): every LDS-DMA byte, fragment read, MFMA, accumulator read
and output store of the real instruction stream, compared with a float64
reference of the same op.  A buffer access outside its resource's
num_records fails the test (on the GPU it would silently read zeros).
The GPU tests (tests/test_ops_gpu.py::test_gemm_asm_*) run the same kernels on
an MI355X."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ASM = os.path.join(os.path.dirname(HERE), "csrc", "asm")
sys.path.insert(0, ASM)

import emu  # noqa: E402
import gemm_gen  # noqa: E402
import host_args  # noqa: E402

TEXT = gemm_gen.generate()


def bf16(x):
    return emu.bf16_rne(np.asarray(x, np.float32)).astype(np.uint16)


def tof(b):
    return (b.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def run_all(kernel, karg, nwg, mem):
    e = emu.Emu(TEXT, kernel)
    for wg in range(nwg):
        e.run(karg, wg, mem)


def close(got, ref, tol=8e-3):
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err < tol, err


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 320)])
def test_asm_gemm_plain_emulated(M, N, K):
    rng = np.random.default_rng(M + N + K)
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((N, K)))
    mem = emu.Memory()
    ax, aw, ac = mem.add(X), mem.add(W), mem.add(np.zeros((M, N), np.uint16))
    karg = host_args.pack(ax, aw, ac, 0, 2 * K, 2 * K, 2 * N, 0, K, M // 256, N // 256)
    run_all("toa_gemm_tn_asm_plain", karg, (M // 256) * (N // 256), mem)
    C = tof(mem.bufs[2][1].view(np.uint16).reshape(M, N))
    ref = tof(X) @ tof(W).T
    close(C, ref)
    # exact to bf16 rounding of the fp32 sum: at most one bf16 ulp apart
    assert np.mean(np.abs(C - tof(bf16(ref))) <= np.abs(ref) * 2 ** -7) > 0.999


@pytest.mark.parametrize("variant", [v for v, k in gemm_gen.PLAIN_VARIANTS if not k.get("diag")])
def test_asm_gemm_variants_match_product_kernel(variant):
    """Each A/B arm of the plain kernel (other LDS pad, DMA spacing, wait slot,
    row-group size) writes exactly the product kernel's C on a 5 x 2 grid."""
    rng = np.random.default_rng(11)
    M, N, K = 1280, 512, 384   # 6 k-tiles: the loop runs (DMA, L2 prefetch past K)
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((N, K)))
    out = []
    persist = dict(gemm_gen.PLAIN_VARIANTS)[variant].get("persist")
    for name in ("toa_gemm_tn_asm_plain", f"toa_gemm_tn_asm_plain_{variant}"):
        mem = emu.Memory()
        ax, aw, ac = mem.add(X), mem.add(W), mem.add(np.zeros((M, N), np.uint16))
        nwg = (M // 256) * (N // 256)
        karg = host_args.pack(ax, aw, ac, 0, 2 * K, 2 * K, 2 * N, 0, K, M // 256, N // 256,
                              grid=nwg if persist else None)
        run_all(name, karg, nwg, mem)
        out.append(mem.bufs[2][1].view(np.uint16).reshape(M, N).copy())
    assert np.array_equal(out[0], out[1])
    close(tof(out[0]), tof(X) @ tof(W).T)


PERSIST_ARMS = [v for v, k in gemm_gen.PLAIN_VARIANTS if k.get("persist") and k.get("store_nt", True)]


@pytest.mark.parametrize("arm", PERSIST_ARMS)
@pytest.mark.parametrize("grid,K", [(1, 320), (3, 320), (10, 320), (3, 192), (4, 256)])
def test_asm_gemm_persistent_arm_emulated(arm, grid, K):
    """The persistent arms: `grid` workgroups walk the 10 tiles of a 5 x 2
    grid (S_ITER += grid), staging the next tile under the epilogue (v3) or
    parking the finished tile's C in AGPRs and storing it during the next
    tile's first k-iteration (v9, deferred stores: the first tile's stores
    dropped by a zero-size resource, the last tile's stored at once); C
    equals the product kernel's bit for bit.  K = 320: odd k-tile count (the
    stage parity fix-up); 192: v9's peeled first iteration and no loop."""
    name = f"toa_gemm_tn_asm_plain_{arm}"
    rng = np.random.default_rng(13)
    M, N = 1280, 512
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((N, K)))
    outs = []
    for kname, g in (("toa_gemm_tn_asm_plain", None), (name, grid)):
        mem = emu.Memory()
        ax, aw, ac = mem.add(X), mem.add(W), mem.add(np.zeros((M, N), np.uint16))
        karg = host_args.pack(ax, aw, ac, 0, 2 * K, 2 * K, 2 * N, 0, K, M // 256, N // 256, grid=g)
        run_all(kname, karg, (M // 256) * (N // 256) if g is None else g, mem)
        outs.append(mem.bufs[2][1].view(np.uint16).reshape(M, N).copy())
    assert np.array_equal(outs[0], outs[1])


def test_asm_gemm_timing_kernel_emulated():
    """The timing diagnostic computes the product kernel's C and writes one
    8-dword record per (workgroup, wave) with ordered stamps."""
    rng = np.random.default_rng(5)
    M, N, K = 512, 256, 384
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((N, K)))
    mem = emu.Memory()
    ax, aw, ac = mem.add(X), mem.add(W), mem.add(np.zeros((M, N), np.uint16))
    nwg = (M // 256) * (N // 256)
    at = mem.add(np.zeros(nwg * 4 * 8, np.uint32))
    karg = host_args.pack(ax, aw, ac, at, 2 * K, 2 * K, 2 * N, 0, K, M // 256, N // 256)
    run_all("toa_gemm_tn_asm_timing", karg, nwg, mem)
    close(tof(mem.bufs[2][1].view(np.uint16).reshape(M, N)), tof(X) @ tof(W).T)
    rec = mem.bufs[3][1].view(np.uint32).reshape(nwg, 4, 8)
    assert (rec[:, :, 5] == K // 64).all() and (rec[:, :, 6] == np.arange(nwg)[:, None]).all()
    assert (rec[:, :, 3] > 0).all() and (rec[:, :, 4] > 0).all()


@pytest.mark.parametrize("phase", [0x10003, 0x20001])
def test_asm_gemm_phase_offsets_same_output(phase):
    """The first wave's start offsets (gemm_gen.phase_delay) change only when
    a workgroup starts: C is the product kernel's bit for bit (the grid spans
    three phase groups, so the sleep loop runs for some workgroups)."""
    rng = np.random.default_rng(19)
    M, N, K = 512, 2560, 128      # 20 workgroups: groups (b >> 3) 0, 1, 2
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((N, K)))
    outs, slept = [], []
    for ph in (0, phase):
        mem = emu.Memory()
        ax, aw, ac = mem.add(X), mem.add(W), mem.add(np.zeros((M, N), np.uint16))
        karg = host_args.pack(ax, aw, ac, 0, 2 * K, 2 * K, 2 * N, 0, K, M // 256, N // 256, phase=ph)
        e = emu.Emu(TEXT, "toa_gemm_tn_asm_plain")
        for wg in range((M // 256) * (N // 256)):
            e.run(karg, wg, mem)
        outs.append(mem.bufs[2][1].view(np.uint16).reshape(M, N).copy())
    assert np.array_equal(outs[0], outs[1])
    close(tof(outs[0]), tof(X) @ tof(W).T)


def test_asm_gemm_strided_rows_emulated():
    """ld > K on both operands and an output view with ld > N, offset columns."""
    rng = np.random.default_rng(7)
    M, N, K, ldx, ldw, ldc = 256, 256, 192, 320, 256, 512
    Xf = bf16(rng.standard_normal((M, ldx)))
    Wf = bf16(rng.standard_normal((N, ldw)))
    Cf = np.zeros((M, ldc), np.uint16)
    mem = emu.Memory()
    ax, aw, ac = mem.add(Xf), mem.add(Wf), mem.add(Cf)
    karg = host_args.pack(ax, aw, ac + 2 * 128, 0, 2 * ldx, 2 * ldw, 2 * ldc, 0, K, 1, 1)
    run_all("toa_gemm_tn_asm_plain", karg, 1, mem)
    C = tof(mem.bufs[2][1].view(np.uint16).reshape(M, ldc))
    close(C[:, 128:384], tof(Xf[:, :K]) @ tof(Wf[:, :K]).T)
    assert not C[:, :128].any() and not C[:, 384:].any()


def test_asm_gemm_swiglu_fwd_emulated():
    rng = np.random.default_rng(1)
    M, F, K = 256, 256, 128
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((2 * F, K)) * 0.1)
    mem = emu.Memory()
    ax, aw = mem.add(X), mem.add(W)
    ag, as_ = mem.add(np.zeros((M, 2 * F), np.uint16)), mem.add(np.zeros((M, F), np.uint16))
    karg = host_args.pack(ax, aw, ag, as_, 2 * K, 2 * K, 4 * F, 2 * F, K, M // 256, F // 128, fw_b=F * 2 * K,
                          fc_b=2 * F)
    run_all("toa_gemm_tn_asm_swiglu_fwd", karg, (M // 256) * (F // 128), mem)
    gu = tof(mem.bufs[2][1].view(np.uint16).reshape(M, 2 * F))
    s = tof(mem.bufs[3][1].view(np.uint16).reshape(M, F))
    ref = tof(X) @ tof(W).T
    close(gu, ref)
    g, u = tof(bf16(ref[:, :F])), tof(bf16(ref[:, F:]))
    close(s, g / (1 + np.exp(-g)) * u)


def test_asm_gemm_swiglu_bwd_emulated():
    rng = np.random.default_rng(2)
    M, F, K = 256, 512, 192
    D = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((F, K)) * 0.1)
    GU = bf16(rng.standard_normal((M, 2 * F)))
    mem = emu.Memory()
    ad, aw, adg, agu = mem.add(D), mem.add(W), mem.add(np.zeros((M, 2 * F), np.uint16)), mem.add(GU)
    karg = host_args.pack(ad, aw, adg, agu, 2 * K, 2 * K, 4 * F, 4 * F, K, M // 256, F // 256, fc_b=2 * F)
    run_all("toa_gemm_tn_asm_swiglu_bwd", karg, (M // 256) * (F // 256), mem)
    dgu = tof(mem.bufs[2][1].view(np.uint16).reshape(M, 2 * F))
    ds = tof(bf16(tof(D) @ tof(W).T))
    g, u = tof(GU[:, :F]), tof(GU[:, F:])
    sg = 1 / (1 + np.exp(-g))
    close(dgu[:, :F], ds * u * sg * (1 + g * (1 - sg)))
    close(dgu[:, F:], ds * g * sg)


@pytest.mark.parametrize("epi,grid", [("swiglu_fwd", 1), ("swiglu_fwd", 4), ("swiglu_bwd", 1), ("swiglu_bwd", 4)])
def test_asm_gemm_swiglu_persistent_emulated(epi, grid):
    """The persistent fused SwiGLU arms (SWIGLU_PERSIST_VARIANTS): `grid`
    workgroups walk the 6 tiles, the next tile's first k-tiles staged before
    the current tile's epilogue (whose gu loads / dgu stores then sit behind
    that DMA in the in-order vmcnt); every output equals the product kernel's
    bit for bit.  K = 320: an odd k-tile count (the stage parity fix-up)."""
    rng = np.random.default_rng(23)
    M, K = 512, 320
    F = 384 if epi == "swiglu_fwd" else 768
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((2 * F if epi == "swiglu_fwd" else F, K)) * 0.1)
    GU = bf16(rng.standard_normal((M, 2 * F)))
    tiles_n = F // 128 if epi == "swiglu_fwd" else F // 256
    outs = []
    for name, g in ((f"toa_gemm_tn_asm_{epi}", None), (f"toa_gemm_tn_asm_{epi}_p1", grid)):
        mem = emu.Memory()
        ax, aw = mem.add(X), mem.add(W)
        if epi == "swiglu_fwd":
            ac, as_ = mem.add(np.zeros((M, 2 * F), np.uint16)), mem.add(np.zeros((M, F), np.uint16))
            karg = host_args.pack(ax, aw, ac, as_, 2 * K, 2 * K, 4 * F, 2 * F, K, M // 256, tiles_n,
                                  fw_b=F * 2 * K, fc_b=2 * F, grid=g)
        else:
            ac, as_ = mem.add(np.zeros((M, 2 * F), np.uint16)), mem.add(GU)
            karg = host_args.pack(ax, aw, ac, as_, 2 * K, 2 * K, 4 * F, 4 * F, K, M // 256, tiles_n, fc_b=2 * F,
                                  grid=g)
        run_all(name, karg, (M // 256) * tiles_n if g is None else g, mem)
        outs.append([mem.bufs[i][1].copy() for i in (2, 3)])
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    if epi == "swiglu_bwd":
        ds = tof(bf16(tof(X) @ tof(W).T))
        dgu = tof(outs[1][0].view(np.uint16).reshape(M, 2 * F))
        close(dgu[:, F:], ds * tof(GU[:, :F]) / (1 + np.exp(-tof(GU[:, :F]))))


def _rope_ref(X, W, cs, B, S, Hq, Hkv):
    D = 128
    qkv = tof(X) @ tof(W).T                                   # [B S, H3 D]
    x = qkv.reshape(B, S, Hq + 2 * Hkv, D)
    c = cs[0].astype(np.float64)[None, :, None, :]             # [1, S, 1, 64]
    sn = cs[1].astype(np.float64)[None, :, None, :]
    rot = x.copy()
    r = slice(0, Hq + Hkv)
    x1, x2 = x[:, :, r, :64], x[:, :, r, 64:]
    rot[:, :, r, :64] = x1 * c - x2 * sn
    rot[:, :, r, 64:] = x2 * c + x1 * sn
    q = rot[:, :, :Hq].transpose(0, 2, 1, 3)
    k = rot[:, :, Hq:Hq + Hkv].transpose(0, 2, 1, 3)
    v = rot[:, :, Hq + Hkv:].transpose(0, 2, 1, 3)
    return np.concatenate([q.reshape(-1), k.reshape(-1), v.reshape(-1)])


@pytest.mark.parametrize("B,S,Hq,Hkv", [(2, 256, 2, 1), (1, 512, 4, 2)])
def test_asm_gemm_rope_epilogue_emulated(B, S, Hq, Hkv):
    """The fused-QKV projection with the RoPE + head-major epilogue: out =
    [q B Hq S 128 | k B Hkv S 128 | v B Hkv S 128], q / k rotated
    (rotate-half, cos / sin [S, 64] fp32 from the fp32 accumulators), v as is."""
    rng = np.random.default_rng(B * S + Hq)
    K = 192
    M, N = B * S, (Hq + 2 * Hkv) * 128
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((N, K)) * 0.2)
    ang = np.arange(S)[:, None] * (10000.0 ** (-np.arange(64) / 64))[None, :]
    cs = np.stack([np.cos(ang), np.sin(ang)]).astype(np.float32)   # [2, S, 64]
    mem = emu.Memory()
    ax, aw = mem.add(X), mem.add(W)
    ao = mem.add(np.zeros(M * N, np.uint16))
    acs = mem.add(cs)
    karg = host_args.pack(ax, aw, ao, acs, 2 * K, 2 * K, 0, 0, K, M // 256, N // 256, fw_b=S, fc_b=Hq | (Hkv << 16))
    run_all("toa_gemm_tn_asm_rope", karg, (M // 256) * (N // 256), mem)
    out = tof(mem.bufs[2][1].view(np.uint16))
    ref = _rope_ref(X, W, cs, B, S, Hq, Hkv)
    close(out, ref)


@pytest.mark.parametrize("tile_map", [0, 1, 2, 3, 4, 16, 17, 18, 19, 20])
def test_asm_gemm_tile_order_is_a_bijection(tile_map):
    """The XCD remap + group walk (row groups, or column groups with the walk
    bit) visits every (tm, tn) exactly once, for grids that are and are not
    multiples of 8 and of the group size (the formulas the prologue
    implements, host_args.tile_order)."""
    for tm_n, tn_n in ((1, 1), (3, 5), (96, 16), (7, 9), (96, 501)):
        seen = host_args.tile_order(tm_n, tn_n, tile_map)
        assert len(seen) == tm_n * tn_n
        assert set(seen) == {(i, j) for i in range(tm_n) for j in range(tn_n)}


@pytest.mark.parametrize("tile_map", [0, 18, 20])
def test_asm_gemm_tile_maps_emulated(tile_map):
    """Other tile orders (single row tiles; column groups of 4 and 16) write
    the default order's C bit for bit: each tile's arithmetic is the same,
    only which workgroup computes it changes."""
    rng = np.random.default_rng(17)
    M, N, K = 768, 1280, 128
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((N, K)))
    outs = []
    for tmap in (gemm_gen.MAP_DEFAULT, tile_map):
        mem = emu.Memory()
        ax, aw, ac = mem.add(X), mem.add(W), mem.add(np.zeros((M, N), np.uint16))
        karg = host_args.pack(ax, aw, ac, 0, 2 * K, 2 * K, 2 * N, 0, K, M // 256, N // 256, tile_map=tmap)
        run_all("toa_gemm_tn_asm_plain", karg, (M // 256) * (N // 256), mem)
        outs.append(mem.bufs[2][1].view(np.uint16).reshape(M, N).copy())
    assert np.array_equal(outs[0], outs[1])


def test_asm_gemm_persistent_refuses_zero_grid():
    """A persistent arm given grid 0 (it would walk its first tile forever)
    ends before any memory access."""
    name = next(f"toa_gemm_tn_asm_plain_{v}" for v, k in gemm_gen.PLAIN_VARIANTS if k.get("persist"))
    M, N, K = 256, 256, 128
    mem = emu.Memory()
    ax, aw = mem.add(np.ones((M, K), np.uint16)), mem.add(np.ones((N, K), np.uint16))
    ac = mem.add(np.full((M, N), 7, np.uint16))
    run_all(name, host_args.pack(ax, aw, ac, 0, 2 * K, 2 * K, 2 * N, 0, K, 1, 1, grid=0), 1, mem)
    assert (mem.bufs[2][1].view(np.uint16) == 7).all()


def test_asm_gemm_rejects_bad_tile_map():
    """A map word the host never packs (log2 group > 6, bits above the walk
    flag) ends every workgroup before any memory access: C untouched."""
    M, N, K = 256, 256, 128
    for bad in (7, 15, 32, 1 << 20):
        mem = emu.Memory()
        ax, aw = mem.add(np.ones((M, K), np.uint16)), mem.add(np.ones((N, K), np.uint16))
        ac = mem.add(np.full((M, N), 7, np.uint16))
        karg = host_args.pack(ax, aw, ac, 0, 2 * K, 2 * K, 2 * N, 0, K, 1, 1, tile_map=bad)
        run_all("toa_gemm_tn_asm_plain", karg, 1, mem)
        assert (mem.bufs[2][1].view(np.uint16) == 7).all()


def test_host_kernel_table_matches_generator():
    """Every kernel name csrc/hip/gemm_asm.hip resolves exists in the code
    object (a missing one fails the module load, i.e. every asm GEMM)."""
    import re

    src = open(os.path.join(os.path.dirname(HERE), "csrc", "hip", "gemm_asm.hip")).read()
    generated = set(re.findall(r"^(toa_\w+):", TEXT, re.M))
    wanted = re.findall(r'"(toa_(?:gemm_tn_asm|wgrad_nt_asm|attn_fwd_asm|attn_dkdv_asm)\w*)"', src)
    assert wanted and set(wanted) <= generated, set(wanted) - generated
    n = int(re.search(r"K_N = (\d+)", src).group(1))
    # + the weight gradient's round-4 arm + the attention forward and its arms + the dK/dV backward
    import attn_bwd_gen
    import attn_gen
    # + the round-4 SwiGLU epilogue arms (2) + the SwiGLU backward's diagnostic arms
    # 11: the six product epilogues (plain, swiglu_fwd, swiglu_bwd, rope, delta, resadd), probe, trace, timing,
    # timing2, wgrad
    assert n == len(wanted) == 11 + len(gemm_gen.PLAIN_VARIANTS) + 2 + len(attn_gen.VARIANTS) + 1 + \
        len(attn_bwd_gen.VARIANTS) + 2 + len(gemm_gen.SWIGLU_BWD_VARIANTS) + len(gemm_gen.SWIGLU_PERSIST_VARIANTS)
    flags = re.search(r"kVariantPersist\[kNumPlainVariants\] = \{([^}]*)\}", src).group(1)
    assert int(re.search(r"kNumPlainVariants = (\d+)", src).group(1)) == len(gemm_gen.PLAIN_VARIANTS)
    assert [f.strip() == "true" for f in flags.split(",")] == [bool(k.get("persist")) for _, k in gemm_gen.PLAIN_VARIANTS]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/clang"), reason="no ROCm LLVM")
def test_asm_gemm_assembles(tmp_path):
    s = tmp_path / "g.s"
    s.write_text(TEXT)
    o = tmp_path / "g.o"
    subprocess.run(["/opt/rocm/lib/llvm/bin/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                    "-mcpu=gfx950", "-c", str(s), "-o", str(o)], check=True)
    assert o.stat().st_size > 0


@pytest.mark.parametrize("B,S,H", [(2, 256, 4), (1, 512, 2)])
def test_asm_gemm_delta_epilogue_emulated(B, S, H):
    """The output projection's data gradient with the attention backward's
    delta fused: C = dY W^T as the plain kernel writes it (bit for bit), and
    ndelta[b, h, s] = -sum_d bf16(C)[t][128 h + d] O[t][128 h + d]."""
    rng = np.random.default_rng(B * S + H)
    K = 128
    M, N = B * S, H * 128
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((N, K)) * 0.3)
    O = bf16(rng.standard_normal((M, N)))
    outs = []
    for name in ("toa_gemm_tn_asm_plain", "toa_gemm_tn_asm_delta"):
        mem = emu.Memory()
        ax, aw, ac = mem.add(X), mem.add(W), mem.add(np.zeros((M, N), np.uint16))
        ao = mem.add(O)
        ad = mem.add(np.full(B * H * S, np.nan, np.float32))
        delta = name.endswith("delta")
        # (the plain kernel reads fc as its diagnostic stage-exit word: 0 there)
        karg = bytearray(host_args.pack(ax, aw, ac, ao, 2 * K, 2 * K, 2 * N, 0, K, M // 256, N // 256,
                                        fw_b=S if delta else 0, fc_b=H if delta else 0))
        if delta:
            karg[88:96] = int(ad).to_bytes(8, "little")
        run_all(name, bytes(karg), (M // 256) * (N // 256), mem)
        outs.append((mem.bufs[2][1].copy(), mem.bufs[4][1].view(np.float32).copy()))
    assert np.array_equal(outs[0][0], outs[1][0])
    C = tof(outs[1][0].view(np.uint16).reshape(M, N))
    ref = -(C * tof(O)).reshape(B, S, H, 128).sum(-1).transpose(0, 2, 1).reshape(-1)
    got = outs[1][1].astype(np.float64)
    assert np.abs(got - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-6, np.abs(got - ref).max()


def test_asm_gemm_resadd_epilogue_emulated():
    """C = X W^T + R with R laid out like C (the output projection's residual
    add in its epilogue): one bf16 rounding of the fp32 sum."""
    rng = np.random.default_rng(31)
    M, N, K = 512, 512, 192
    X = bf16(rng.standard_normal((M, K)))
    W = bf16(rng.standard_normal((N, K)) * 0.2)
    R = bf16(rng.standard_normal((M, N)))
    mem = emu.Memory()
    ax, aw, ac, ar_ = mem.add(X), mem.add(W), mem.add(np.zeros((M, N), np.uint16)), mem.add(R)
    karg = host_args.pack(ax, aw, ac, ar_, 2 * K, 2 * K, 2 * N, 0, K, M // 256, N // 256)
    run_all("toa_gemm_tn_asm_resadd", karg, (M // 256) * (N // 256), mem)
    C = tof(mem.bufs[2][1].view(np.uint16).reshape(M, N))
    ref = tof(X) @ tof(W).T + tof(R)
    close(C, ref)
    assert np.mean(np.abs(C - tof(bf16(ref))) <= np.abs(ref) * 2 ** -7) > 0.999
