"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference (MI355X)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lib():
    from tf_operator_amd.ops import _lib

    assert _lib.available(), _lib.load_error()
    return _lib


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("cols", [4096, 1024, 200, 8192])
@pytest.mark.parametrize("res", [False, True])
def test_rmsnorm_fwd_bwd(cols, res):
    _lib()
    from tf_operator_amd.ops.norm import _ref_norm, _ref_norm_bwd, add_rms_norm, rms_norm

    torch.manual_seed(0)
    rows = 777
    x = torch.randn(rows, cols, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(rows, cols, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(cols, device=DEV)).to(torch.bfloat16).requires_grad_()
    if res:
        h, y = add_rms_norm(x, r, w, 1e-5)
        href = (x.float() + r.float())
        assert rel(h, href) < 1e-2
    else:
        y = rms_norm(x, w, 1e-5)
        href = x.float()
    yref = href * torch.rsqrt(href.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    assert rel(y, yref) < 1e-2
    dy = torch.randn_like(y)
    if res:
        dh = torch.randn_like(y)
        torch.autograd.backward([h, y], [dh, dy])
    else:
        y.backward(dy)
    hr = href.detach().clone().requires_grad_()
    wr = w.detach().float().clone().requires_grad_()
    yr = hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    yr.backward(dy.float())
    dx_ref = hr.grad + (dh.float() if res else 0)
    assert rel(x.grad, dx_ref) < 2e-2
    assert rel(w.grad, wr.grad) < 2e-2


@pytest.mark.parametrize("cols", [2048, 4096, 6144, 8192])
def test_rmsnorm_row_and_wave_forms_agree(cols):
    """The one-row-per-workgroup RMSNorm kernels (default for bf16 rows of
    2048-8192 columns) against the one-row-per-wave ones
    (toa_norm_set_row(0)): same h and y (bit for bit: same per-element
    arithmetic), dx and dW to summation-order rounding."""
    L = _lib()
    from tf_operator_amd.ops.norm import add_rms_norm

    torch.manual_seed(cols)
    rows = 301
    x = torch.randn(rows, cols, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(rows, cols, device=DEV, dtype=torch.bfloat16)
    w0 = (1 + 0.1 * torch.randn(cols, device=DEV)).to(torch.bfloat16)
    dy, dh = torch.randn_like(x), torch.randn_like(x)
    outs = []
    try:
        for form in (1, 0):
            L.call("toa_norm_set_row", form)
            a, b = x.clone().requires_grad_(), r.clone().requires_grad_()
            w = w0.clone().requires_grad_()
            h, y = add_rms_norm(a, b, w, 1e-5)
            torch.autograd.backward([h, y], [dh, dy])
            outs.append((h.detach(), y.detach(), a.grad, w.grad))
        torch.cuda.synchronize()
    finally:
        L.call("toa_norm_set_row", -1)
    (h1, y1, dx1, dw1), (h0, y0, dx0, dw0) = outs
    assert torch.equal(h1, h0)
    assert rel(y1, y0) < 1e-2 and rel(dx1, dx0) < 1e-2 and rel(dw1, dw0) < 1e-3


@pytest.mark.parametrize("cols", [4096, 512, 1000, 8192])
def test_layernorm_fwd_bwd(cols):
    _lib()
    from tf_operator_amd.ops.norm import layer_norm

    torch.manual_seed(1)
    for dt in (torch.bfloat16, torch.float32):
        x = torch.randn(300, cols, device=DEV, dtype=dt, requires_grad=True)
        w = torch.randn(cols, device=DEV, dtype=dt, requires_grad=True)
        b = torch.randn(cols, device=DEV, dtype=dt, requires_grad=True)
        y = layer_norm(x, w, b, 1e-5)
        xr, wr, br = [t.detach().float().clone().requires_grad_() for t in (x, w, b)]
        yr = torch.nn.functional.layer_norm(xr, (cols,), wr, br, 1e-5)
        tol = 1e-2 if dt == torch.bfloat16 else 1e-5
        assert rel(y, yr) < tol
        dy = torch.randn_like(yr)
        y.backward(dy.to(dt))
        yr.backward(dy)
        assert rel(x.grad, xr.grad) < 2 * tol + 1e-5
        assert rel(w.grad, wr.grad) < 2 * tol + 1e-5
        assert rel(b.grad, br.grad) < 2 * tol + 1e-5


def test_rope_qkv_roundtrip():
    _lib()
    from tf_operator_amd.ops import llm

    torch.manual_seed(2)
    B, S, Hq, Hkv, D = 2, 64, 8, 2, 128
    cos, sin = llm.rope_tables(S, D, device=DEV)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    for rep in (Hq // Hkv, 1):
        q, k, v = llm.rope_qkv(qkv, cos, sin, B, S, Hq, Hkv, D, rep)
        qc = qkv.detach().cpu().requires_grad_()
        qr, kr, vr = llm.rope_qkv(qc, cos.cpu(), sin.cpu(), B, S, Hq, Hkv, D, rep)
        assert rel(q.cpu(), qr) < 1e-2 and rel(k.cpu(), kr) < 1e-2 and rel(v.cpu(), vr) < 1e-3
        gq, gk, gv = torch.randn_like(q), torch.randn_like(k), torch.randn_like(v)
        (g,) = torch.autograd.grad([q, k, v], [qkv], [gq, gk, gv])
        (gr,) = torch.autograd.grad([qr, kr, vr], [qc], [gq.cpu(), gk.cpu(), gv.cpu()])
        assert rel(g.cpu(), gr) < 1e-2


@pytest.mark.parametrize("F", [1024, 1000, 14336])
def test_swiglu(F):
    L = _lib()
    from tf_operator_amd.ops import llm

    torch.manual_seed(3)
    gu = torch.randn(333, 2 * F, device=DEV, dtype=torch.bfloat16)
    out = llm.swiglu(gu)
    ref = torch.nn.functional.silu(gu[:, :F].float()) * gu[:, F:].float()
    assert rel(out, ref) < 1e-2
    d = torch.randn(333, F, device=DEV, dtype=torch.bfloat16)
    dgu = llm.swiglu_bwd(d, gu)
    g = gu.float().requires_grad_()
    (torch.nn.functional.silu(g[:, :F]) * g[:, F:]).backward(d.float())
    assert rel(dgu, g.grad) < 1e-2
    # the default row-structured non-temporal kernels are bit-identical to the flat ones
    old = L.lib().toa_set_stream_variant(0)
    try:
        assert torch.equal(llm.swiglu(gu), out)
        assert torch.equal(llm.swiglu_bwd(d, gu), dgu)
    finally:
        L.lib().toa_set_stream_variant(old)
    assert old & 2, "row-structured SwiGLU is the default"


@pytest.mark.parametrize("V", [128256, 1000, 10])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_cross_entropy(V, dt):
    _lib()
    from tf_operator_amd.ops.llm import cross_entropy

    torch.manual_seed(4)
    rows = 65
    x = (3 * torch.randn(rows, V, device=DEV)).to(dt).requires_grad_()
    t = torch.randint(0, V, (rows,), device=DEV)
    t[5] = -100
    loss = cross_entropy(x, t)
    xr = x.detach().float().requires_grad_()
    lr = torch.nn.functional.cross_entropy(xr, t, ignore_index=-100)
    assert abs(float(loss) - float(lr)) < 1e-3 * max(1, abs(float(lr)))
    loss.backward()
    lr.backward()
    assert rel(x.grad, xr.grad) < 1e-2


def test_adamw_flat_matches_reference():
    _lib()
    from tf_operator_amd.ops.optim import adamw_reference, grad_norm_sq
    from tf_operator_amd.ops import _lib as L

    torch.manual_seed(5)
    n = 1 << 20
    master = torch.randn(n, device=DEV)
    param = master.to(torch.bfloat16)
    grad = torch.randn(n, device=DEV).to(torch.bfloat16)
    m = torch.randn(n, device=DEV).abs() * 0.01
    v = torch.rand(n, device=DEV) * 0.01
    ref = [t.clone() for t in (master, m, v)]
    nsq = grad_norm_sq(grad)
    assert abs(float(nsq) - float(grad.float().pow(2).sum())) < 1e-3 * float(nsq)
    L.call("toa_adamw_flat", L.ptr(master), L.ptr(param), L.ptr(grad), 1, L.ptr(m), L.ptr(v), n, 1e-3, 0.9,
           0.95, 1e-8, 0.1, 3, 0.5, L.ptr(nsq), 1.0, L.stream(master))
    adamw_reference(ref[0], grad, ref[1], ref[2], lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1,
                    step=3, grad_scale=0.5, norm_sq=nsq, max_norm=1.0)
    torch.cuda.synchronize()
    assert rel(master, ref[0]) < 1e-6
    assert rel(m, ref[1]) < 1e-6 and rel(v, ref[2]) < 1e-6
    assert rel(param, ref[0]) < 1e-2


def test_llama_tiny_gpu_matches_cpu_reference():
    _lib()
    from tf_operator_amd.models.llama import PRESETS, Llama

    torch.manual_seed(6)
    cfg = PRESETS["llama-tiny"]
    m_gpu = Llama(cfg, device=DEV)
    m_gpu.init_weights(0)
    m_cpu = Llama(cfg, device="cpu")
    m_cpu.load_state_dict({k: v.cpu() for k, v in m_gpu.state_dict().items()})
    tok = torch.randint(0, cfg.vocab_size, (2, 64))
    tgt = torch.randint(0, cfg.vocab_size, (2, 64))
    lg = m_gpu(tok.to(DEV), tgt.to(DEV))
    lc = m_cpu(tok, tgt)
    assert abs(float(lg) - float(lc)) < 2e-2
    lg.backward()
    lc.backward()
    for (n, pg), (_, pc) in zip(m_gpu.named_parameters(), m_cpu.named_parameters()):
        assert rel(pg.grad.cpu(), pc.grad) < 5e-2, n


def test_trainer_tiny_loss_decreases():
    _lib()
    from tf_operator_amd.models.llama import PRESETS
    from tf_operator_amd.train.llm import LlamaTrainer

    tr = LlamaTrainer(PRESETS["llama-tiny"], torch.device(DEV), micro_batch=2, seq_len=128, lr=1e-3)
    b = tr.synthetic_batch()
    losses = [float(tr.step([b])) for _ in range(5)]
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
def test_embedding_backward_deterministic(gdt):
    """csrc/hip/llm.hip embed_bwd_kernel vs an fp32 index_add reference, with
    heavy id repetition; two runs are bit-identical."""
    _lib()
    from tf_operator_amd.ops.embedding import _scatter_rows

    torch.manual_seed(3)
    V, D, n = 50, 264, 3000
    idx = torch.randint(0, V, (n,), device=DEV)
    idx[:700] = 7  # one long run
    dy = torch.randn(n, D, device=DEV).to(torch.bfloat16)
    base = torch.randn(V, D, device=DEV).to(gdt)
    ref = base.float().index_add(0, idx, dy.float())
    outs = []
    for _ in range(2):
        g = base.clone()
        _scatter_rows(g, idx, dy)
        outs.append(g)
    assert torch.equal(outs[0], outs[1])
    tol = 2e-2 if gdt == torch.bfloat16 else 1e-4
    assert (outs[0].float() - ref).abs().max() <= tol * ref.abs().max()


@pytest.mark.parametrize("N,K,T,beta,split", [(256, 256, 1024, 0, 1), (512, 768, 2048, 1, 2), (768, 512, 4096, 1, 4),
                                             (1024, 256, 3072, 1, 3)])
def test_wgrad_nt_kernel(N, K, T, beta, split):
    """csrc/hip/wgrad.hip: g (+)= dy^T x against an fp32 reference, incl. a
    strided dy view and the split-K workspace reduction."""
    _lib()
    from tf_operator_amd.ops import gemm

    torch.manual_seed(N + K + T)
    big = (torch.rand(T, N + 256, device=DEV) * 2 - 1).to(torch.bfloat16)
    dy = big[:, 128:128 + N]  # row stride N + 256
    x = (torch.rand(T, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    g = (torch.rand(N, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    ref = dy.float().t() @ x.float() + (g.float() if beta else 0)
    assert gemm.wgrad_hip_ok(g, dy, x)
    gemm.wgrad_hip_(g, dy, x, beta=float(beta), split=split)
    err = (g.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)


@pytest.mark.parametrize("N,K,T,beta,want_split", [(4352, 4096, 4096, 1, 4), (5376, 4096, 3072, 0, 3),
                                                   (1024, 1024, 2048, 1, 4), (4096, 4096, 2048, 1, 1)])
def test_wgrad_nt_auto_plan(N, K, T, beta, want_split):
    """Auto plan (split=None): whole-K tiles for the full waves of 256 CUs,
    only the tail tiles cut into K-pieces reduced from a tile-major
    workspace; bit-identical to a uniform-split run's math within bf16."""
    _lib()
    from tf_operator_amd.ops import _lib as L
    from tf_operator_amd.ops import gemm

    assert L.call_ret("toa_wgrad_split", N, K, T) == want_split
    torch.manual_seed(N + K + T)
    dy = (torch.rand(T, N, device=DEV) * 2 - 1).to(torch.bfloat16)
    x = (torch.rand(T, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    g0 = (torch.rand(N, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    ref = dy.float().t() @ x.float() + (g0.float() if beta else 0)
    g = g0.clone()
    gemm.wgrad_hip_(g, dy, x, beta=float(beta))
    err = (g.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)
    g2 = g0.clone()
    gemm.wgrad_hip_(g2, dy, x, beta=float(beta))
    assert torch.equal(g, g2)  # deterministic


@pytest.mark.parametrize("N,K,T,beta,split", [(256, 256, 1024, 0, 1), (512, 768, 2048, 1, 1),
                                              (4352, 4096, 4096, 1, None), (5376, 4096, 3072, 0, None),
                                              (1024, 1024, 2048, 1, 2), (28672, 4096, 1024, 0, None)])
def test_wgrad_split_tail_and_strided(N, K, T, beta, split):
    """The weight-gradient kernel against an fp32 reference on the Llama
    shapes, incl. the split-K tail pieces and a strided dy view."""
    _lib()
    from tf_operator_amd.ops import gemm

    torch.manual_seed(N + K + T + 4)
    big = (torch.rand(T, N + 256, device=DEV) * 2 - 1).to(torch.bfloat16)
    dy = big[:, 128:128 + N]
    x = (torch.rand(T, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    g0 = (torch.rand(N, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    ref = dy.float().t() @ x.float() + (g0.float() if beta else 0)
    g = g0.clone()
    gemm.wgrad_hip_(g, dy, x, beta=float(beta), split=split)
    g2 = g0.clone()
    gemm.wgrad_hip_(g2, dy, x, beta=float(beta), split=split)
    torch.cuda.synchronize()
    err = (g.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)
    assert torch.equal(g, g2)  # deterministic


@pytest.mark.parametrize("N,K,T,beta,split", [(256, 256, 256, 0, 1), (512, 768, 2048, 1, 1),
                                              (4352, 4096, 4096, 1, None), (5376, 4096, 3072, 0, None),
                                              (1024, 1024, 2048, 1, 2), (1024, 512, 4096, 0, 4),
                                              (28672, 4096, 1024, 0, None)])
def test_wgrad_asm_matches_fp32_and_hip(N, K, T, beta, split):
    """The assembly NT weight-gradient kernel (csrc/asm/wgrad_gen.py) vs an
    fp32 reference and vs the HIP kernel: whole-K tiles with beta 0 / 1, the
    auto plan's split tail, explicit splits, a strided dy view; two launches
    bit for bit (fixed k order, fixed-order reduce)."""
    L = _lib()
    from tf_operator_amd.ops import gemm

    torch.manual_seed(N + K + T)
    big = (torch.rand(T, N + 256, device=DEV) * 2 - 1).to(torch.bfloat16)
    dy = big[:, 128:128 + N]
    x = (torch.rand(T, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    g0 = (torch.rand(N, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    ref = dy.float().t() @ x.float() + (g0.float() if beta else 0)
    sp = 0 if split is None else int(split)
    nbytes = int(L.call_ret("toa_wgrad_workspace", N, K, T, sp))
    ws = torch.empty(max(nbytes, 16) // 4, device=DEV, dtype=torch.float32)
    outs = []
    for _ in range(2):
        g = g0.clone()
        L.call("toa_wgrad_asm", L.ptr(dy), dy.stride(0), L.ptr(x), x.stride(0), L.ptr(g), K, L.ptr(ws), N, K, T, sp,
               int(beta), L.stream(g))
        outs.append(g)
    torch.cuda.synchronize()
    err = (outs[0].float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)
    assert torch.equal(outs[0], outs[1])
    gh = g0.clone()
    gemm.wgrad_hip_(gh, dy, x, beta=float(beta), split=split)
    torch.cuda.synchronize()
    assert rel(outs[0], gh) < 1e-2


def test_wgrad_routing_matches_hipblaslt():
    """accumulate_mm sends a Linear weight gradient through the HIP kernel;
    the result matches hipBLASLt's addmm_ to bf16 rounding."""
    _lib()
    from tf_operator_amd.ops import gemm
    from tf_operator_amd.ops.grad import accumulate_mm

    torch.manual_seed(5)
    w = torch.nn.Parameter(torch.zeros(512, 256, device=DEV, dtype=torch.bfloat16))
    w.main_grad = torch.zeros_like(w)
    dy = torch.randn(2048, 512, device=DEV).to(torch.bfloat16)
    x = torch.randn(2048, 256, device=DEV).to(torch.bfloat16)
    assert gemm.wgrad_hip_ok(w.main_grad, dy, x)
    accumulate_mm(w, dy.t(), x)
    ref = torch.zeros_like(w).addmm_(dy.t(), x)
    assert (w.main_grad.float() - ref.float()).abs().max() <= 2e-2 * ref.float().abs().max()


@pytest.mark.parametrize("R,C,pad", [(64, 64, 0), (128, 320, 0), (6144, 4096, 0), (192, 256, 64), (256, 384, 64),
                                     (4096, 14336, 0)])
def test_transpose_bf16_kernel(R, C, pad):
    """csrc/hip/transpose.hip is an exact transpose, incl. strided source /
    destination rows."""
    _lib()
    from tf_operator_amd.ops.wt import transpose_into

    torch.manual_seed(R + C)
    big = torch.randn(R, C + pad, device=DEV).to(torch.bfloat16)
    src = big[:, :C]
    dbig = torch.zeros(C, R + pad, device=DEV, dtype=torch.bfloat16)
    dst = dbig[:, :R]
    transpose_into(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(dst, src.t())
    if pad:
        assert not dbig[:, R:].any()


def test_dgrad_on_transposed_weight_matches_nn():
    """linear_dgrad routes through param._toa_wt (dy (W^T)^T, the forward's
    GEMM form) and matches hipBLASLt's dy @ W to bf16 rounding."""
    _lib()
    from tf_operator_amd.ops import gemm
    from tf_operator_amd.ops.wt import transpose_into

    torch.manual_seed(9)
    w = torch.nn.Parameter(torch.randn(768, 512, device=DEV).to(torch.bfloat16))
    dy = torch.randn(2048, 768, device=DEV).to(torch.bfloat16)
    ref = dy.float() @ w.float()
    w._toa_wt = transpose_into(torch.empty(512, 768, device=DEV, dtype=torch.bfloat16), w.data)
    got = gemm.linear_dgrad(dy, w)
    assert (got.float() - ref).abs().max() <= 1e-2 * ref.abs().max()


def test_trainer_transposed_weights_refresh():
    """With the W^T copies (TOA_DGRAD_WT default) every copy equals the
    current weights after each optimizer step, and the training trajectory
    matches the trainer without them to bf16 GEMM rounding."""
    _lib()
    from tf_operator_amd.models.llama import PRESETS
    from tf_operator_amd.train.llm import LlamaTrainer

    runs = []
    for use_wt in (False, True):
        for overlap in ((False, True) if use_wt else (False,)):
            tr = LlamaTrainer(PRESETS["llama-tiny"], torch.device(DEV), micro_batch=2, seq_len=128, lr=1e-3,
                              bucket_mb=0.25, overlap_optimizer=overlap)
            if not use_wt:
                tr.wt.detach()
                tr.wt = None
                tr.opt.post_update = None
            b = tr.synthetic_batch()
            losses = [float(tr.step([b])) for _ in range(4)]
            tr.opt.wait_all()
            torch.cuda.synchronize()
            if use_wt:
                assert len(tr.wt.items) == 4 * 2 + 1
                for _, _, p, view in tr.wt.items:
                    assert torch.equal(view, p.data.t()), "stale W^T"
            runs.append(losses)
    for losses in runs[1:]:
        assert max(abs(a - b) for a, b in zip(losses, runs[0])) < 2e-2, runs


def test_trainer_overlapped_optimizer_matches_serial():
    """FlatAdamW overlap mode (per-bucket update on a side stream, fused grad
    zeroing, forward pre-hook waits) is bit-identical to the serial step."""
    _lib()
    from tf_operator_amd.models.llama import PRESETS
    from tf_operator_amd.train.llm import LlamaTrainer, trainer_state

    out = []
    for overlap in (False, True):
        tr = LlamaTrainer(PRESETS["llama-tiny"], torch.device(DEV), micro_batch=2, seq_len=128, lr=1e-3,
                          bucket_mb=0.25, overlap_optimizer=overlap)
        assert tr.opt.overlap == overlap
        if overlap:
            assert len(tr.bucketer.buckets) > 2
        b = tr.synthetic_batch()
        losses = [float(tr.step([b, b])) for _ in range(4)]
        st = trainer_state(tr)
        out.append((losses, st["flat"]["master"].clone(), tr.flat.param.detach().clone()))
    assert out[0][0] == out[1][0]
    assert torch.equal(out[0][1], out[1][1])
    assert torch.equal(out[0][2], out[1][2])


def _attn_ref(q, k, v, scale):
    rep = q.shape[1] // k.shape[1]
    kf = k.float().repeat_interleave(rep, 1)
    vf = v.float().repeat_interleave(rep, 1)
    s = torch.matmul(q.float(), kf.transpose(-1, -2)) * scale
    S = q.shape[2]
    mask = torch.triu(torch.ones(S, S, dtype=torch.bool, device=q.device), 1)
    s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, -1)
    return torch.matmul(torch.softmax(s, -1), vf), lse


@pytest.mark.parametrize("B,H,Hk,S,D,spike", [(1, 2, 2, 128, 128, False), (2, 4, 2, 384, 128, False),
                                               (1, 8, 2, 1024, 128, False), (1, 2, 1, 1024, 128, True),
                                               # ragged S: tails of the 64-key tiles / 256-row and 128-key blocks
                                               (1, 2, 1, 1, 128, False), (2, 4, 2, 100, 128, False),
                                               (1, 4, 4, 333, 128, False), (1, 2, 2, 1000, 128, True),
                                               # head_dim 64 (Llama-3.2-1B / llama-tiny)
                                               (1, 2, 2, 128, 64, False), (2, 4, 2, 384, 64, False),
                                               (1, 8, 2, 1024, 64, True), (2, 4, 1, 77, 64, False),
                                               (1, 4, 2, 530, 64, False)])
def test_flash_attention_fwd_bwd(B, H, Hk, S, D, spike):
    L = _lib()
    from tf_operator_amd.ops import llm

    torch.manual_seed(7)
    scale = 1.0 / math.sqrt(D)
    q = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    if spike:  # force the deferred-rescale branch (guide rule 26): late keys dominate
        with torch.no_grad():
            k[:, :, 600:] *= 6.0
            k[:, :, 900] = 4.0 * q[0, 0, 950].to(k.dtype)
    o = llm._FlashAttn.apply(q, k, v, scale)
    qr, kr, vr = [t.detach().float().requires_grad_() for t in (q, k, v)]
    orf, lse_ref = _attn_ref(qr, kr, vr, scale)
    assert rel(o, orf) < 2e-2, rel(o, orf)
    # lse from a direct forward call
    o2 = torch.empty_like(q)
    lse = torch.empty(B, H, S, device=DEV, dtype=torch.float32)
    L.call("toa_attn_fwd", L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(o2), L.ptr(lse), B, H, Hk, S, D, 1, scale,
           L.stream(q))
    torch.cuda.synchronize()
    assert float((lse - lse_ref).abs().max()) < 2e-2
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    # relative error with a floor: at S = 1 the exact dK is 0 (one key, p = 1)
    # and the kernel's is bf16 rounding noise of delta = rowsum(dO * O)
    for got, ref in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        err = float((got.float() - ref).norm())
        assert err <= 3e-2 * max(float(ref.norm()), 1e-2 * ref.numel() ** 0.5), err


def test_flash_attention_bench_shape():
    """The flagship shape (Llama-3-8B, micro-batch 6: B=6, H=32, Hkv=8,
    S=4096, D=128, O/dO in [B,S,H,D]) through the model's entry point; the
    fp32 reference is computed for sampled (batch, kv-group) slices (the
    first and last of each), which checks the XCD-aware block mapping at
    the corners of the grid."""
    _lib()
    from tf_operator_amd.ops import llm

    torch.manual_seed(11)
    B, H, Hk, S, D = 6, 32, 8, 4096, 128
    rep = H // Hk
    scale = 1.0 / math.sqrt(D)
    q = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = llm.causal_attention(q, k, v, out_layout="bshd")  # [B, S, H, D]
    do = torch.randn_like(o)
    o.backward(do)
    torch.cuda.synchronize()
    for b, g in ((0, 0), (B - 1, Hk - 1), (2, 3)):
        hs = slice(g * rep, (g + 1) * rep)
        qr = q[b:b + 1, hs].detach().float().requires_grad_()
        kr = k[b:b + 1, g:g + 1].detach().float().requires_grad_()
        vr = v[b:b + 1, g:g + 1].detach().float().requires_grad_()
        orf, _ = _attn_ref(qr, kr, vr, scale)
        got = o[b:b + 1, :, hs].transpose(1, 2)
        assert rel(got, orf) < 2e-2, (b, g, rel(got, orf))
        orf.backward(do[b:b + 1, :, hs].transpose(1, 2).float())
        assert rel(q.grad[b:b + 1, hs], qr.grad) < 3e-2, (b, g)
        assert rel(k.grad[b:b + 1, g:g + 1], kr.grad) < 3e-2, (b, g)
        assert rel(v.grad[b:b + 1, g:g + 1], vr.grad) < 3e-2, (b, g)
        del qr, kr, vr, orf


@pytest.mark.parametrize("B,H,Hk,S,D,bshd", [(1, 2, 2, 256, 128, False), (2, 4, 2, 512, 128, True),
                                              (1, 8, 2, 1024, 128, True), (1, 4, 1, 768, 128, False),
                                              (2, 4, 2, 512, 64, False), (1, 2, 1, 1024, 64, True),
                                              # long sequence: 256 x 257 / 2 dS blocks per head
                                              (1, 4, 2, 8192, 128, True)])
def test_flash_attention_bwd_ds_form(B, H, Hk, S, D, bshd):
    """The dS-through-HBM backward (delta pass, dK/dV storing the lower-
    triangular dS blocks, dQ as a GEMM over them) vs the fp32 reference and
    vs the split form (dK/dV on the assembly kernel at D = 128, the HIP one at 64)."""
    L = _lib()
    torch.manual_seed(5)
    scale = 1.0 / math.sqrt(D)
    q = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    o = torch.empty(B, S, H, D, device=DEV, dtype=torch.bfloat16) if bshd else torch.empty_like(q)
    lse = torch.empty(B, H, S, device=DEV, dtype=torch.float32)
    flags = 1 | (2 if bshd else 0)
    P = L.ptr
    L.call("toa_attn_fwd", P(q), P(k), P(v), P(o), P(lse), B, H, Hk, S, D, flags, scale, L.stream(q))
    do = torch.randn_like(o)
    grads = {}
    try:
        for form in (0, 1):
            L.call("toa_attn_set_bwd_variant", form)
            nws = L.call_ret("toa_attn_bwd_ws_bytes", B, H, S, D)
            assert (nws > 0) == (form == 1)
            ws = torch.full((nws,), 0xFF, device=DEV, dtype=torch.uint8) if nws else None  # NaN-poisoned
            delta = torch.empty(B, H, S, device=DEV, dtype=torch.float32)
            dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
            L.call("toa_attn_bwd", P(q), P(k), P(v), P(o), P(do), P(lse), P(delta), P(ws), P(dq), P(dk), P(dv),
                   B, H, Hk, S, D, flags, scale, L.stream(q))
            torch.cuda.synchronize()
            grads[form] = (dq, dk, dv, delta)
    finally:
        L.call("toa_attn_set_bwd_variant", -1)
    (dq0, dk0, dv0, de0), (dq1, dk1, dv1, de1) = grads[0], grads[1]
    assert torch.isfinite(dq1.float()).all()
    assert rel(-de1, de0) < 1e-5  # the dS form's delta pass leaves -delta (the dP accumulators' start)
    assert rel(dk1, dk0) < 1e-2 and rel(dv1, dv0) < 1e-2
    assert rel(dq1, dq0) < 1e-2, rel(dq1, dq0)
    qr, kr, vr = [t.float().requires_grad_() for t in (q, k, v)]
    orf, _ = _attn_ref(qr, kr, vr, scale)
    orf.backward((do.transpose(1, 2) if bshd else do).float())
    for got, ref in ((dq1, qr.grad), (dk1, kr.grad), (dv1, vr.grad)):
        assert rel(got, ref) < 3e-2, rel(got, ref)


def test_attention_bwd_timing_instrumentation():
    """toa_attn_set_bwd_timing: the dS-form dK/dV kernel's s_memtime
    instrumentation (scripts/attn_bwd_ab.py --timing) runs, writes one
    {issue, wait, steps, 0} record per wave, and leaves the gradients
    bit-identical to the uninstrumented kernel."""
    L = _lib()
    torch.manual_seed(3)
    B, H, Hk, S, D = 1, 4, 2, 512, 128
    scale = 1.0 / math.sqrt(D)
    q = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    o = torch.empty(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, S, device=DEV, dtype=torch.float32)
    P = L.ptr
    L.call("toa_attn_fwd", P(q), P(k), P(v), P(o), P(lse), B, H, Hk, S, D, 3, scale, L.stream(q))
    do = torch.randn_like(o)
    nws = L.call_ret("toa_attn_bwd_ws_bytes", B, H, S, D)
    assert nws > 0
    nblk = (S // 128) * B * Hk
    ts = torch.zeros(nblk * 8 * 4, device=DEV, dtype=torch.int64)
    outs = []
    L.call("toa_attn_set_dkdv_variant", 0)   # the instrumented kernel is the HIP one: compare like with like
    for timed in (False, True):
        ws = torch.empty(nws, device=DEV, dtype=torch.uint8)
        delta = torch.empty(B, H, S, device=DEV, dtype=torch.float32)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        L.call("toa_attn_set_bwd_timing", P(ts) if timed else None)
        try:
            L.call("toa_attn_bwd", P(q), P(k), P(v), P(o), P(do), P(lse), P(delta), P(ws), P(dq), P(dk), P(dv),
                   B, H, Hk, S, D, 3, scale, L.stream(q))
            torch.cuda.synchronize()
        finally:
            L.call("toa_attn_set_bwd_timing", None)
        outs.append((dq, dk, dv))
    L.call("toa_attn_set_dkdv_variant", -1)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    t = ts.view(nblk, 8, 4).cpu()
    assert (t[..., 2] > 0).all()  # every wave records its step count
    assert (t[..., 0] > 0).all() and (t[..., 3] == 0).all()


@pytest.mark.parametrize("B,H,Hk,S,D,bshd", [(1, 4, 2, 512, 128, True), (2, 8, 2, 1024, 128, False),
                                              (1, 4, 1, 768, 64, True)])
def test_flash_attention_fwd_forms_identical(B, H, Hk, S, D, bshd):
    """The LDS-DMA-staged forward (default at S % 256 == 0) and the
    register-staged one run the same arithmetic: O and lse bit-identical."""
    L = _lib()
    torch.manual_seed(9)
    q = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    outs = []
    try:
        for form in (0, 1):
            L.call("toa_attn_set_fwd_variant", form)
            o = torch.empty(B, S, H, D, device=DEV, dtype=torch.bfloat16) if bshd else torch.empty_like(q)
            lse = torch.empty(B, H, S, device=DEV, dtype=torch.float32)
            L.call("toa_attn_fwd", L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(o), L.ptr(lse), B, H, Hk, S, D,
                   1 | (2 if bshd else 0), 1.0 / math.sqrt(D), L.stream(q))
            outs.append((o, lse))
        torch.cuda.synchronize()
    finally:
        L.call("toa_attn_set_fwd_variant", -1)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("B,H,Hk,S,bshd,spike", [(1, 2, 1, 256, False, False), (2, 4, 2, 512, True, False),
                                                   (1, 16, 8, 1024, True, False), (1, 4, 1, 768, False, True),
                                                   (2, 8, 2, 2048, True, True), (6, 32, 8, 4096, True, False)])
def test_attn_fwd_asm(B, H, Hk, S, bshd, spike):
    """The assembly forward (csrc/asm/attn_gen.py, forward variant 2) against
    the HIP LDS-DMA kernel (variant 1) and fp32: O to bf16 rounding, lse to
    the bf16 P the row sums are taken from.  `spike`: late keys dominate, so
    the deferred rescale runs (guide rule 26); B Hk % 8 == 0 takes the
    XCD-grouped block order."""
    L = _lib()
    torch.manual_seed(21)
    D = 128
    scale = 1.0 / math.sqrt(D)
    q = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    if spike:
        k[:, :, S // 2:] *= 6.0
        k[:, :, S - 37] = 4.0 * q[0, 0, S - 20]
    outs = {}
    try:
        for form in (1, 2):
            L.call("toa_attn_set_fwd_variant", form)
            o = torch.full((B, S, H, D) if bshd else (B, H, S, D), float("nan"), device=DEV, dtype=torch.bfloat16)
            lse = torch.full((B, H, S), float("nan"), device=DEV, dtype=torch.float32)
            L.call("toa_attn_fwd", L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(o), L.ptr(lse), B, H, Hk, S, D,
                   1 | (2 if bshd else 0), scale, L.stream(q))
            torch.cuda.synchronize()
            outs[form] = ((o.transpose(1, 2) if bshd else o).float(), lse)
    finally:
        L.call("toa_attn_set_fwd_variant", -1)
    (o1, l1), (o2, l2) = outs[1], outs[2]
    assert torch.isfinite(o2).all() and torch.isfinite(l2).all()
    assert rel(o2, o1) < 1e-2, rel(o2, o1)
    assert float((l2 - l1).abs().max()) < 5e-3 * max(1.0, float(l1.abs().max()))
    if B * H * S <= 32768:
        orf, lse_ref = _attn_ref(q.float(), k.float(), v.float(), scale)
        assert rel(o2, orf) < 2e-2, rel(o2, orf)
        assert float((l2 - lse_ref).abs().max()) < 2e-2


@pytest.mark.parametrize("B,H,Hk,S,D", [(2, 8, 2, 512, 128), (1, 4, 1, 1024, 64), (1, 4, 2, 300, 128)])
def test_rope_attention_matches_two_nodes(B, H, Hk, S, D):
    """rope_attention (one autograd node; the backward writes d(qkv) from
    the attention kernels' epilogues where the dS form runs, S % 256 == 0,
    else attention backward + RoPE backward) against rope_qkv +
    causal_attention: same O, d(qkv) equal up to where bf16 rounding happens."""
    _lib()
    from tf_operator_amd.ops import llm

    torch.manual_seed(3)
    cos, sin = llm.rope_tables(S, D, device=DEV)
    qkv = torch.randn(B * S, (H + 2 * Hk) * D, device=DEV, dtype=torch.bfloat16)
    a = qkv.clone().requires_grad_()
    b = qkv.clone().requires_grad_()
    o1 = llm.rope_attention(a, cos, sin, B, S, H, Hk, D)
    q, k, v = llm.rope_qkv(b, cos, sin, B, S, H, Hk, D, 1)
    o2 = llm.causal_attention(q, k, v, out_layout="bshd")
    assert torch.equal(o1, o2)
    do = torch.randn_like(o1)
    o1.backward(do)
    o2.backward(do)
    torch.cuda.synchronize()
    assert rel(a.grad, b.grad) < 1e-2, rel(a.grad, b.grad)
    # per part (q / k / v) too: a wrong column block would hide in the total
    for lo, hi in ((0, H * D), (H * D, (H + Hk) * D), ((H + Hk) * D, (H + 2 * Hk) * D)):
        assert rel(a.grad[:, lo:hi], b.grad[:, lo:hi]) < 1e-2, (lo, hi)


def test_attention_gpu_has_no_library_fallback():
    """A GPU tensor the HIP kernel cannot take raises instead of silently
    running a library (SDPA / aotriton) kernel."""
    _lib()
    from tf_operator_amd.ops import llm

    q = torch.randn(1, 2, 64, 96, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="head_dim"):
        llm.causal_attention(q, q, q)
    with pytest.raises(RuntimeError, match="bf16"):
        llm.causal_attention(q.float()[..., :64], q.float()[..., :64], q.float()[..., :64])


def test_flash_attention_in_llama_layer():
    """A D=128 Llama block through the packed-GQA HIP attention path vs CPU fp32."""
    _lib()
    from tf_operator_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(8)
    cfg = LlamaConfig(vocab_size=256, hidden=512, layers=1, heads=4, kv_heads=2, ffn=1024, max_seq=256)
    m_gpu = Llama(cfg, device=DEV)
    m_gpu.init_weights(0)
    m_cpu = Llama(cfg, device="cpu")
    m_cpu.load_state_dict({k: v.cpu() for k, v in m_gpu.state_dict().items()})
    tok = torch.randint(0, cfg.vocab_size, (2, 256))
    tgt = torch.randint(0, cfg.vocab_size, (2, 256))
    lg = m_gpu(tok.to(DEV), tgt.to(DEV))
    lc = m_cpu(tok, tgt)
    assert abs(float(lg) - float(lc)) < 2e-2
    lg.backward()
    lc.backward()
    for (n, pg), (_, pc) in zip(m_gpu.named_parameters(), m_cpu.named_parameters()):
        assert rel(pg.grad.cpu(), pc.grad) < 5e-2, n


@pytest.mark.parametrize("M,K,N,act,keep", [(100, 784, 128, "relu", 1.0), (64, 100, 10, "none", 1.0),
                                            (256, 512, 300, "relu", 0.9), (33, 64, 96, "gelu", 0.75)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_dense_bias_act_dropout(M, K, N, act, keep, dt):
    """Fused MFMA dense (csrc/hip/mlp.hip) vs the fp32 CPU reference, same
    counter-hash dropout mask (exact mask parity)."""
    _lib()
    from tf_operator_amd.ops.mlp import linear_bias_act

    torch.manual_seed(0)
    # the GEMM runs on bf16 MFMA (fp32 accumulate) for fp32 inputs too: give
    # both paths bf16-representable operands so ReLU masks agree exactly
    x = torch.randn(M, K).to(torch.bfloat16).to(dt)
    w = (torch.randn(N, K) / K ** 0.5).to(torch.bfloat16).to(dt)
    b = (torch.randn(N) * 0.1).to(dt)
    dy = torch.randn(M, N, dtype=dt)
    outs = []
    for dev in ("cpu", DEV):
        xx = x.detach().to(dev).requires_grad_()
        ww = w.detach().to(dev).requires_grad_()
        bb = b.detach().to(dev).requires_grad_()
        y = linear_bias_act(xx, ww, bb, act, keep, seed=1234)
        y.backward(dy.to(dev))
        g = [t.grad for t in (xx, ww, bb)]
        outs.append([y.detach().cpu()] + [t.detach().cpu() for t in g])
    tol = 2e-2 if dt == torch.bfloat16 else 5e-3
    for a, r, name in zip(outs[1], outs[0], ["y", "dx", "dw", "db"]):
        assert rel(a, r) < tol, (name, rel(a, r))


@pytest.mark.parametrize("C", [10, 1000])
def test_accuracy_kernel(C):
    _lib()
    from tf_operator_amd.ops.mlp import accuracy

    torch.manual_seed(1)
    lg = torch.randn(517, C)
    lab = torch.randint(0, C, (517,))
    lab[:200] = lg[:200].argmax(-1)
    ref = float((lg.argmax(-1) == lab).float().mean())
    got = float(accuracy(lg.to(DEV, torch.bfloat16), lab.to(DEV)))
    ref_bf = float((lg.to(torch.bfloat16).float().argmax(-1) == lab).float().mean())
    assert abs(got - ref_bf) < 1e-6 and abs(ref_bf - ref) < 0.05


@pytest.mark.parametrize("M,K,N", [(256, 512, 384), (1000, 768, 1024)])
def test_tuned_gemm_forms(M, K, N):
    """ops/gemm.py's three hipBLASLt forms vs fp32 torch."""
    _lib()
    from tf_operator_amd.ops import gemm

    gemm._MODE = "tuned"  # exercise the native layer (default routes to torch.matmul)
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    assert rel(gemm.linear_fwd(x, w), x.float() @ w.float().t()) < 1e-2
    assert rel(gemm.linear_dgrad(dy, w), dy.float() @ w.float()) < 1e-2
    g0 = torch.randn(N, K, device=DEV, dtype=torch.float32)
    g = g0.clone()
    gemm.wgrad_acc_(g, dy, x)
    assert rel(g, g0 + dy.float().t() @ x.float()) < 1e-2
    gb = g0.to(torch.bfloat16)
    gemm.wgrad_acc_(gb, dy, x)
    assert rel(gb, g0 + dy.float().t() @ x.float()) < 2e-2
    # tuning a small form runs and installs a solution
    key = (1, 0, N, M, K, K, K, N, 0)
    idx, best, dflt, n = gemm.tune_form(key)
    assert n > 0 and best <= dflt * 1.05
    assert gemm.current_algo(key) == idx
    assert rel(gemm.linear_fwd(x, w), x.float() @ w.float().t()) < 1e-2


def test_gemm_prewarm_resolves_table():
    """gemm.prewarm() on its helper thread resolves every installed nosk
    table entry to the table's solution before any GEMM runs."""
    _lib()
    import json

    from tf_operator_amd.ops import gemm

    gemm.set_mode("nosk")
    try:
        with open(gemm.TABLE_NOSK) as f:
            tab = json.load(f)
        th = gemm.prewarm(DEV)
        assert th is not None
        th.join(timeout=60)
        assert not th.is_alive()
        if tab.get("hipblaslt") != gemm.hipblaslt_build():
            pytest.skip("nosk table measured with another hipBLASLt build")
        for e in tab["entries"]:
            key = (e["ta"], e["tb"], e["m"], e["n"], e["k"], e["lda"], e["ldb"], e["ldc"], e["beta_nz"])
            assert gemm.current_algo(key) == e["index"], key
    finally:
        gemm.set_mode("auto")


def test_first_step_gemms_run_on_the_assembly_kernel():
    """gemm.first_step (a trainer's step 0 under the hipBLASLt policies):
    forward GEMMs the assembly kernel takes run on it -- bit-identical to a
    direct toa_gemm_asm launch -- so the step never waits for the hipBLASLt
    plans still loading; other shapes take the library path."""
    L = _lib()
    from tf_operator_amd.ops import gemm

    old = gemm.mode()
    gemm.set_mode("nosk")
    try:
        torch.manual_seed(1)
        x = torch.randn(512, 384, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(768, 384, device=DEV, dtype=torch.bfloat16) / 384 ** 0.5
        direct = torch.empty(512, 768, device=DEV, dtype=torch.bfloat16)
        L.call("toa_gemm_asm", L.ptr(x), 384, L.ptr(w), 384, L.ptr(direct), 768, 512, 768, 384, L.stream(x))
        with gemm.first_step(True):
            assert gemm._asm_shape_ok(x, w)
            y = gemm.linear_fwd(x, w)
            xo = torch.randn(100, 384, device=DEV, dtype=torch.bfloat16)  # not a 256-row multiple: the library
            assert not gemm._asm_shape_ok(xo, w)
            yo = gemm.linear_fwd(xo, w)
        assert not gemm._asm_shape_ok(x, w)  # outside the scope: the policy's library path
        torch.cuda.synchronize()
        assert torch.equal(y, direct)
        assert rel(y, x.float() @ w.float().t()) < 1e-2
        assert rel(yo, xo.float() @ w.float().t()) < 1e-2
    finally:
        gemm.set_mode(old)


@pytest.mark.parametrize("B,H,Hk,S", [(2, 4, 2, 384), (1, 8, 2, 1024)])
def test_flash_attention_bshd_output_layout(B, H, Hk, S):
    """O written / dO read as [B, S, H, D] (no transpose copies in the model)
    matches the head-major path exactly."""
    _lib()
    from tf_operator_amd.ops import llm

    torch.manual_seed(11)
    D = 128
    scale = 1.0 / math.sqrt(D)
    base = [torch.randn(B, h, S, D, device=DEV, dtype=torch.bfloat16) for h in (H, Hk, Hk)]
    q1, k1, v1 = [t.clone().requires_grad_() for t in base]
    q2, k2, v2 = [t.clone().requires_grad_() for t in base]
    o1 = llm._FlashAttn.apply(q1, k1, v1, scale, False)
    o2 = llm._FlashAttn.apply(q2, k2, v2, scale, True)
    assert o2.shape == (B, S, H, D)
    assert torch.equal(o1.transpose(1, 2), o2)
    do = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16)
    o1.backward(do.transpose(1, 2))
    o2.backward(do)
    for a, b in ((q1, q2), (k1, k2), (v1, v2)):
        assert torch.equal(a.grad, b.grad)


def _mnist_trainer(graph, lr=0.01):
    from tf_operator_amd.models.vision import MnistMLP
    from tf_operator_amd.ops.llm import cross_entropy
    from tf_operator_amd.train import simple

    class _RT:
        is_chief, rank, world = True, 0, 1

        def first_step_done(self):
            pass

        def log(self, msg):
            print(msg)

    torch.manual_seed(0)
    model = MnistMLP(100, dtype=torch.bfloat16, device=DEV)
    return simple.DPTrainer(model, lambda o, y: cross_entropy(o.float(), y), _RT(), lr=lr, graph=graph)


def test_dp_trainer_hip_graph_matches_eager():
    """The captured whole-step HIP graph (device-side Adam step count, input
    copies + one replay per step, re-capture on a learning-rate change)
    follows the eager step."""
    _lib()
    from tf_operator_amd.train.data import SyntheticMNIST

    runs = []
    for graph in (False, True):
        tr = _mnist_trainer(graph)
        assert tr.use_graph == graph
        data = SyntheticMNIST(100, device=DEV, dtype=torch.bfloat16, pool=16)
        losses = []
        for i in range(12):
            if i == 8:
                tr.opt.lr = 0.002  # per-epoch decay: the graph must pick it up
            x, y = data.next()
            loss, _ = tr.step(x, y)
            losses.append(float(loss))
        if graph:
            assert tr._graph is not None and tr._key[0] == 0.002
            assert tr.opt.sync_step_count() == 12
        runs.append((losses, tr.flat.master.clone()))
    (l0, m0), (l1, m1) = runs
    assert max(abs(a - b) for a, b in zip(l0, l1)) < 1e-3, (l0, l1)
    assert float((m0 - m1).abs().max()) <= 1e-4 * float(m0.abs().max()) + 1e-6


@pytest.mark.parametrize("n", [1000, 8 * 256 * 2048 + 24, 40_000_000])
def test_grad_norm_sq_matches_fp64(n):
    """toa_sumsq at one 8-element chunk per thread (up to 32768 partials,
    then a grid-stride loop) against an fp64 sum of squares; bf16 and fp32,
    with a tail that is not a multiple of 8."""
    _lib()
    from tf_operator_amd.ops.optim import grad_norm_sq

    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    x = torch.randn(n, device=DEV, generator=g)
    for t in (x.to(torch.bfloat16), x):
        ref = float(t.double().pow(2).sum())
        got = float(grad_norm_sq(t))
        assert abs(got - ref) <= 1e-5 * ref, (t.dtype, got, ref)


def test_sum_slices_bf16_matches_fp32():
    """The copy-engine reduce-scatter's owner-side sum (toa_sum_slices_bf16):
    dst + slices summed in fp32 in order and rounded once, bit for bit."""
    _lib()
    from tf_operator_amd.ops import _lib as L

    n, k = 3 * 1024 * 1024 + 8, 7
    g = torch.Generator(device=DEV)
    g.manual_seed(9)
    dst = torch.randn(n, device=DEV, generator=g).to(torch.bfloat16)
    src = torch.randn(k * n, device=DEV, generator=g).to(torch.bfloat16)
    acc = dst.float()
    for j in range(k):
        acc += src[j * n:(j + 1) * n].float()
    want = acc.to(torch.bfloat16)
    L.call("toa_sum_slices_bf16", L.ptr(dst), L.ptr(src), k, n, n, L.stream(dst))
    torch.cuda.synchronize()
    assert torch.equal(dst.view(torch.int16), want.view(torch.int16))


def test_adamw_device_step_matches_host_step():
    _lib()
    from tf_operator_amd.ops import _lib as L

    n = 4096
    out = []
    for dev_step in (False, True):
        torch.manual_seed(3)
        master = torch.randn(n, device=DEV)
        g = torch.randn(n, device=DEV)
        m = torch.zeros(n, device=DEV)
        v = torch.zeros(n, device=DEV)
        st = torch.zeros(1, device=DEV, dtype=torch.int32)
        for k in range(1, 6):
            s = L.stream(master)
            if dev_step:
                L.call("toa_step_inc", L.ptr(st), s)
                L.call("toa_adamw_flat_dstep", L.ptr(master), None, L.ptr(g), 0, L.ptr(m), L.ptr(v), n, 1e-3, 0.9,
                       0.999, 1e-8, 0.01, L.ptr(st), 1.0, None, 0.0, s)
            else:
                L.call("toa_adamw_flat", L.ptr(master), None, L.ptr(g), 0, L.ptr(m), L.ptr(v), n, 1e-3, 0.9, 0.999,
                       1e-8, 0.01, k, 1.0, None, 0.0, s)
        out.append(master)
    assert float((out[0] - out[1]).abs().max()) < 1e-6


@pytest.mark.parametrize("N,K,T", [(100, 784, 100), (10, 100, 100), (64, 576, 64)])
def test_wgrad_fp32_accumulate(N, K, T):
    """bf16 dY^T X accumulated straight into an fp32 master gradient (one
    hipBLASLt call, beta = 1) against an fp32 reference."""
    _lib()
    from tf_operator_amd.ops import gemm

    torch.manual_seed(N + K)
    dy = torch.randn(T, N, device=DEV).to(torch.bfloat16)
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    g = torch.randn(N, K, device=DEV)
    ref = g + dy.float().t() @ x.float()
    gemm.wgrad_acc_(g, dy, x)
    assert float((g - ref).abs().max()) <= 1e-3 * float(ref.abs().max())


@pytest.mark.parametrize("M,N", [(100, 100), (100, 10), (150, 500), (1, 33)])
def test_bias_act_bwd_column_sums(M, N):
    _lib()
    from tf_operator_amd.ops import _lib as L

    torch.manual_seed(M * N)
    dy = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    y = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    dz = torch.empty_like(dy)
    db = torch.empty(N, device=DEV)
    L.call("toa_bias_act_bwd", 0, L.ptr(dy), L.ptr(y), L.ptr(dz), L.ptr(db), M, N, 1, L.stream(dy))
    g = dy.float() * (y.float() > 0)
    assert torch.equal(dz, g.to(torch.bfloat16))
    assert float((db - g.sum(0)).abs().max()) <= 1e-4 * max(1.0, float(g.abs().sum(0).max()))


@pytest.mark.parametrize("N,C,H,W,relu,res", [(4, 64, 28, 28, True, False), (2, 256, 14, 14, True, True),
                                              (3, 2048, 7, 7, False, True), (1, 24, 5, 9, True, False),
                                              (64, 128, 3, 3, False, False)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_fused_batchnorm_act(N, C, H, W, relu, res, dt):
    """HIP BatchNorm(+residual)(+ReLU), channels-last (csrc/hip/bn.hip), vs
    the fp32 PyTorch reference: output, running statistics, dx, dres,
    dgamma, dbeta; then eval mode with the updated running statistics."""
    _lib()
    from tf_operator_amd.ops.bn import batch_norm_act

    torch.manual_seed(3)
    x = (torch.randn(N, C, H, W, device=DEV) * 2 + 0.7).to(dt).to(memory_format=torch.channels_last)
    r = torch.randn(N, C, H, W, device=DEV).to(dt).to(memory_format=torch.channels_last) if res else None
    g = (torch.rand(C, device=DEV) + 0.5).to(dt)
    b = (torch.randn(C, device=DEV) * 0.1).to(dt)
    rm, rv = torch.zeros(C, device=DEV, dtype=dt), torch.ones(C, device=DEV, dtype=dt)
    xa, ga, ba = x.clone().requires_grad_(), g.clone().requires_grad_(), b.clone().requires_grad_()
    ra = r.clone().requires_grad_() if res else None
    y = batch_norm_act(xa, ga, ba, rm, rv, training=True, momentum=0.1, eps=1e-5, relu=relu, residual=ra)
    xf, gf, bf = x.float().requires_grad_(), g.float().requires_grad_(), b.float().requires_grad_()
    rf = r.float().requires_grad_() if res else None
    rmf, rvf = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    yf = torch.nn.functional.batch_norm(xf, rmf, rvf, gf, bf, True, 0.1, 1e-5)
    if res:
        yf = yf + rf
    if relu:
        yf = torch.relu(yf)
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    assert y.is_contiguous(memory_format=torch.channels_last)
    assert rel(y, yf) < tol, rel(y, yf)
    assert rel(rm, rmf) < tol and rel(rv, rvf) < tol
    dy = torch.randn_like(yf)
    y.backward(dy.to(dt))
    yf.backward(dy)
    assert rel(xa.grad, xf.grad) < 3 * tol, rel(xa.grad, xf.grad)
    assert rel(ga.grad, gf.grad) < 3 * tol, rel(ga.grad, gf.grad)
    assert rel(ba.grad, bf.grad) < 3 * tol, rel(ba.grad, bf.grad)
    if res:
        assert rel(ra.grad, rf.grad) < 3 * tol
    with torch.no_grad():
        ye = batch_norm_act(x, g, b, rm, rv, training=False, eps=1e-5, relu=relu, residual=r)
        yef = torch.nn.functional.batch_norm(x.float(), rm.float(), rv.float(), g.float(), b.float(), False, 0.1, 1e-5)
        if res:
            yef = yef + r.float()
        if relu:
            yef = torch.relu(yef)
    assert rel(ye, yef) < tol


def test_fused_batchnorm_grads_into_flat_buffer():
    """With FlatParams-managed gamma / beta, the BN backward kernel adds
    dgamma / dbeta straight into the fp32 flat gradient buffer (on top of
    what is there) and fires the bucket hooks; values match the plain path."""
    _lib()
    from tf_operator_amd.ops.bn import FusedBatchNorm2d
    from tf_operator_amd.parallel.flat import FlatParams

    torch.manual_seed(5)
    C = 64
    x = torch.randn(4, C, 8, 8, device=DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    dy = torch.randn(4, C, 8, 8, device=DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    ref = FusedBatchNorm2d(C, relu=True).to(DEV, torch.bfloat16)
    bn = FusedBatchNorm2d(C, relu=True).to(DEV, torch.bfloat16)
    xr = x.clone().requires_grad_()
    ref(xr).backward(dy)
    flat = FlatParams([bn.weight, bn.bias], grad_dtype=torch.float32)
    fired = []
    for p in (bn.weight, bn.bias):
        p._toa_ready = fired.append
    flat.grad.fill_(0.25)  # accumulate onto what is there
    xb = x.clone().requires_grad_()
    bn(xb).backward(dy)
    torch.cuda.synchronize()
    assert bn.weight.grad is None and bn.bias.grad is None and len(fired) == 2
    assert rel(bn.weight.main_grad - 0.25, ref.weight.grad.float()) < 1e-2
    assert rel(bn.bias.main_grad - 0.25, ref.bias.grad.float()) < 1e-2
    assert torch.equal(xb.grad, xr.grad)


def test_fused_batchnorm_large_mean_variance():
    """Shifted-data variance: a channel with mean 1000 and std 0.5 keeps its
    variance (no E[x^2] - E[x]^2 cancellation)."""
    _lib()
    from tf_operator_amd.ops.bn import batch_norm_act

    torch.manual_seed(4)
    x = (torch.randn(8, 64, 32, 32, device=DEV) * 0.5 + 1000.0).to(memory_format=torch.channels_last)
    rm, rv = torch.zeros(64, device=DEV), torch.ones(64, device=DEV)
    batch_norm_act(x, None, None, rm, rv, training=True, momentum=1.0, relu=False)
    ref = x.float().permute(1, 0, 2, 3).reshape(64, -1).var(1)
    assert float(((rv - ref) / ref).abs().max()) < 1e-3


def test_fused_batchnorm_momentum_none_matches_torch():
    """HIP BN with momentum=None keeps torch's cumulative running average."""
    _lib()
    from tf_operator_amd.ops.bn import FusedBatchNorm2d

    torch.manual_seed(6)
    ref = torch.nn.BatchNorm2d(32, momentum=None).to(DEV)
    bn = FusedBatchNorm2d(32, momentum=None).to(DEV)
    for i in range(3):
        x = (torch.randn(8, 32, 6, 6, device=DEV) * (i + 1) + i).to(memory_format=torch.channels_last)
        ref(x.float())
        bn(x)
    assert rel(bn.running_mean, ref.running_mean) < 1e-4
    assert rel(bn.running_var, ref.running_var) < 1e-4


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 384), (1024, 1536, 4096), (768, 512, 256),
                                   (512, 256, 192), (2048, 1024, 1152)])
def test_gemm_asm_matches_fp32(M, N, K):
    """The hand-written assembly GEMM (csrc/asm/gemm_gen.py), plain epilogue:
    y = x w^T vs fp32 torch, with an asymmetric non-square operand (guide
    section 3: catch a transposed C write), padded row strides on every
    operand, and K values that run 0, 1 and many main-loop iterations."""
    L = _lib()
    torch.manual_seed(M + N + K)
    xb = torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)[:, :K]
    w = (torch.randn(N, K, device=DEV) * 0.5 + torch.arange(N, device=DEV)[:, None] / N).to(torch.bfloat16)
    yb = torch.full((M, N + 256), 7.0, device=DEV, dtype=torch.bfloat16)
    y = yb[:, 128:128 + N]
    L.call("toa_gemm_asm", L.ptr(xb), xb.stride(0), L.ptr(w), w.stride(0), L.ptr(y), yb.stride(0), M, N, K, L.stream(y))
    ref = xb.float() @ w.float().t()
    torch.cuda.synchronize()
    assert rel(y, ref) < 1e-2, rel(y, ref)
    assert bool((yb[:, :128] == 7.0).all()) and bool((yb[:, 128 + N:] == 7.0).all())  # nothing outside C


@pytest.mark.parametrize("M,N,K", [(512, 512, 128), (2048, 1024, 4096), (768, 1280, 640)])
def test_gemm_asm_repeatable_bit_for_bit(M, N, K):
    """Eleven launches agree bit for bit: the k order is fixed, so a staging
    race (an LDS stage read before its DMA landed, or overwritten while
    read) shows up as a difference."""
    L = _lib()
    torch.manual_seed(K)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    ys = []
    for _ in range(11):
        y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        L.call("toa_gemm_asm", L.ptr(x), K, L.ptr(w), K, L.ptr(y), N, M, N, K, L.stream(y))
        ys.append(y)
    torch.cuda.synchronize()
    for y in ys[1:]:
        assert torch.equal(ys[0], y)


def test_gemm_asm_rejects_shapes_it_does_not_tile():
    """The launcher refuses (hipErrorInvalidValue) rather than run a shape
    whose tiles the kernel does not cover."""
    L = _lib()
    x = torch.randn(256, 128, device=DEV).to(torch.bfloat16)
    w = torch.randn(256, 128, device=DEV).to(torch.bfloat16)
    y = torch.empty(256, 256, device=DEV, dtype=torch.bfloat16)
    for M, N, K in ((255, 256, 128), (256, 200, 128), (256, 256, 96), (256, 256, 64)):
        rc = L.call_ret("toa_gemm_asm", L.ptr(x), 128, L.ptr(w), 128, L.ptr(y), 256, M, N, K, L.stream(y))
        assert rc != 0, (M, N, K)


def test_gemm_asm_prologue_matches_emulator():
    """The diagnostic probe kernel runs the plain kernel's prologue (tile
    mapping, buffer resources, DMA and fragment offsets) and dumps every
    register; the CPU emulator of the same instructions must agree for every
    workgroup (this caught a v_readfirstlane read-after-write hazard)."""
    import os
    import sys

    import numpy as np

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "asm"))
    import emu
    import gemm_gen
    import host_args

    L = _lib()
    skip = {0, 1, 27, 31, 48, 49, 50, 51, 52, 67, 68, 69, 70, 71, 72}
    text = gemm_gen.generate()
    for M, N, K in ((512, 768, 320), (2048, 1280, 256)):
        x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
        y = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        nwg = (M // 256) * (N // 256)
        out = torch.zeros(nwg * gemm_gen.PROBE_WORDS, device=DEV, dtype=torch.int32)
        L.call("toa_gemm_asm_probe", L.ptr(out), L.ptr(x), K, L.ptr(w), K, L.ptr(y), N, M, N, K, L.stream(x))
        torch.cuda.synchronize()
        hw = out.cpu().numpy().view(np.uint32).reshape(nwg, -1)
        karg = host_args.pack(x.data_ptr(), w.data_ptr(), y.data_ptr(), out.data_ptr(), 2 * K, 2 * K, 2 * N, 0, K,
                              M // 256, N // 256, *gemm_gen.PROBE_MAGIC)
        ref = np.zeros(nwg * gemm_gen.PROBE_WORDS, np.uint32)
        mem = emu.Memory()
        mem.add_at(out.data_ptr(), ref)
        e = emu.Emu(text, "toa_gemm_tn_asm_probe")
        for b in range(nwg):
            e.run(karg, b, mem)
        ref = ref.reshape(nwg, -1)
        bad = [(b, i) for b in range(nwg) for i in np.nonzero(hw[b] != ref[b])[0] if int(i) not in skip]
        assert not bad, bad[:10]


@pytest.mark.parametrize("M,F,K", [(256, 128, 128), (512, 384, 256), (1024, 1024, 1024)])
def test_gemm_asm_swiglu_epilogues(M, F, K):
    """Fused SwiGLU forward (gu and s from one GEMM, W kept [gate; up]) and
    backward (dgu from the down projection's data gradient, ds never
    stored) vs fp32 references."""
    from tf_operator_amd.ops import gemm, llm

    _lib()
    torch.manual_seed(3)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    wgu = (torch.randn(2 * F, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    old = gemm.mode()
    gemm.set_mode("asm")
    try:
        gu, s = gemm.swiglu_gate_up(x, wgu)
        ref_gu = x.float() @ wgu.float().t()
        assert rel(gu, ref_gu) < 1e-2
        g, u = gu[:, :F].float(), gu[:, F:].float()
        assert rel(s, torch.nn.functional.silu(g) * u) < 1e-2
        # backward: dgu from d2 [M, K] and Wd [K, F] (its transposed copy [F, K] feeds the kernel)
        if F % 256 == 0:
            wd = (torch.randn(K, F, device=DEV) / F ** 0.5).to(torch.bfloat16)
            wd._toa_wt = wd.t().contiguous()
            d2 = torch.randn(M, K, device=DEV).to(torch.bfloat16)
            dgu = gemm.swiglu_down_dgrad(d2, wd, gu)
            ds = (d2.float() @ wd.float()).to(torch.bfloat16)
            ref = llm.swiglu_bwd(ds, gu)
            assert dgu is not None and rel(dgu, ref) < 2e-2, rel(dgu, ref)
    finally:
        gemm.set_mode(old)
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,F,K", [(1024, 1536, 320), (2048, 3072, 4096)])
def test_gemm_asm_swiglu_persistent_bit_identical(M, F, K):
    """The persistent fused SwiGLU GEMMs (toa_gemm_asm_set_swiglu_persist:
    a workgroup per CU walks its tiles) write the product kernels' gu, s and
    dgu bit for bit: the grid of 2048 x 3072 has more tiles than CUs, so
    workgroups walk several (the emulator covers 1-4 workgroups)."""
    from tf_operator_amd.ops import gemm

    _lib()
    torch.manual_seed(4)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    wgu = (torch.randn(2 * F, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    wd = (torch.randn(K, F, device=DEV) / F ** 0.5).to(torch.bfloat16)
    wd._toa_wt = wd.t().contiguous()
    d2 = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    old = gemm.mode()
    gemm.set_mode("asm")
    outs = []
    try:
        for bits in (0, 3):
            _lib().call("toa_gemm_asm_set_swiglu_persist", bits)
            gu, s = gemm.swiglu_gate_up(x, wgu)
            dgu = gemm.swiglu_down_dgrad(d2, wd, gu)
            torch.cuda.synchronize()
            outs.append((gu.clone(), s.clone(), dgu.clone()))
    finally:
        _lib().call("toa_gemm_asm_set_swiglu_persist", 0)
        gemm.set_mode(old)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_llama_layer_fused_mlp_matches_library_path():
    """A llama-tiny128 training step with the assembly GEMMs and the fused
    SwiGLU (TOA_GEMM=asm, the default) follows the hipBLASLt path's loss."""
    from tf_operator_amd.ops import gemm
    from tf_operator_amd.train.llm import LlamaTrainer

    _lib()
    losses = {}
    for mode in ("nosk", "asm"):
        gemm.set_mode(mode)
        try:
            tr = LlamaTrainer("llama-tiny128", torch.device(DEV), micro_batch=2, seq_len=256, seed=0)
            b = tr.synthetic_batch()
            losses[mode] = [float(tr.step([b])) for _ in range(3)]
            del tr
        finally:
            gemm.set_mode("auto")
    for a, b in zip(losses["nosk"], losses["asm"]):
        assert abs(a - b) < 2e-2 * abs(a), losses


@pytest.mark.parametrize("B,H,Hk,S,bshd,rope", [(1, 4, 1, 256, True, False), (2, 8, 2, 1024, False, False),
                                               (1, 8, 2, 2048, True, True), (2, 32, 8, 512, True, True)])
def test_attn_dkdv_asm_vs_hip(B, H, Hk, S, bshd, rope):
    """The assembly dK/dV kernel of the dS form (csrc/asm/attn_bwd_gen.py, the
    default at D = 128) against the HIP one (attn_bwd_dkdv_ds_kernel): the
    same dK / dV / dQ to bf16 accuracy (different fp32 summation order), both
    through toa_attn_bwd and through the fused RoPE backward (d(qkv) rows);
    the assembly path deterministic run to run; and every dS block slot
    written (NaN-poisoned workspace -> finite dQ)."""
    L = _lib()
    torch.manual_seed(21)
    D = 128
    scale = 1.0 / math.sqrt(D)
    q = torch.randn(B, H, S, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, Hk, S, D, device=DEV, dtype=torch.bfloat16)
    o = torch.empty(B, S, H, D, device=DEV, dtype=torch.bfloat16) if bshd else torch.empty_like(q)
    lse = torch.empty(B, H, S, device=DEV, dtype=torch.float32)
    flags = 1 | (2 if bshd else 0)
    P = L.ptr
    L.call("toa_attn_fwd", P(q), P(k), P(v), P(o), P(lse), B, H, Hk, S, D, flags, scale, L.stream(q))
    do = torch.randn_like(o)
    nws = L.call_ret("toa_attn_bwd_ws_bytes", B, H, S, D)
    H3 = H + 2 * Hk
    pos = torch.arange(S, device=DEV, dtype=torch.float32)[:, None]
    inv = 10000.0 ** (-torch.arange(D // 2, device=DEV, dtype=torch.float32) * 2.0 / D)
    cosv, sinv = torch.cos(pos * inv).contiguous(), torch.sin(pos * inv).contiguous()

    def run(asm):
        L.call("toa_attn_set_dkdv_variant", 1 if asm else 0)
        ws = torch.full((nws,), 0xFF, device=DEV, dtype=torch.uint8)
        delta = torch.empty(B, H, S, device=DEV, dtype=torch.float32)
        if rope:
            dqkv = torch.full((B * S, H3 * D), float("nan"), device=DEV, dtype=torch.bfloat16)
            L.call("toa_attn_bwd_rope", P(q), P(k), P(v), P(o), P(do), P(lse), P(delta), P(ws), P(cosv), P(sinv),
                   P(dqkv), B, H, Hk, S, D, flags, scale, L.stream(q))
            torch.cuda.synchronize()
            x = dqkv.view(B, S, H3, D)
            return x[:, :, :H].clone(), x[:, :, H:H + Hk].clone(), x[:, :, H + Hk:].clone()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        L.call("toa_attn_bwd", P(q), P(k), P(v), P(o), P(do), P(lse), P(delta), P(ws), P(dq), P(dk), P(dv),
               B, H, Hk, S, D, flags, scale, L.stream(q))
        torch.cuda.synchronize()
        return dq, dk, dv

    try:
        hip = run(False)
        asm = run(True)
        asm2 = run(True)
    finally:
        L.call("toa_attn_set_dkdv_variant", -1)
    for name, a, h, a2 in zip(("dq", "dk", "dv"), asm, hip, asm2):
        assert torch.isfinite(a.float()).all(), name
        assert rel(a, h) < 1e-2, (name, rel(a, h))
        assert torch.equal(a, a2), name


def test_cu_masked_stream_runs_kernels():
    """toa_stream_create_cu_mask (the overlapped AdamW's TOA_OPT_CUS stream):
    a kernel on a stream limited to 32 CUs computes what it computes on the
    default stream; bad arguments are refused."""
    import ctypes

    from tf_operator_amd.ops.optim import masked_stream

    lib = _lib()
    st = masked_stream(32, 1, torch.device(DEV))
    x = torch.randn(1 << 20, device=DEV)
    ref = (x * 2).sum()
    with torch.cuda.stream(st):
        got = (x * 2).sum()
    st.synchronize()
    assert torch.equal(got, ref)
    h = ctypes.c_void_p()
    with pytest.raises(RuntimeError):
        lib.call("toa_stream_create_cu_mask", 2, 32, ctypes.byref(h))
    with pytest.raises(RuntimeError):
        lib.call("toa_stream_create_cu_mask", 1, 0, ctypes.byref(h))


def test_fused_clipping_norm_matches_full_pass(monkeypatch):
    """World 1: the clipping norm from the weight-gradient kernels' partials
    (ops/gemm.SumsqSession, TOA_FUSED_NORM default) equals the full pass over
    the gradient to fp32 summation order, every step is served from the
    partials, and the training trajectory follows the full-pass trainer."""
    from tf_operator_amd.models.llama import PRESETS
    from tf_operator_amd.train.llm import LlamaTrainer

    _lib()
    runs = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("TOA_FUSED_NORM", fused)
        tr = LlamaTrainer(PRESETS["llama-tiny128"], torch.device(DEV), micro_batch=2, seq_len=512, seed=0)
        assert (tr.opt.sumsq is not None) == (fused == "1")
        b = tr.synthetic_batch()
        norms, losses = [], []
        for _ in range(3):
            losses.append(float(tr.step([b])))
            norms.append(float(tr.opt.last_norm_sq))
        if fused == "1":
            assert tr.opt.sumsq.hits == 3, "a step fell back to the full pass"
            # the partials' region layout covers every linear weight; the rest is embeddings / norms
            assert len(tr.opt.sumsq.regions) == 2 * 4 + 1   # wqkv, wo, wgu, wd per layer + lm_head
        runs[fused] = (norms, losses)
    for a, b in zip(runs["1"][0], runs["0"][0]):
        assert abs(a - b) <= 1e-3 * b, (runs["1"][0], runs["0"][0])
    for a, b in zip(runs["1"][1], runs["0"][1]):
        assert abs(a - b) <= 2e-2, (runs["1"][1], runs["0"][1])


def test_wgrad_sumsq_partials_whole_and_split_tiles():
    """The weight-gradient GEMM with a partials region: 384 tiles = 256
    whole-K tiles (assembly epilogue) + 128 tail tiles in 2 k-pieces (the
    reduce kernel) -- the region sums to the squared norm of the result."""
    import types

    from tf_operator_amd.ops import gemm

    _lib()
    torch.manual_seed(6)
    T, N, K = 2048, 6144, 4096
    dy = torch.randn(T, N, device=DEV).to(torch.bfloat16)
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    w = torch.nn.Parameter(torch.zeros(N, K, device=DEV, dtype=torch.bfloat16))
    w.main_grad = torch.zeros(N, K, device=DEV, dtype=torch.bfloat16)
    seg = types.SimpleNamespace(param=w, offset=0, numel=N * K)
    flat = types.SimpleNamespace(segments=[seg], device=torch.device(DEV), numel=N * K, grad=w.main_grad.view(-1))
    sess = gemm.SumsqSession(flat, [w])
    gemm._SESSIONS.add(sess)
    try:
        gemm.wgrad_hip_(w.main_grad, dy, x, 0.0)
        torch.cuda.synchronize()
    finally:
        gemm._SESSIONS.discard(sess)
    assert sess.written == {w.main_grad.data_ptr()}
    got = float(sess.buf.double().sum())
    want = float(w.main_grad.double().pow(2).sum())
    assert abs(got - want) <= 1e-3 * want, (got, want)
    out, ws = torch.zeros(1, device=DEV), torch.empty(32768, device=DEV)
    sess.norm_sq(out, ws)
    assert abs(float(out) - want) <= 1e-3 * want


def test_adamw_writes_transposed_copies_bit_identical(monkeypatch):
    """TOA_ADAM_WT (default): the update writes each weight's W^T copy in the
    same pass (toa_adamw_wt) -- master, moments and bf16 weights bit for bit
    as the flat update + separate refresh, and every copy equals W^T."""
    from tf_operator_amd.models.llama import PRESETS
    from tf_operator_amd.train.llm import LlamaTrainer

    _lib()
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("TOA_ADAM_WT", mode)
        tr = LlamaTrainer(PRESETS["llama-tiny128"], torch.device(DEV), micro_batch=2, seq_len=512, seed=0)
        assert (tr.opt.fused_wt is not None) == (mode == "1")
        if mode == "1":
            assert len(tr.opt._fused_items()) == 2 * 4 + 1
        b = tr.synthetic_batch()
        losses = [float(tr.step([b])) for _ in range(3)]
        torch.cuda.synchronize()
        for _, _, p, view in tr.wt.items:
            assert torch.equal(view, p.data.t())
        f = tr.flat
        out[mode] = (losses, f.master.clone(), f.exp_avg.clone(), f.exp_avg_sq.clone(), f.param.detach().clone())
    assert out["1"][0] == out["0"][0]
    for a, b in zip(out["1"][1:], out["0"][1:]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,S,Hq,Hkv", [(2, 512, 4, 2), (1, 1024, 8, 4)])
def test_qkv_rope_attention_fused_matches_two_nodes(B, S, Hq, Hkv):
    """toa_gemm_asm_rope (the QKV projection writing rotated head-major
    q | k | v) + attention against linear + rope_attention: the output and
    the input / weight gradients, to bf16 rounding (the fused path rotates
    the fp32 accumulators, the other the bf16 GEMM output)."""
    from tf_operator_amd.ops import gemm, llm
    from tf_operator_amd.ops.linear import linear

    _lib()
    rope_tables = llm.rope_tables
    old = gemm.mode()
    gemm.set_mode("asm")
    try:
        torch.manual_seed(S + Hq)
        D, Hd = 128, 512
        x0 = torch.randn(B * S, Hd, device=DEV).to(torch.bfloat16)
        w0 = (torch.randn((Hq + 2 * Hkv) * D, Hd, device=DEV) / Hd ** 0.5).to(torch.bfloat16)
        cos, sin = rope_tables(S, D, device=DEV)
        dout = torch.randn(B, S, Hq, D, device=DEV).to(torch.bfloat16)
        res = []
        for fused in (True, False):
            x = x0.clone().requires_grad_()
            w = torch.nn.Parameter(w0.clone())
            w.main_grad = torch.zeros_like(w)
            assert llm.qkv_rope_attention_ok(x, w, S, Hq, Hkv, D)
            o = (llm.qkv_rope_attention(x, w, cos, sin, B, S, Hq, Hkv, D) if fused
                 else llm.rope_attention(linear(x, w), cos, sin, B, S, Hq, Hkv, D))
            o.backward(dout)
            torch.cuda.synchronize()
            res.append((o.detach().float(), x.grad.float(), w.main_grad.float()))
    finally:
        gemm.set_mode(old)
    for a, b in zip(*res):
        assert rel(a, b) < 2e-2, rel(a, b)


def test_attn_out_proj_delta_rows(monkeypatch):
    """_AttnOutProj: the output projection's data gradient through
    toa_gemm_asm_delta equals the plain data gradient bit for bit, the -delta
    rows it leaves equal -rowsum(dO * O) per head, and a llama-tiny128
    trainer with the rows handed to the attention backward follows the one
    with the attention's own delta pass."""
    from tf_operator_amd.models.llama import PRESETS
    from tf_operator_amd.ops import gemm, llm
    from tf_operator_amd.train.llm import LlamaTrainer

    _lib()
    old = gemm.mode()
    gemm.set_mode("asm")
    try:
        torch.manual_seed(8)
        B, S, H, D = 2, 512, 4, 128
        o = torch.randn(B * S, H * D, device=DEV).to(torch.bfloat16).requires_grad_()
        wo = torch.nn.Parameter((torch.randn(H * D, H * D, device=DEV) / (H * D) ** 0.5).to(torch.bfloat16))
        wo.main_grad = torch.zeros_like(wo)
        wo._toa_wt = wo.data.t().contiguous()
        dy = torch.randn(B * S, H * D, device=DEV).to(torch.bfloat16)
        llm.attn_out_proj(o, wo, B, S, H).backward(dy)
        torch.cuda.synchronize()
        pend = llm._PENDING_DELTA
        llm._PENDING_DELTA = None
        assert pend is not None and pend[0] == o.grad.data_ptr()
        assert torch.equal(o.grad, gemm.linear_dgrad(dy, wo))
        ref = -(o.grad.float() * o.detach().float()).view(B, S, H, D).sum(-1).permute(0, 2, 1).reshape(-1)
        assert rel(pend[2], ref) < 1e-4
    finally:
        gemm.set_mode(old)
    losses = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("TOA_ATTN_DELTA_FUSED", fused)
        tr = LlamaTrainer(PRESETS["llama-tiny128"], torch.device(DEV), micro_batch=2, seq_len=512, seed=0)
        b = tr.synthetic_batch()
        losses[fused] = [float(tr.step([b])) for _ in range(3)]
        assert llm._PENDING_DELTA is None
    for a, c in zip(losses["1"], losses["0"]):
        assert abs(a - c) <= 1e-3 * abs(c), losses


def test_resadd_epilogue_and_presummed_norm(monkeypatch):
    """The residual add in the output projection's epilogue
    (toa_gemm_asm_resadd) + the presummed RMSNorm: out = o wo^T + h to one
    bf16 rounding, and a llama-tiny128 trainer with it follows the one that
    adds in the norm kernel."""
    from tf_operator_amd.models.llama import PRESETS
    from tf_operator_amd.ops import gemm, llm
    from tf_operator_amd.train.llm import LlamaTrainer

    _lib()
    old = gemm.mode()
    gemm.set_mode("asm")
    try:
        torch.manual_seed(12)
        T, Hd = 1024, 512
        o = torch.randn(T, Hd, device=DEV).to(torch.bfloat16)
        wo = (torch.randn(Hd, Hd, device=DEV) / Hd ** 0.5).to(torch.bfloat16)
        h = torch.randn(T, Hd, device=DEV).to(torch.bfloat16)
        assert llm.attn_out_proj_resadd_ok(o, wo, h)
        out = llm._AttnOutProj.apply(o, wo, 2, 512, 4, h)
        ref = o.float() @ wo.float().t() + h.float()
        assert rel(out, ref) < 1e-2
    finally:
        gemm.set_mode(old)
    losses = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("TOA_RESADD_FUSED", fused)
        tr = LlamaTrainer(PRESETS["llama-tiny128"], torch.device(DEV), micro_batch=2, seq_len=512, seed=0)
        b = tr.synthetic_batch()
        losses[fused] = [float(tr.step([b])) for _ in range(3)]
    for a, c in zip(losses["1"], losses["0"]):
        assert abs(a - c) <= 2e-3 * abs(c), losses
