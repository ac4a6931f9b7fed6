"""RMSNorm.presummed: the residual-sum-already-added form of the norm.

It must run the module's forward pre-hooks -- ZeRO-1 hangs each module's
parameter all-gather wait on them (train/llm._install_param_waits); a direct
_NormFn call skipped the wait and read the weight mid-gather (the
intermittent world-4/8 mismatch with TOA_RESADD_FUSED=1, profiles/r6_zrep3).
"""
import torch

from tf_operator_amd.ops.norm import RMSNorm


def test_presummed_runs_pre_hooks_and_matches_rms_norm():
    torch.manual_seed(0)
    n = RMSNorm(64, dtype=torch.float32)
    with torch.no_grad():
        n.weight.uniform_(0.5, 1.5)
    calls = []
    n.register_forward_pre_hook(lambda mod, args: calls.append(1))
    h = torch.randn(3, 5, 64, requires_grad=True)
    h_out, y = n.presummed(h)
    assert calls == [1]
    ref = h.float() * torch.rsqrt(h.float().pow(2).mean(-1, keepdim=True) + n.eps) * n.weight
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(h_out, h)
    # backward: dh flows through both outputs (the h pass-through and the norm)
    g = torch.randn_like(y)
    (y * g).sum().add(h_out.sum()).backward()
    h2 = h.detach().clone().requires_grad_(True)
    ref2 = h2 * torch.rsqrt(h2.pow(2).mean(-1, keepdim=True) + n.eps) * n.weight.detach()
    (ref2 * g).sum().add(h2.sum()).backward()
    torch.testing.assert_close(h.grad, h2.grad, rtol=1e-4, atol=1e-5)
