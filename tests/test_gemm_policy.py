"""ops/gemm.py policy switches and failure paths that need no GPU:
the TOA_WGRAD / TOA_GEMM_TN_FIRST opt-outs, the assembly weight gradient's
fallback to the HIP kernel on a refused shape, and prewarm_early's tolerance
of a kubelet that cannot answer."""
import pytest
import torch

from tf_operator_amd.ops import _lib, gemm


@pytest.fixture
def fresh_wgrad(monkeypatch):
    monkeypatch.setattr(gemm, "_WGRAD_KERNEL", None)
    yield
    gemm._WGRAD_KERNEL = None


def test_wgrad_env_opt_out(monkeypatch, fresh_wgrad):
    monkeypatch.setenv("TOA_WGRAD", "hip")
    assert gemm.wgrad_kernel() == "hip"


def test_wgrad_env_rejects_unknown(monkeypatch, fresh_wgrad):
    monkeypatch.setenv("TOA_WGRAD", "cublas")
    with pytest.raises(ValueError):
        gemm.wgrad_kernel()


def test_wgrad_asm_refusal_falls_back_to_hip(monkeypatch, fresh_wgrad):
    calls = []
    monkeypatch.setattr(gemm, "_WGRAD_KERNEL", "asm")
    monkeypatch.setattr(_lib, "use_hip", lambda t: True)
    monkeypatch.setattr(_lib, "ptr", lambda t: 0)
    monkeypatch.setattr(_lib, "stream", lambda t: 0)

    def call_ret(name, *a):
        calls.append(name)
        return 0 if name == "toa_wgrad_workspace" else gemm.HIP_ERROR_INVALID_VALUE

    monkeypatch.setattr(_lib, "call_ret", call_ret)
    monkeypatch.setattr(_lib, "call", lambda name, *a: calls.append(name))
    g = torch.zeros(256, 256, dtype=torch.bfloat16)
    dy = torch.zeros(1024, 256, dtype=torch.bfloat16)
    gemm.wgrad_hip_(g, dy, dy)
    assert calls == ["toa_wgrad_workspace", "toa_wgrad_asm", "toa_wgrad"]
    monkeypatch.setattr(_lib, "call_ret", lambda name, *a: 0 if name == "toa_wgrad_workspace" else 700)
    with pytest.raises(RuntimeError, match="hipError 700"):
        gemm.wgrad_hip_(g, dy, dy)


def test_first_step_opt_out(monkeypatch):
    monkeypatch.setattr(gemm, "_MODE", "nosk")
    monkeypatch.setattr(_lib, "has", lambda name: True)
    assert gemm.first_step().on
    monkeypatch.setenv("TOA_GEMM_TN_FIRST", "0")
    assert not gemm.first_step().on


@pytest.mark.parametrize("exc", ["grpc", ImportError("No module named 'grpc'"), OSError("socket")])
def test_prewarm_early_tolerates_kubelet_lookup_failures(monkeypatch, exc):
    from tf_operator_amd.train import dist as tdist

    if exc == "grpc":
        grpc = pytest.importorskip("grpc")

        class _Rpc(grpc.RpcError):
            pass

        exc = _Rpc("kubelet pod-resources socket unavailable")

    def boom():
        raise exc

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(tdist, "local_device_index", boom)
    monkeypatch.setattr(gemm, "_MODE", "nosk")
    assert gemm.prewarm_early() is None
