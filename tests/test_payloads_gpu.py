"""The bundled payloads' training steps on one MI355X: losses stay finite
and fall (a NaN in any fused kernel of the path shows up here), and the
ResNet payload's PS-mode worker step (no peer: the process group is the
worker alone, so only the plumbing, not RCCL, is exercised)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _RT:
    rank, world, is_chief = 0, 1, True

    def first_step_done(self):
        pass

    def log(self, *a):
        pass


@pytest.mark.parametrize("graph", [False, True])
def test_resnet_payload_trains_finite(graph):
    from tf_operator_amd.models.vision import ResNet
    from tf_operator_amd.ops import _lib
    from tf_operator_amd.ops.llm import cross_entropy
    from tf_operator_amd.train import simple
    from tf_operator_amd.train.data import SyntheticImages

    assert _lib.available(), _lib.load_error()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = ResNet(layers=(1, 1, 1, 1), num_classes=100, dtype=torch.bfloat16, device=dev)
    m = m.to(memory_format=torch.channels_last)
    tr = simple.DPTrainer(m, lambda o, y: cross_entropy(o.float(), y), _RT(), lr=1e-3, bucket_mb=64, graph=graph)
    data = SyntheticImages(32, (3, 64, 64), classes=100, rank=0, device=dev, dtype=torch.bfloat16)
    losses = []
    for _ in range(8):
        loss, out = tr.step(*data.next())
        losses.append(float(loss))
    torch.cuda.synchronize()
    assert all(x == x and abs(x) < 1e4 for x in losses), losses
    assert losses[-1] < losses[0], losses
    assert torch.isfinite(tr.flat.param).all() and torch.isfinite(tr.flat.master).all()
