"""Where does the ResNet-50 payload's loss go NaN on the GPU?  Runs the
DPTrainer on one batch, printing loss / grad norm / param finiteness per
step, with and without the whole-step HIP graph."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from tf_operator_amd.models.vision import resnet50  # noqa: E402
from tf_operator_amd.ops.llm import cross_entropy  # noqa: E402
from tf_operator_amd.train import simple  # noqa: E402
from tf_operator_amd.train.data import SyntheticImages  # noqa: E402


class RT:
    rank, world, is_chief = 0, 1, True

    def first_step_done(self):
        pass

    def log(self, *a):
        print(*a, flush=True)


def run(graph, steps=int(os.environ.get("STEPS", "12")), batch=int(os.environ.get("B", "64"))):
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m = resnet50(dtype=torch.bfloat16, device=dev).to(memory_format=torch.channels_last)
    tr = simple.DPTrainer(m, lambda o, y: cross_entropy(o.float(), y), RT(), lr=1e-3, bucket_mb=64, graph=graph)
    data = SyntheticImages(batch, (3, 224, 224), rank=0, device=dev, dtype=torch.bfloat16)
    for i in range(steps):
        loss, out = tr.step(*data.next())
        torch.cuda.synchronize()
        f = tr.flat
        print(f"bn={os.environ.get('TOA_BN', 'hip')} graph={graph} step {i}: loss {float(loss):.4f} out_finite {bool(torch.isfinite(out).all())} "
              f"param_finite {bool(torch.isfinite(f.param).all())} master_finite {bool(torch.isfinite(f.master).all())} "
              f"|m| {float(f.exp_avg.abs().max()):.3e} |v| {float(f.exp_avg_sq.abs().max()):.3e}", flush=True)


if __name__ == "__main__":
    from tf_operator_amd.examples.common import use_shipped_miopen_find_db

    if os.environ.get("FINDDB", "1") == "1":
        use_shipped_miopen_find_db()
    for g in os.environ.get("GRAPH", "0,1").split(","):
        run(graph=g == "1")
