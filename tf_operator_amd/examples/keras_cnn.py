"""Multi-worker CNN (reference: examples/v1/distribution_strategy/keras-API/
multi_worker_strategy-with-keras.py): 3x Conv3x3 + 2x MaxPool + Dense64 +
Dense10 on MNIST-shaped images, batch 64 per replica, Adam with the
1e-3/1e-4/1e-5 epoch decay, all-reduce DP (RCCL on MI355X -- the NCCL
CollectiveCommunication of the reference), checkpoint every epoch, final
model saved by the chief."""
from __future__ import annotations

import argparse
import os

import torch

from tf_operator_amd.examples.common import model_dtype, pick_device
from tf_operator_amd.models.vision import KerasCNN
from tf_operator_amd.ops.llm import cross_entropy
from tf_operator_amd.ops.mlp import accuracy
from tf_operator_amd.train import checkpoint as ckpt
from tf_operator_amd.train import simple
from tf_operator_amd.train.data import SyntheticMNIST
from tf_operator_amd.train.runtime import Runtime


def decay(epoch):
    return 1e-3 if epoch < 3 else (1e-4 if epoch < 7 else 1e-5)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--steps_per_epoch", type=int, default=70)
    p.add_argument("--batch_per_replica", type=int, default=64)
    p.add_argument("--saved_model_dir", default=os.environ.get("TOA_CHECKPOINT_DIR", "/tmp/keras-ckpt"))
    a = p.parse_args(argv)
    rt = Runtime()
    rt.install_preemption_handler()
    rt.init_dist()
    dev = pick_device()
    torch.manual_seed(0)
    model = KerasCNN(dtype=model_dtype(dev), device=dev)
    tr = simple.DPTrainer(model, lambda o, y: cross_entropy(o.float(), y), rt, lr=decay(0))
    data = SyntheticMNIST(a.batch_per_replica, rt.rank, rt.world, device=dev, image=True, dtype=model_dtype(dev),
                          pool=a.steps_per_epoch)
    start = tr.maybe_resume(a.saved_model_dir)
    if start:
        rt.log(f"resumed from checkpoint at step {start} (epoch {start // a.steps_per_epoch})")
    for epoch in range(start // a.steps_per_epoch, a.epochs):
        tr.opt.lr = decay(epoch)
        for _ in range(a.steps_per_epoch):
            x, y = data.next()
            loss, out = tr.step(x, y)
        rt.log(f"epoch {epoch + 1}/{a.epochs} loss {float(loss):.4f} acc {float(accuracy(out, y)):.3f} "
               f"lr {tr.opt.lr}")
        tr.save(a.saved_model_dir)  # ModelCheckpoint per epoch (chief writes)
        if rt.preempted.is_set():
            raise SystemExit(143)
    if rt.is_chief:
        ckpt.save(os.path.join(a.saved_model_dir, "final"), tr.step_idx, tr.state(), keep=1)


if __name__ == "__main__":
    main()
