"""ResNet-50 synthetic-ImageNet payload (BASELINE config #2: TFJob PS=1
Worker=2, each worker on 1x MI355X).  Workers train in the all-reduce world
(bf16 channels-last convs through MIOpen, fused HIP dense head and Adam);
the PS replica of the TFJob spec is idle in this mode (PS mode is the
parity path in dist_mnist).  Reports samples/sec to the operator."""
from __future__ import annotations

import argparse
import time

import torch

from tf_operator_amd.examples.common import model_dtype, pick_device
from tf_operator_amd.models.vision import resnet50
from tf_operator_amd.ops.llm import cross_entropy
from tf_operator_amd.train import simple
from tf_operator_amd.train.data import SyntheticImages
from tf_operator_amd.train.runtime import Runtime


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--image", type=int, default=224)
    a = p.parse_args(argv)
    rt = Runtime()
    if rt.role == "ps":
        while True:
            time.sleep(3600)
    info = rt.init_dist()
    dev = pick_device() if info.backend != "gloo" else torch.device("cpu")
    dt_ = model_dtype(dev)
    torch.manual_seed(0)
    model = resnet50(dtype=dt_, device=dev).to(memory_format=torch.channels_last)
    tr = simple.DPTrainer(model, lambda o, y: cross_entropy(o.float(), y), rt, lr=1e-3, bucket_mb=64)
    data = SyntheticImages(a.batch, (3, a.image, a.image), rank=rt.rank, device=dev, dtype=dt_)
    for _ in range(a.warmup):
        tr.step(*data.next())
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss, _ = tr.step(*data.next())
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sps = a.batch * rt.world * a.steps / dt
    rt.report(samples_per_sec=sps)
    rt.log(f"resnet50 {sps:.1f} samples/s ({dt / a.steps * 1e3:.1f} ms/step, loss {float(loss):.3f})")


if __name__ == "__main__":
    main()
