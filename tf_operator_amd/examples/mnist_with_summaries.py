"""Single-worker MNIST with summaries (reference:
examples/v1/mnist_with_summaries/mnist_with_summaries.py): 784 -> 500 ReLU ->
dropout(keep 0.9, fused in the MFMA epilogue) -> 10, Adam, accuracy every 10
steps (HIP argmax kernel), scalar summaries to <log_dir>/events.jsonl and a
kernel-trace marker every 100th step (the FULL_TRACE analog)."""
from __future__ import annotations

import argparse
import json
import os
import time

import torch

from tf_operator_amd.examples.common import model_dtype, pick_device
from tf_operator_amd.models.vision import MnistMLP
from tf_operator_amd.ops.llm import cross_entropy
from tf_operator_amd.ops.mlp import accuracy
from tf_operator_amd.train import simple
from tf_operator_amd.train.data import SyntheticMNIST
from tf_operator_amd.train.runtime import Runtime
from tf_operator_amd.utils.profiling import trace_step


class SummaryWriter:
    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.f = open(os.path.join(log_dir, "events.jsonl"), "a")

    def scalar(self, tag, value, step):
        self.f.write(json.dumps({"wall_time": time.time(), "step": step, "tag": tag, "value": float(value)}) + "\n")
        self.f.flush()


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--max_steps", type=int, default=1000)
    p.add_argument("--learning_rate", type=float, default=0.001)
    p.add_argument("--batch_size", type=int, default=150)
    p.add_argument("--dropout", type=float, default=0.9, help="keep probability")
    p.add_argument("--log_dir", default=os.environ.get("TOA_LOG_DIR", "/tmp/tensorflow/mnist/logs"))
    p.add_argument("--trace_every", type=int, default=100,
                   help="FULL_TRACE analog (mnist_with_summaries.py:162-171): every N-th step runs under "
                        "torch.profiler and is written as a Chrome trace; 0 disables")
    a = p.parse_args(argv)
    rt = Runtime()
    rt.init_dist()
    dev = pick_device()
    torch.manual_seed(0)
    model = MnistMLP(500, keep_prob=a.dropout, dtype=model_dtype(dev), device=dev)
    tr = simple.DPTrainer(model, lambda o, y: cross_entropy(o.float(), y), rt, lr=a.learning_rate)
    data = SyntheticMNIST(a.batch_size, rt.rank, rt.world, device=dev, dtype=model_dtype(dev))
    test_x, test_y = SyntheticMNIST(1000, rank=99, device=dev, dtype=model_dtype(dev)).next()
    sw = SummaryWriter(os.path.join(a.log_dir, "train"))
    for i in range(1, a.max_steps + 1):
        x, y = data.next()
        model.train()
        if a.trace_every and i % a.trace_every == a.trace_every - 1:
            path = os.path.join(a.log_dir, "train", f"trace_step{i}.json")
            loss, _ = trace_step(lambda: tr.step(x, y), path)
            sw.scalar("trace_written", 1, i)
        else:
            loss, _ = tr.step(x, y)
        if i % 10 == 0:
            model.eval()
            with torch.no_grad():
                acc = float(accuracy(model(test_x), test_y))
            sw.scalar("accuracy", acc, i)
            sw.scalar("cross_entropy", float(loss), i)
            rt.log(f"Accuracy at step {i}: {acc:.3f}")
    rt.report(samples_per_sec=None)


if __name__ == "__main__":
    main()
