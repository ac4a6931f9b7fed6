"""Keras-model-to-estimator payload (reference: examples/v1/
distribution_strategy/estimator-API/keras_model_to_estimator.py):
Dense(16, ReLU) -> Dense(1, sigmoid) on 1024 x 10 random features, SGD 0.2,
batch 32.  train_and_evaluate semantics: Chief/Worker replicas train in the
all-reduce world and the chief writes checkpoints; the Evaluator replica
(outside the world) polls the checkpoint directory and evaluates
each new checkpoint until the trainers finish."""
from __future__ import annotations

import argparse
import os
import time

import torch

from tf_operator_amd.models.vision import EstimatorDNN
from tf_operator_amd.train import checkpoint as ckpt
from tf_operator_amd.train import simple
from tf_operator_amd.train.data import SyntheticBinary
from tf_operator_amd.train.runtime import Runtime


def bce(logits, y):
    return torch.nn.functional.binary_cross_entropy_with_logits(logits, y)


def evaluate(model, ckpt_dir, rt, timeout, want_step):
    seen, deadline = None, time.time() + timeout
    x, y = SyntheticBinary(1024, 1024, rank=7).next()
    while time.time() < deadline:
        path = ckpt.latest_path(ckpt_dir)
        if path and path != seen:
            seen = path
            payload = ckpt.load_latest(ckpt_dir)
            flat = payload["state"]["flat"]
            off = 0
            with torch.no_grad():
                for (_, off0, n), p in zip(flat["layout"], reversed([q for q in model.parameters()])):
                    p.copy_(flat["master"][off0:off0 + n].view_as(p).to(p.dtype))
                acc = float(((model(x) > 0).float() == y).float().mean())
            rt.log(f"evaluated checkpoint step {payload['step']}: accuracy {acc:.3f}")
            if payload["step"] >= want_step:
                return acc
        time.sleep(0.2)
    raise SystemExit("evaluator timed out waiting for checkpoints")


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--ckpt_dir", default=os.environ.get("TOA_CHECKPOINT_DIR", "/tmp/estimator-ckpt"))
    p.add_argument("--eval_timeout", type=float, default=120)
    a = p.parse_args(argv)
    rt = Runtime()
    torch.manual_seed(0)
    model = EstimatorDNN(device="cpu")
    if rt.role == "evaluator":
        evaluate(model, a.ckpt_dir, rt, a.eval_timeout, a.steps)
        return
    if rt.role == "ps":
        while True:
            time.sleep(3600)
    rt.init_dist()
    tr = simple.DPTrainer(model, bce, rt, lr=0.2, optimizer="sgd")
    simple.run(tr, SyntheticBinary(rank=rt.rank), a.steps, log_every=50, ckpt_dir=a.ckpt_dir, ckpt_every=50,
               samples_per_step=32 * rt.world)


if __name__ == "__main__":
    main()
