"""Distributed MNIST MLP -- the reference's flagship TFJob payload
(examples/v1/dist-mnist/dist_mnist.py), rebuilt for PyTorch-ROCm.

Model (dist_mnist.py:166-192): 784 -> hidden (ReLU) -> 10 softmax, Adam,
batch 100, `--train_steps` global steps.  Two distribution modes:

* all-reduce DP (default; MI355X path): every replica in the RCCL/gloo world
  (Chief/Master/Worker) trains on its own shard; gradients are all-reduced
  from the flat buffer; fused HIP Adam.
* parameter server (`--mode ps`, or automatic when the TFJob has PS
  replicas): PS replicas own flat parameter shards and apply Adam; workers
  push gradients / pull parameters every step (async), or with
  `--sync_replicas` the PS aggregates `--replicas_to_aggregate` gradients per
  update (SyncReplicasOptimizer, dist_mnist.py:196-219).

Data is synthetic MNIST-shaped with learnable labels (no downloads).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

from tf_operator_amd.examples.common import model_dtype, pick_device
from tf_operator_amd.models.vision import MnistMLP
from tf_operator_amd.ops.llm import cross_entropy
from tf_operator_amd.ops.mlp import accuracy
from tf_operator_amd.train import simple
from tf_operator_amd.train.data import SyntheticMNIST
from tf_operator_amd.train.runtime import Runtime


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--train_steps", type=int, default=2000)
    p.add_argument("--batch_size", type=int, default=100)
    p.add_argument("--learning_rate", type=float, default=0.01)
    p.add_argument("--hidden_units", type=int, default=100)
    p.add_argument("--mode", choices=["auto", "allreduce", "ps"], default="auto")
    p.add_argument("--sync_replicas", action="store_true")
    p.add_argument("--replicas_to_aggregate", type=int, default=0)
    p.add_argument("--log_every", type=int, default=100)
    p.add_argument("--checkpoint_every", type=int, default=0)
    p.add_argument("--min_accuracy", type=float, default=0.0, help="fail (exit 1) below this final accuracy")
    return p.parse_args(argv)


def loss_fn(logits, y):
    return cross_entropy(logits.float(), y)


def run_allreduce(a, rt):
    dev = pick_device()
    torch.manual_seed(0)
    model = MnistMLP(a.hidden_units, dtype=model_dtype(dev), device=dev)
    tr = simple.DPTrainer(model, loss_fn, rt, lr=a.learning_rate)
    if tr.bucketer.enabled:
        rt.log(f"gradient all-reduce: one-shot IPC {'on' if tr.bucketer.ipc is not None else 'off'} "
               f"({getattr(tr.bucketer, 'ipc_reason', '')})")
    data = SyntheticMNIST(a.batch_size, rt.rank, rt.world, device=dev, dtype=model_dtype(dev), pool=600)
    steps = max(1, a.train_steps // rt.world)  # train_steps is global (dist_mnist.py:64-69)
    last = simple.run(tr, data, steps, a.log_every, rt.ckpt_dir, a.checkpoint_every, metric_fn=accuracy,
                      samples_per_step=a.batch_size * rt.world)
    x, y = SyntheticMNIST(2000, rank=10_000, device=dev, dtype=model_dtype(dev)).next()
    with torch.no_grad():
        acc = float(accuracy(model(x), y))
    rt.log(f"validation accuracy {acc:.3f}")
    return acc


def _flat_params(model):
    return torch.cat([p.detach().float().reshape(-1).cpu() for p in model.parameters()]).numpy()


def _load_flat(model, flat):
    off = 0
    with torch.no_grad():
        for p in model.parameters():
            n = p.numel()
            p.copy_(torch.from_numpy(flat[off:off + n]).view_as(p).to(p.dtype))
            off += n


def run_ps(a, rt):
    from tf_operator_amd.parallel.ps import ParameterServer, PSClient, shard_sizes
    from tf_operator_amd.train.dist import own_port, resolve_endpoint

    hosts = [h for h in os.environ.get("TOA_PS_HOSTS", "").split(",") if h]
    torch.manual_seed(0)
    cpu_model = MnistMLP(a.hidden_units, dtype=torch.float32, device="cpu")
    flat0 = _flat_params(cpu_model)
    sizes = shard_sizes(flat0.size, len(hosts))
    n_workers = int(os.environ.get("WORLD_SIZE", "1"))
    if rt.role == "ps":
        idx = int(os.environ.get("TOA_REPLICA_INDEX", "0"))
        off = sum(sizes[:idx])
        agg = (a.replicas_to_aggregate or n_workers) if a.sync_replicas else 0
        ps = ParameterServer(flat0[off:off + sizes[idx]], lr=a.learning_rate, sync_replicas=agg,
                             port=own_port(2222))
        rt.log(f"parameter server shard {idx} ({sizes[idx]} params) on :{ps.port} sync={agg}")
        ps.serve_forever()  # like server.join(): PS replicas never finish on their own
        return None
    dev = pick_device()
    model = MnistMLP(a.hidden_units, dtype=torch.float32, device=dev)
    client = None
    for _ in range(600):  # PS may start later than the worker
        try:
            client = PSClient([resolve_endpoint(h) for h in hosts], sizes)
            break
        except OSError:
            time.sleep(0.1)
    if client is None:
        raise SystemExit("could not reach the parameter servers")
    _load_flat(model, client.pull())
    data = SyntheticMNIST(a.batch_size, int(os.environ.get("RANK", "0")), n_workers, device=dev)
    steps = max(1, a.train_steps // n_workers)
    for s in range(1, steps + 1):
        x, y = data.next()
        model.zero_grad(set_to_none=True)
        loss = loss_fn(model(x), y)
        loss.backward()
        g = torch.cat([p.grad.float().reshape(-1) for p in model.parameters()]).cpu().numpy()
        _load_flat(model, client.push(g))
        if s == 1:
            rt.first_step_done()
        if a.log_every and s % a.log_every == 0:
            rt.log(f"step {s} loss {float(loss):.4f} ps-version {client.version}")
    x, y = SyntheticMNIST(2000, rank=10_000, device=dev).next()
    with torch.no_grad():
        acc = float(accuracy(model(x), y))
    rt.log(f"validation accuracy {acc:.3f}")
    client.close()
    return acc


def main(argv=None):
    a = parse(argv)
    rt = Runtime()
    rt.install_preemption_handler()
    mode = a.mode
    if mode == "auto":
        mode = "ps" if os.environ.get("TOA_PS_HOSTS") else "allreduce"
    if mode == "ps":
        if rt.role != "ps":
            rt.info = None
        acc = run_ps(a, rt)
    else:
        if rt.role == "ps":  # PS replicas are idle in all-reduce mode
            rt.log("PS replica idle in all-reduce mode")
            while True:
                time.sleep(3600)
        rt.init_dist()
        acc = run_allreduce(a, rt)
    if acc is not None and acc < a.min_accuracy:
        rt.log(f"accuracy {acc:.3f} < required {a.min_accuracy}")
        sys.exit(1)


if __name__ == "__main__":
    main()
