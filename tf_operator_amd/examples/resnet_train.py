"""ResNet-50 synthetic-ImageNet payload (BASELINE config #2: TFJob PS=1
Worker=2, each replica on 1x MI355X).

With PS replicas in the TFJob (``TOA_PS_HOSTS``) the servers own the
parameters and the optimizer (reference: dist_mnist.py:149-219,
replica_device_setter + SyncReplicasOptimizer): workers run forward +
backward (bf16 channels-last convs through MIOpen, fused HIP dense head),
reduce their gradients onto the servers bucket by bucket during backward
(``--ps-mode sync``, replicas_to_aggregate = workers) or push them as they
finish (``async``), and receive the servers' new weights; the servers run
the fused HIP AdamW on their fp32 shards (parallel/ps_collective.py, RCCL
over xGMI).  Without PS replicas (or ``--ps-mode none``) the workers
all-reduce among themselves.  Reports samples/sec to the operator."""
from __future__ import annotations

import argparse
import os
import time

import torch

from tf_operator_amd.examples.common import model_dtype, pick_device, use_shipped_miopen_find_db
from tf_operator_amd.models.vision import ResNet, resnet50
from tf_operator_amd.ops.llm import cross_entropy
from tf_operator_amd.parallel import ps_collective
from tf_operator_amd.train import simple
from tf_operator_amd.train.data import SyntheticImages
from tf_operator_amd.train.runtime import Runtime


def build(arch, dt_, dev, classes):
    if arch == "resnet50":
        m = resnet50(num_classes=classes, dtype=dt_, device=dev)
    elif arch == "resnet-tiny":  # CI plumbing: one bottleneck per stage
        m = ResNet(layers=(1, 1, 1, 1), num_classes=classes, dtype=dt_, device=dev)
    else:
        raise SystemExit(f"unknown --arch {arch}")
    return m.to(memory_format=torch.channels_last)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--image", type=int, default=224)
    p.add_argument("--arch", default="resnet50", choices=("resnet50", "resnet-tiny"))
    p.add_argument("--classes", type=int, default=1000)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--clip", type=float, default=0.0,
                   help="global gradient-norm clipping (device-side, in the fused AdamW); 0 = off")
    p.add_argument("--fixed-labels", action="store_true",
                   help="one fixed batch (the model memorises it; see train/data.SyntheticImages)")
    p.add_argument("--ps-mode", default="auto", choices=("auto", "sync", "async", "none"),
                   help="auto = sync when the job has PS replicas")
    a = p.parse_args(argv)
    use_shipped_miopen_find_db()
    rt = Runtime()
    workers, servers, role, idx = ps_collective.ps_world_env()
    mode = a.ps_mode if a.ps_mode != "auto" else ("sync" if servers else "none")
    if mode != "none" and not servers:
        raise SystemExit(f"--ps-mode {mode} needs PS replicas (TOA_PS_HOSTS)")
    if mode == "none" and role == "ps":  # all-reduce mode: the PS replica has nothing to do
        while True:
            time.sleep(3600)
    if mode != "none":
        ps_collective.join_ps_world(workers, servers, role, idx)
    info = rt.init_dist()
    if mode != "none":
        owner = "operator" if os.environ.get("TOA_PS_IN_WORLD") == "1" else "payload"
        rt.log(f"ps world ({owner}): {workers} trainers + {servers} servers, rank {info.rank} of {info.world}")
    dev = pick_device() if info.backend != "gloo" else torch.device("cpu")
    dt_ = model_dtype(dev)
    torch.manual_seed(0)
    model = build(a.arch, dt_, dev, a.classes)
    loss_fn = lambda o, y: cross_entropy(o.float(), y)  # noqa: E731
    total = a.warmup + a.steps
    if mode != "none" and role == "ps":
        ps = simple.parameter_server(model, workers, servers, mode=mode, lr=a.lr)
        t0 = time.perf_counter()
        ps.serve(total)
        rt.log(f"ps {idx}: {ps.updates} {mode} updates of {ps.ranges[ps.p][1] - ps.ranges[ps.p][0]} parameters "
               f"in {time.perf_counter() - t0:.2f}s")
        return
    if mode != "none":
        tr = simple.PSTrainer(model, loss_fn, rt, workers, servers, mode=mode, lr=a.lr)
    else:
        tr = simple.DPTrainer(model, loss_fn, rt, lr=a.lr, bucket_mb=64, max_grad_norm=a.clip)
    data = SyntheticImages(a.batch, (3, a.image, a.image), classes=a.classes, rank=rt.rank, device=dev, dtype=dt_,
                           fresh_labels=not a.fixed_labels)
    for _ in range(a.warmup):
        tr.step(*data.next())
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = None
    for i in range(a.steps):
        loss, _ = tr.step(*data.next())
        if (i + 1) % 10 == 0 or i + 1 == a.steps:
            rt.log(f"step {a.warmup + i + 1} loss {float(loss):.4f}")
    if hasattr(tr, "sync_params"):
        # sync PS: the last step's parameter pulls are part of the step (gloo
        # work is not covered by cuda.synchronize), so they end inside the clock
        tr.sync_params()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sps = a.batch * workers * a.steps / dt
    rt.report(samples_per_sec=sps)
    rt.log(f"{a.arch} [{mode if mode != 'none' else 'all-reduce'}] {sps:.1f} samples/s "
           f"({dt / a.steps * 1e3:.1f} ms/step, loss {float(loss):.3f})")


if __name__ == "__main__":
    main()
