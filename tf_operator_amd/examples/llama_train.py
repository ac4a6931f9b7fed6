"""Llama-family DP training payload (BASELINE configs #3 / #4 / #5):
TFJob/PyTorchJob Worker=N, one GPU per worker, RCCL over xGMI, fused HIP
kernels, AdamW -- the same step as bench.py (ZeRO-1 sharded optimizer for
N > 1 unless ``--zero 0``).  Every rank checkpoints its own optimizer shard
(train/sharded_ckpt.py, asynchronous) every `--checkpoint-every` steps and
on SIGTERM (preemption; the ranks agree on the stop step first) to
TOA_CHECKPOINT_DIR, and resumes from it on restart -- with ANY world size,
which is what the elastic policy relies on."""
from __future__ import annotations

import argparse
import os
import time

import torch

from tf_operator_amd.examples.common import pick_device
from tf_operator_amd.train import dist as tdist
from tf_operator_amd.train import sharded_ckpt
from tf_operator_amd.train.data import SyntheticTokens
from tf_operator_amd.train.llm import LlamaTrainer, load_trainer_state, trainer_state
from tf_operator_amd.train.runtime import Runtime


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama-tiny")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--seq-len", type=int, default=128)
    p.add_argument("--micro-batch", type=int, default=2)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--checkpoint-every", type=int, default=0)
    p.add_argument("--step-sleep", type=float, default=0.0, help="testing: slow steps down")
    p.add_argument("--report-every", type=int, default=0, help="report samples/sec to the operator every N steps")
    p.add_argument("--fixed-batch", action="store_true", help="reuse one resident batch (benchmarking)")
    p.add_argument("--zero", choices=("auto", "0", "1"), default="auto",
                   help="ZeRO-1 sharded optimizer; auto = on for world > 1 (bench.py's default)")
    a = p.parse_args(argv)
    from tf_operator_amd.ops import gemm

    gemm.prewarm_early()  # GEMM plans resolve while the process group and the model come up
    rt = Runtime()
    rt.install_preemption_handler()
    info = rt.init_dist()
    rt.mark("dist_init")
    with rt.guard():
        _train(a, rt, info)


def _stop_agreed(rt, dev) -> bool:
    """True on every rank once ANY rank got SIGTERM (a MAX all-reduce of the
    flag), so all ranks stop -- and save -- after the same step."""
    flag = rt.preempted.is_set()
    if rt.world == 1 or not torch.distributed.is_initialized():
        return flag
    t = torch.tensor([1.0 if flag else 0.0], device=dev)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return bool(t.item() > 0)


def _train(a, rt, info):
    # gloo is the CPU plumbing backend, unless asked for explicitly
    # (TOA_DIST_BACKEND=gloo: replicas sharing one GPU, device tensors over gloo)
    dev = pick_device() if info.backend != "gloo" or os.environ.get("TOA_DIST_BACKEND") else torch.device("cpu")
    zero = rt.world > 1 if a.zero == "auto" else a.zero == "1"
    tr = LlamaTrainer(a.model, dev, micro_batch=a.micro_batch, seq_len=a.seq_len, lr=a.lr, shard_optimizer=zero)
    rt.mark("model_init")
    tr.on_phase = rt.mark  # the first step's host-side issue points, in the start-up phases
    ck = sharded_ckpt.Checkpointer(rt.ckpt_dir, rt.rank, rt.world) if rt.ckpt_dir else None
    if ck is not None:
        ck.sync_attempt()  # markers of a crashed earlier attempt never commit this run's saves
    # a resumable stream: batch i of rank r is a function of (seed, r, i), so
    # the checkpointed cursor continues the uninterrupted run's data exactly
    data = SyntheticTokens(a.micro_batch, a.seq_len, tr.cfg.vocab_size, rank=rt.rank, device=dev,
                           fixed=a.fixed_batch)
    shares = sharded_ckpt.load_latest(rt.ckpt_dir)
    if shares is not None:
        load_trainer_state(tr, shares, data=data)  # re-shards a checkpoint of any world size
        rt.log(f"resumed at step {tr.step_idx} (world {rt.world}) from a world-{shares[0]['world']} checkpoint"
               f" at data cursor {data.cursor}")
        rt.mark("checkpoint_load")
    t0, n0 = time.perf_counter(), tr.step_idx
    while tr.step_idx < a.steps:
        loss = tr.step([data.next()])
        if tr.step_idx == n0 + 1:
            if dev.type == "cuda":
                torch.cuda.synchronize()
            rt.first_step_done()
            t1 = time.perf_counter()
        if tr.step_idx % 5 == 0 or tr.step_idx == a.steps:
            rt.log(f"step {tr.step_idx} loss {float(loss):.4f}")
        if a.report_every and (tr.step_idx - n0) % a.report_every == 0 and tr.step_idx > n0 + 1:
            # throughput since the first step of this generation (excludes start-up)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            el = time.perf_counter() - t1
            rt.report(samples_per_sec=a.micro_batch * rt.world * (tr.step_idx - n0 - 1) / max(el, 1e-9),
                      step=tr.step_idx, world=rt.world)
        if ck and a.checkpoint_every and tr.step_idx % a.checkpoint_every == 0:
            ck.save(tr.step_idx, trainer_state(tr, data))  # every rank, its own shard; asynchronous
        if _stop_agreed(rt, dev):
            if ck:
                t_s = time.time()
                ck.save(tr.step_idx, trainer_state(tr, data), block=True)
                rt.log(f"preemption checkpoint at step {tr.step_idx} in {time.time() - t_s:.2f}s "
                       f"{ck.last_timing}")
            rt.log(f"preempted at step {tr.step_idx}")
            tdist.shutdown()
            raise SystemExit(143)
        if a.step_sleep:
            time.sleep(a.step_sleep)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    done = tr.step_idx - n0
    if done:
        rt.report(samples_per_sec=a.micro_batch * rt.world * done / dt)
    if ck:
        ck.save(tr.step_idx, trainer_state(tr, data), block=True)
    rt.log(f"done: {tr.step_idx} steps")


if __name__ == "__main__":
    main()
