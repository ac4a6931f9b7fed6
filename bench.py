#!/usr/bin/env python3
"""Flagship benchmark: data-parallel Llama-3-8B bf16 training step on MI355X.

BASELINE.json config #3 -- "TFJob Worker=8 all-reduce Llama-3-8B bf16, RCCL
ring over xGMI, 1 GPU/worker" -- metric "samples/sec (8-worker TFJob)".
One process per GPU (torchrun or the operator's TFJob env contract), weak
scaling (fixed per-GPU micro-batch), synthetic tokens, random-init weights.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  `value` = whole-job samples/sec (sequences of
`seq_len` tokens), MAX step time over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_PROC_START = time.time()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=6)  # 228 GB peak of 288 GB; 2 % over mb4
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--zero", choices=("auto", "0", "1"), default="auto",
                    help="sharded optimizer (reduce-scatter / owned-shard AdamW / all-gather); auto = on for N > 1")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.cuda profiler markers")
    args = ap.parse_args()

    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from tf_operator_amd.train import dist as tdist
    from tf_operator_amd.train.llm import LlamaTrainer

    info = tdist.init()
    n_gpus = info.world
    if args.gpus != n_gpus and info.rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={n_gpus}; using WORLD_SIZE", file=sys.stderr)
    dev = info.device
    torch.manual_seed(0)
    zero = n_gpus > 1 if args.zero == "auto" else args.zero == "1"
    tr = LlamaTrainer(args.model, dev, micro_batch=args.micro_batch, seq_len=args.seq_len,
                      grad_accum=args.grad_accum, bucket_mb=args.bucket_mb, shard_optimizer=zero)
    batches = [tr.synthetic_batch(seed=1000 + info.rank * 97 + i) for i in range(args.grad_accum)]

    # first step (submit -> first-step proxy inside the replica: process start -> step 1 done)
    loss = tr.step(batches)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    first_step_s = time.time() - T_PROC_START
    for _ in range(max(args.warmup - 1, 0)):
        loss = tr.step(batches)
    tdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = tr.step(batches)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    tdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt = tdist.all_max(dt, dev)
    loss_v = float(loss)
    ms = dt / args.steps * 1e3
    global_batch = args.micro_batch * args.grad_accum * n_gpus
    samples_s = global_batch * args.steps / dt
    tokens_s = samples_s * args.seq_len
    cfg = tr.cfg
    flops = cfg.flops_per_token(args.seq_len) * tokens_s
    peak_mem = torch.cuda.max_memory_allocated(dev) / 2**30 if dev.type == "cuda" else 0.0

    if info.rank == 0:
        out = {
            "metric": "samples/sec (8-worker TFJob)",
            "value": round(samples_s, 4),
            "unit": "samples/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {
                "model": "Llama-3-8B" if args.model == "llama3-8b" else args.model,
                "global_batch": global_batch,
                "seq_len": args.seq_len,
                "parallelism": f"dp{n_gpus}",
                "micro_batch_per_gpu": args.micro_batch,
                "grad_accum": args.grad_accum,
                "optimizer": "AdamW (fused HIP, fp32 master, clip 1.0)"
                             + (", ZeRO-1 sharded" if tr.bucketer.shard else ""),
                "tfjob": f"Worker={n_gpus}",
                "weights": "random-init",
            },
            "tokens_per_sec": round(tokens_s, 1),
            "model_tflops_per_gpu": round(flops / n_gpus / 1e12, 1),
            "first_step_s": round(first_step_s, 2),
            "loss": round(loss_v, 4),
            "peak_mem_gib": round(peak_mem, 1),
        }
        print(json.dumps(out), flush=True)
    tdist.shutdown()


if __name__ == "__main__":
    main()
