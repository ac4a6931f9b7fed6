#!/usr/bin/env python3
"""Flagship benchmark: Llama-3-8B bf16 data-parallel training submitted as a
TFJob Worker=N on MI355X (BASELINE.json config #3, metric "samples/sec
(8-worker TFJob) + p50 submit->first-step latency at 1/2/4/8 GPUs").

    python bench.py --gpus N --steps K --warmup W          # through the operator
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   # one rank per GPU
    python bench.py --direct ...                            # no operator (profilers)

Rank 0 prints ONE JSON line: ``value`` = whole-job samples/sec (sequences of
``seq_len`` tokens), MAX step time over ranks, plus ``submit_to_first_step_p50_s``.
Implementation: :mod:`tf_operator_amd.bench.flagship`.
"""
from __future__ import annotations

import os
import sys
import time

T_PROC_START = time.time()

if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from tf_operator_amd.bench.flagship import main

    sys.exit(main(t_proc_start=T_PROC_START))
