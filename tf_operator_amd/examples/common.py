"""Shared bits of the bundled payloads."""
from __future__ import annotations

import os

import torch


def pick_device():
    if os.environ.get("TOA_NO_GPU") or os.environ.get("TOA_FORCE_CPU"):
        return torch.device("cpu")
    if not torch.cuda.is_available():
        return torch.device("cpu")
    from ..train.dist import local_device_index

    return torch.device("cuda", local_device_index() % max(torch.cuda.device_count(), 1))


def model_dtype(device):
    # bf16 compute on MI355X; the CPU reference path stays fp32
    return torch.bfloat16 if device.type == "cuda" else torch.float32
