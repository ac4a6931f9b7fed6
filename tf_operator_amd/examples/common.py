"""Shared bits of the bundled payloads."""
from __future__ import annotations

import os

import torch


def pick_device():
    if os.environ.get("TOA_NO_GPU") or os.environ.get("TOA_FORCE_CPU"):
        return torch.device("cpu")
    return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")


def model_dtype(device):
    # bf16 compute on MI355X; the CPU reference path stays fp32
    return torch.bfloat16 if device.type == "cuda" else torch.float32
