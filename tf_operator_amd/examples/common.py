"""Shared bits of the bundled payloads."""
from __future__ import annotations

import glob
import os
import shutil
import tempfile

import torch

MIOPEN_DB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "miopen_db")


def use_shipped_miopen_find_db() -> str | None:
    """Point MIOpen at the find-db recorded on an MI355X for the payloads'
    convolution shapes (``examples/miopen_db``), unless the user set one.

    Without it every fresh pod runs MIOpen's exhaustive find on its first
    step (64.7 s before the ResNet-50 payload's first step vs 0.8 s with the
    db, profiles/r2_resnet/find_db.log), and the timing-based choice varies
    from box to box (the same payload measured 4.6k-7.3k samples/s).  The
    db is copied to a per-user temp dir because MIOpen updates it in place;
    a file whose MIOpen version does not match is simply not used.  Call
    before the first convolution."""
    if os.environ.get("MIOPEN_USER_DB_PATH"):
        return None
    src = glob.glob(os.path.join(MIOPEN_DB, "*.ufdb.txt"))
    if not src:
        return None
    dst = os.path.join(tempfile.gettempdir(), f"toa-miopen-db-{os.getuid()}")
    os.makedirs(dst, exist_ok=True)
    for f in src:
        out = os.path.join(dst, os.path.basename(f))
        if not os.path.exists(out):
            # atomic: the replicas of one node start together, and MIOpen must
            # never read a half-copied db (an existing copy is kept: MIOpen
            # appends what it finds for other shapes to it)
            tmp = f"{out}.{os.getpid()}.tmp"
            shutil.copyfile(f, tmp)
            os.replace(tmp, out)
    os.environ["MIOPEN_USER_DB_PATH"] = dst
    return dst


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
