"""Checkpoint / resume for the bundled trainers (SURVEY 5 "Checkpoint / resume").

The reference leaves this to the payload (Keras ModelCheckpoint on a PVC,
multi_worker_strategy-with-keras.py:92-109; TF Supervisor logdir,
dist_mnist.py:222-239).  Here it is a library used by every bundled trainer
and by the elastic restart path (SURVEY P9 / BASELINE config #5):

* rank 0 writes ``<dir>/step_<N>.pt`` (model/optimizer flat buffers, step,
  RNG state, user extras) to a temp file and atomically renames it, then
  atomically rewrites ``<dir>/latest``;
* because data-parallel replicas are identical, every rank (of ANY world
  size) resumes from the same file -- which is what lets an elastic job
  restart with fewer or more workers;
* old checkpoints beyond ``keep`` are pruned;
* loads use ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
import re
import tempfile
import time

import torch


def _tensors_to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().to("cpu")
    if isinstance(obj, dict):
        return {k: _tensors_to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_tensors_to_cpu(v) for v in obj)
    return obj


def save(ckpt_dir: str, step: int, state: dict, keep: int = 2) -> str:
    os.makedirs(ckpt_dir, exist_ok=True)
    payload = {"step": int(step), "time": time.time(), "state": _tensors_to_cpu(state),
               "rng_cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        payload["rng_cuda"] = torch.cuda.get_rng_state()
    path = os.path.join(ckpt_dir, f"step_{int(step):08d}.pt")
    fd, tmp = tempfile.mkstemp(dir=ckpt_dir, prefix=".tmp_ckpt_", suffix=".pt")
    with os.fdopen(fd, "wb") as f:
        torch.save(payload, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    fd, tmpl = tempfile.mkstemp(dir=ckpt_dir, prefix=".tmp_latest_")
    with os.fdopen(fd, "w") as f:
        f.write(os.path.basename(path))
    os.replace(tmpl, os.path.join(ckpt_dir, "latest"))
    _prune(ckpt_dir, keep)
    return path


def _prune(ckpt_dir, keep):
    files = sorted(f for f in os.listdir(ckpt_dir) if re.fullmatch(r"step_\d+\.pt", f))
    for f in files[:-keep] if keep > 0 else []:
        try:
            os.remove(os.path.join(ckpt_dir, f))
        except OSError:
            pass


def latest_path(ckpt_dir: str | None):
    if not ckpt_dir or not os.path.isdir(ckpt_dir):
        return None
    p = os.path.join(ckpt_dir, "latest")
    if os.path.exists(p):
        name = open(p).read().strip()
        full = os.path.join(ckpt_dir, name)
        if os.path.exists(full):
            return full
    files = sorted(f for f in os.listdir(ckpt_dir) if re.fullmatch(r"step_\d+\.pt", f))
    return os.path.join(ckpt_dir, files[-1]) if files else None


def load_latest(ckpt_dir: str | None, map_location="cpu"):
    p = latest_path(ckpt_dir)
    if p is None:
        return None
    payload = torch.load(p, map_location=map_location, weights_only=True)
    if "rng_cpu" in payload:
        torch.set_rng_state(payload["rng_cpu"])
    return payload
