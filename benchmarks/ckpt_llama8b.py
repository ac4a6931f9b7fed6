"""Checkpoint save / load / time-to-resume of the full Llama-3-8B training
state on one MI355X (BASELINE config #5; SURVEY 5 "checkpoint / resume").

The state is this rank's fp32 master + AdamW m + v (12 B/param, 96 GB at
world 1), written by ``train/sharded_ckpt.Checkpointer``:

* ``stall_s``   -- how long the training loop is blocked: ``save()`` enqueues
  the device -> pinned-host copies and returns; the next optimizer step is
  stream-ordered after them, so the stall is the D2H copy time;
* ``write_s``   -- the background writer (raw fp32 files + fsync + manifest
  commit), overlapped with training steps that we time meanwhile;
* ``load_s``    -- ``load_latest`` (memmaps, nothing unpickled) +
  ``load_trainer_state`` (host -> device copies into the held ranges);
* ``resume_s``  -- load + first training step after it.

The restored master/m/v are checked bit-exactly against what was saved.

    python benchmarks/ckpt_llama8b.py [--model llama3-8b] [--dir /tmp/x]

Writes one JSON line.  Needs ~1.1x the state size free on ``--dir``;
otherwise it says so and exits 0 (nothing measured).  The MI355X boxes here
have a 79 GB root disk, so the recorded run targets tmpfs (``/dev/shm``):
it prices the staging / writer / commit pipeline, and a real volume adds
its own write bandwidth on top (``write_GBps`` is what the pipeline
sustained).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--dir", default=None, help="checkpoint root (default: a fresh dir under $TMPDIR)")
    ap.add_argument("--overlap-steps", type=int, default=3, help="training steps timed while the writer runs")
    a = ap.parse_args()

    import torch

    from tf_operator_amd.train import sharded_ckpt
    from tf_operator_amd.train.llm import LlamaTrainer, load_trainer_state, trainer_state

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.time()
    tr = LlamaTrainer(a.model, dev, micro_batch=a.micro_batch, seq_len=a.seq_len)
    batch = [tr.synthetic_batch()]
    tr.step(batch)
    torch.cuda.synchronize()
    base_ms = []
    for _ in range(2):
        t = time.perf_counter()
        tr.step(batch)
        torch.cuda.synchronize()
        base_ms.append((time.perf_counter() - t) * 1e3)
    st = trainer_state(tr)
    fl = st["flat"]
    nbytes = sum(fl[k].numel() * fl[k].element_size() for k in sharded_ckpt.STATE_KEYS if fl.get(k) is not None)
    root = a.dir or tempfile.mkdtemp(prefix="toa-ckpt8b-")
    os.makedirs(root, exist_ok=True)
    free = shutil.disk_usage(root).free
    out = {"metric": "checkpoint save/load of the full training state", "model": a.model,
           "state_bytes": nbytes, "dir": root, "dir_free_bytes": free, "init_s": round(time.time() - t0, 2),
           "step_ms_baseline": [round(x, 1) for x in base_ms]}
    if free < 1.1 * nbytes:
        out["skipped"] = f"only {free / 1e9:.1f} GB free on {root}, need {1.1 * nbytes / 1e9:.1f}"
        print(json.dumps(out), flush=True)
        return 0
    # reference copies of a few slices to check the restore bit-exactly
    probes = {}
    for k in sharded_ckpt.STATE_KEYS:
        t = fl[k]
        n = t.numel()
        probes[k] = [(i, t.reshape(-1)[i:i + 4096].clone()) for i in (0, n // 3, n - 4096)]

    try:
        return _measure(tr, batch, st, fl, probes, root, nbytes, out, a)
    finally:
        shutil.rmtree(root, ignore_errors=True)


def _measure(tr, batch, st, fl, probes, root, nbytes, out, a):
    import torch

    from tf_operator_amd.train import sharded_ckpt
    from tf_operator_amd.train.llm import load_trainer_state, trainer_state

    ck = sharded_ckpt.Checkpointer(root, 0, 1, keep=1)
    # first save allocates (and pins) the staging buffers: time it apart
    t = time.perf_counter()
    ck.save(tr.step_idx, st)
    t_ret = time.perf_counter() - t
    torch.cuda.synchronize()
    out["first_save_stall_s"] = round(time.perf_counter() - t, 3)
    out["first_save_return_s"] = round(t_ret, 3)
    ck.wait()
    out["first_save"] = dict(ck.last_timing)
    print(f"[ckpt] first save {out['first_save']}", flush=True)
    # host RAM: pinned staging (1x state) + a tmpfs target must not hold two
    # committed copies at once
    for n in os.listdir(root):
        if n.startswith("step_"):
            shutil.rmtree(os.path.join(root, n), ignore_errors=True)

    # steady-state save: stall + overlapped training steps + write
    tr.step(batch)
    st = trainer_state(tr)
    for k in sharded_ckpt.STATE_KEYS:  # re-snapshot the probes at the saved step
        t = st["flat"][k].reshape(-1)
        probes[k] = [(i, t[i:i + 4096].clone()) for i, _ in probes[k]]
    saved_step = tr.step_idx
    torch.cuda.synchronize()
    t = time.perf_counter()
    ck.save(saved_step, st)
    torch.cuda.synchronize()
    out["stall_s"] = round(time.perf_counter() - t, 3)
    ov = []
    for _ in range(a.overlap_steps):
        if not ck.busy:
            break
        ts = time.perf_counter()
        tr.step(batch)
        torch.cuda.synchronize()
        ov.append((time.perf_counter() - ts) * 1e3)
    ck.wait()
    out["save"] = dict(ck.last_timing)
    out["step_ms_during_write"] = [round(x, 1) for x in ov]
    print(f"[ckpt] steady save {out['save']} stall {out['stall_s']}s", flush=True)

    # load: clobber the state, restore, check, then one step (= time to resume)
    for k in sharded_ckpt.STATE_KEYS:
        tr.flat.state_dict()[k].zero_()
    torch.cuda.synchronize()
    t = time.perf_counter()
    shares = sharded_ckpt.load_latest(root)
    load_trainer_state(tr, shares)
    torch.cuda.synchronize()
    out["load_s"] = round(time.perf_counter() - t, 3)
    out["load_GBps"] = round(nbytes / max(out["load_s"], 1e-9) / 1e9, 2)
    ok = True
    now = tr.flat.state_dict()
    for k in sharded_ckpt.STATE_KEYS:
        t = now[k].reshape(-1)
        for i, ref in probes[k]:
            ok &= bool(torch.equal(t[i:i + 4096], ref))
    out["restored_bit_exact"] = ok
    tr.step_idx = shares[0]["step"]
    t2 = time.perf_counter()
    loss = float(tr.step(batch))
    torch.cuda.synchronize()
    out["first_step_after_load_s"] = round(time.perf_counter() - t2, 3)
    out["resume_s"] = round(out["load_s"] + out["first_step_after_load_s"], 3)
    out["loss_after_resume"] = round(loss, 4)
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
