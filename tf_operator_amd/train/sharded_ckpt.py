"""Per-rank sharded, asynchronous checkpoints of the flat training state
(SURVEY 5 "checkpoint / resume"; BASELINE config #5: elastic TFJob with
checkpoint/restore on preemption).

The reference leaves checkpointing to the payload: every worker of the Keras
job runs ``ModelCheckpoint`` each epoch (``multi_worker_strategy-with-keras.py:108``).
At Llama-3-8B the training state is 112 GB (bf16 weights + fp32 master, m,
v); one rank pickling it synchronously cannot finish inside a pod's
termination grace period.  Here:

* **every rank saves its own share** -- the fp32 master / m / v ranges it
  holds (1/world of them under ZeRO-1, parallel/zero.py) -- as raw
  little-endian fp32 files, no pickle;
* **asynchronously**: :meth:`Checkpointer.save` enqueues device -> pinned host
  copies on the current stream (stream-ordered before the next optimizer
  step; ~50 GB/s) and returns; a background thread waits for them and
  writes + fsyncs the files.  The training loop only stalls for the copy;
* **atomically**: each rank's files land in ``step_N.partial/`` and end with
  a per-rank ``rank<r>.json`` marker; rank 0's writer waits for all
  markers, writes ``manifest.json``, renames the directory to ``step_N`` and
  rewrites ``latest`` -- a crash at any point leaves the previous step as
  ``latest``;
* **per attempt**: a marker names the save attempt that wrote it (an id
  every rank of one run shares: :meth:`Checkpointer.sync_attempt`, or the
  elastic generation / restart count from the environment), and rank 0
  commits only markers of ITS attempt whose byte counts match the files on
  disk.  A ``step_N.partial`` left by a crashed earlier attempt therefore
  never satisfies the wait: its markers name the old attempt, and every
  rank deletes its own stale marker before it rewrites its files;
* **RNG and data position**: each rank's marker also carries its CPU/GPU
  RNG states and data-stream cursor (``trainer_state``), so a resumed run
  continues the uninterrupted run's random and data sequence exactly;
* **re-sharding on load**: :func:`load_latest` returns every rank's share as
  read-only ``numpy.memmap`` views (nothing is unpickled), and
  ``FlatParams.load_state_shards`` copies the pieces intersecting this
  rank's ranges -- any world size can resume any other's checkpoint
  (the elastic policy's min/max replicas).

No collectives run in the background thread: the commit protocol is
file-based, so the save never races the training step's RCCL stream.
"""
from __future__ import annotations

import base64
import json
import os
import re
import shutil
import threading
import time

import numpy as np
import torch

STATE_KEYS = ("master", "exp_avg", "exp_avg_sq")
_STEP_RE = re.compile(r"step_(\d{8})")


def _step_dir(root: str, step: int, partial=False) -> str:
    return os.path.join(root, f"step_{int(step):08d}" + (".partial" if partial else ""))


def _atomic_write_text(path: str, text: str):
    tmp = f"{path}.tmp.{os.getpid()}.{threading.get_ident()}"
    with open(tmp, "w") as f:
        f.write(text)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def _fsync_dir(path: str):
    try:
        fd = os.open(path, os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def _env_attempt() -> str:
    """An attempt id all ranks of one launch agree on without talking:
    explicit TOA_CKPT_ATTEMPT, else the elastic generation / restart counts
    the operator (csrc/core/elastic.cc) and torchrun inject."""
    if os.environ.get("TOA_CKPT_ATTEMPT"):
        return os.environ["TOA_CKPT_ATTEMPT"]
    return "g{}.r{}.t{}".format(os.environ.get("TOA_ELASTIC_GENERATION", "0"),
                                os.environ.get("TOA_ELASTIC_RESTARTS", "0"),
                                os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))


def _b64(x) -> str | None:
    if x is None:
        return None
    if torch.is_tensor(x):
        x = x.cpu().numpy().tobytes()
    return base64.b64encode(bytes(x)).decode("ascii")


def _unb64(s) -> torch.Tensor | None:
    if s is None:
        return None
    return torch.frombuffer(bytearray(base64.b64decode(s)), dtype=torch.uint8).clone()


def _write_raw(path: str, arr: np.ndarray, chunk=1 << 28):
    with open(path, "wb", buffering=0) as f:
        mv = memoryview(arr.reshape(-1).view(np.uint8))
        for i in range(0, len(mv), chunk):  # file writes release the GIL
            f.write(mv[i:i + chunk])
        os.fsync(f.fileno())


class Checkpointer:
    """One per rank.  ``save()`` is cheap and asynchronous; ``wait()`` blocks
    until the last save is durable (and, on rank 0, committed)."""

    def __init__(self, root: str, rank: int = 0, world: int = 1, keep: int = 2, commit_timeout: float = 600.0,
                 io_threads: int = 3, attempt: str | None = None):
        self.root = root
        self.rank, self.world = int(rank), int(world)
        self.attempt = str(attempt) if attempt is not None else _env_attempt()
        self.keep = keep
        self.commit_timeout = commit_timeout
        self.io_threads = io_threads
        self._staging: dict[str, torch.Tensor] = {}
        self._thread: threading.Thread | None = None
        self._error: BaseException | None = None
        self._last_step: int | None = None
        self.last_timing: dict = {}
        os.makedirs(root, exist_ok=True)

    def sync_attempt(self, group=None) -> str:
        """Collective (call once at setup, every rank): adopt a fresh attempt
        id drawn by rank 0.  Covers restarts the environment does not count
        (a whole-group container restart under OnFailure)."""
        import torch.distributed as dist

        if dist.is_initialized() and dist.get_world_size(group) > 1:
            obj = [f"{self.attempt}.{os.urandom(6).hex()}" if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0, group=group)
            self.attempt = obj[0]
        else:
            self.attempt = f"{self.attempt}.{os.urandom(6).hex()}"
        return self.attempt

    # ------------------------------------------------------------------ staging
    def _stage(self, name: str, t: torch.Tensor) -> torch.Tensor:
        buf = self._staging.get(name)
        if buf is None or buf.numel() != t.numel() or buf.dtype != t.dtype:
            pin = t.is_cuda and torch.cuda.is_available()
            buf = torch.empty(t.numel(), dtype=t.dtype, pin_memory=pin)
            self._staging[name] = buf
        buf.copy_(t.detach().reshape(-1), non_blocking=t.is_cuda)
        return buf

    # ------------------------------------------------------------------ save
    def save(self, step: int, state: dict, extra: dict | None = None, block: bool = False):
        """`state` = ``train.llm.trainer_state`` (this rank's share).  A step
        this rank already saved is not written again (a periodic save that
        lands on the last step, then the final save): a second round of the
        same step directory could race rank 0's rename of the first and leave
        its commit waiting for a share written into the old directory."""
        self.wait()  # one save in flight: the staging buffers are reused
        if self._last_step == int(step):
            return
        self._last_step = int(step)
        t0 = time.time()
        fl = state["flat"]
        staged = {k: self._stage(k, fl[k]) for k in STATE_KEYS if fl.get(k) is not None}
        ev = None
        if any(fl[k].is_cuda for k in staged):
            ev = torch.cuda.Event()
            ev.record()
        meta = {"rank": self.rank, "world": self.world, "step": int(step),
                "state_ranges": [list(map(int, r)) for r in fl["state_ranges"]], "numel": int(fl["numel"]),
                "layout": [list(x) for x in fl["layout"]], "opt": state.get("opt") or {},
                "dtype": {k: "float32" for k in staged}, "extra": extra or {}, "attempt": self.attempt,
                "rng": {k: _b64(v) for k, v in (state.get("rng") or {}).items()}, "data": state.get("data")}
        self._error = None
        self._thread = threading.Thread(target=self._write, args=(int(step), staged, ev, meta, t0),
                                        name=f"ckpt-writer-{self.rank}", daemon=True)
        self._thread.start()
        if block:
            self.wait()

    def _write(self, step, staged, ev, meta, t0):
        try:
            if ev is not None:
                ev.synchronize()
            t_staged = time.time()
            d = _step_dir(self.root, step, partial=True)
            os.makedirs(d, exist_ok=True)
            # a crashed earlier attempt's marker must go BEFORE this rank's
            # files are rewritten (its attempt id already keeps rank 0 from
            # committing it; this keeps the directory honest too)
            marker = os.path.join(d, f"rank{self.rank:05d}.json")
            if os.path.exists(marker):
                os.remove(marker)
            files = {}
            threads = []
            for k, buf in staged.items():
                fn = f"rank{self.rank:05d}.{k}.f32"
                files[k] = fn
                arr = buf.numpy()
                th = threading.Thread(target=_write_raw, args=(os.path.join(d, fn), arr))
                th.start()
                threads.append(th)
            for th in threads:
                th.join()
            meta["files"] = files
            meta["bytes"] = int(sum(b.numel() * b.element_size() for b in staged.values()))
            _atomic_write_text(marker, json.dumps(meta))
            t_written = time.time()
            if self.rank == 0:
                self._commit(step, d, meta)
            self.last_timing = {"stage_s": round(t_staged - t0, 3), "write_s": round(t_written - t_staged, 3),
                                "total_s": round(time.time() - t0, 3), "bytes": meta["bytes"],
                                "write_GBps": round(meta["bytes"] / max(t_written - t_staged, 1e-9) / 1e9, 2)}
        except BaseException as e:  # surfaced by wait()
            self._error = e

    def _marker_ok(self, d, path):
        """A rank's marker counts only if it is this attempt's and every file
        it names is on disk at the size it records."""
        try:
            with open(path) as f:
                m = json.load(f)
        except (OSError, ValueError):
            return None
        if m.get("attempt") != self.attempt:
            return None
        n = sum(hi - lo for lo, hi in m["state_ranges"])
        for fn in m.get("files", {}).values():
            try:
                if os.path.getsize(os.path.join(d, fn)) != 4 * n:
                    return None
            except OSError:
                return None
        return m

    def _commit(self, step, d, meta0):
        deadline = time.monotonic() + self.commit_timeout
        want = [os.path.join(d, f"rank{r:05d}.json") for r in range(self.world)]
        got = [None] * self.world
        while True:
            for r, p in enumerate(want):
                if got[r] is None and os.path.exists(p):
                    got[r] = self._marker_ok(d, p)
            if all(m is not None for m in got):
                break
            if time.monotonic() > deadline:
                raise TimeoutError(f"checkpoint step {step}: not every rank finished its share "
                                   f"(attempt {self.attempt})")
            time.sleep(0.05)
        shards = []
        for m in got:
            shards.append({"rank": m["rank"], "state_ranges": m["state_ranges"], "files": m["files"],
                           "bytes": m["bytes"], "rng": m.get("rng") or {}, "data": m.get("data")})
        manifest = {"format": "toa-sharded-v1", "step": step, "attempt": self.attempt, "world": self.world,
                    "numel": meta0["numel"],
                    "layout": meta0["layout"], "opt": meta0["opt"], "extra": meta0["extra"], "time": time.time(),
                    "shards": shards}
        _atomic_write_text(os.path.join(d, "manifest.json"), json.dumps(manifest))
        _fsync_dir(d)
        final = _step_dir(self.root, step)
        if os.path.exists(final):
            shutil.rmtree(final)
        os.replace(d, final)
        _fsync_dir(self.root)
        _atomic_write_text(os.path.join(self.root, "latest"), os.path.basename(final))
        self._prune()

    def _prune(self):
        steps = sorted(n for n in os.listdir(self.root) if _STEP_RE.fullmatch(n))
        for n in steps[:-self.keep] if self.keep > 0 else []:
            shutil.rmtree(os.path.join(self.root, n), ignore_errors=True)
        # stale partial directories of steps older than the newest commit
        newest = int(steps[-1][5:]) if steps else -1
        for n in os.listdir(self.root):
            m = re.fullmatch(r"step_(\d{8})\.partial", n)
            if m and int(m.group(1)) < newest:
                shutil.rmtree(os.path.join(self.root, n), ignore_errors=True)

    def wait(self):
        th = self._thread
        if th is not None:
            th.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise RuntimeError(f"checkpoint write failed on rank {self.rank}") from e

    @property
    def busy(self) -> bool:
        return self._thread is not None and self._thread.is_alive()


def latest_dir(root: str | None) -> str | None:
    if not root or not os.path.isdir(root):
        return None
    p = os.path.join(root, "latest")
    if os.path.exists(p):
        with open(p) as f:
            d = os.path.join(root, f.read().strip())
        if os.path.exists(os.path.join(d, "manifest.json")):
            return d
    steps = sorted(n for n in os.listdir(root) if _STEP_RE.fullmatch(n)
                   and os.path.exists(os.path.join(root, n, "manifest.json")))
    return os.path.join(root, steps[-1]) if steps else None


def load_latest(root: str | None):
    """[share, ...] of the newest committed step (every saving rank's share,
    tensors as read-only memmaps) or None.  Feed to ``load_trainer_state``."""
    d = latest_dir(root)
    if d is None:
        return None
    with open(os.path.join(d, "manifest.json")) as f:
        man = json.load(f)
    out = []
    for sh in man["shards"]:
        n = sum(hi - lo for lo, hi in sh["state_ranges"])
        flat = {"state_ranges": [tuple(r) for r in sh["state_ranges"]], "numel": man["numel"],
                "layout": man["layout"]}
        for k, fn in sh["files"].items():
            arr = np.memmap(os.path.join(d, fn), dtype=np.float32, mode="r")
            if arr.shape[0] != n:
                raise ValueError(f"{fn}: {arr.shape[0]} elements, manifest says {n}")
            flat[k] = arr
        out.append({"flat": flat, "opt": man["opt"], "step": man["step"], "rank": sh["rank"],
                    "world": man["world"], "extra": man.get("extra", {}),
                    "rng": {k: _unb64(v) for k, v in (sh.get("rng") or {}).items() if v is not None},
                    "data": sh.get("data")})
    return out
