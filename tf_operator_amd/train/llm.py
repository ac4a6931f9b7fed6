"""Data-parallel Llama trainer step (the flagship MI355X training path).

One process per GPU.  Per step: forward (fused HIP ops + the gfx950
assembly GEMMs and attention, ops/gemm.py, ops/llm.py),
backward writing weight gradients straight into the flat bf16 gradient
buffer, bucketed RCCL all-reduce overlapped with backward, one fused AdamW
over the flat fp32 master/m/v (device-side grad clipping, no host sync).

shard_optimizer=True (``TOA_ZERO=1``; bench.py's default for N > 1):
reduce-scatter instead of all-reduce, AdamW over this rank's shards only,
then an in-place all-gather of the bf16 weights that the next forward waits
for per bucket (parallel/zero.py).  The tail is pipelined (``TOA_ZERO_PIPE``,
default on): buckets are updated in forward-need order and each bucket's
all-gather is launched right after its shard's update, so the first gather
no longer waits for the whole update.
"""
from __future__ import annotations

import os
import time

import torch

from ..models.llama import PRESETS, Llama, LlamaConfig
from ..ops.optim import FlatAdamW
from ..ops.wt import TransposedWeights, enabled_default
from ..parallel.ddp import GradBucketer, broadcast_params
from ..parallel import zero
from ..parallel.flat import FlatParams
from ..parallel.zero import ParamGather


class LlamaTrainer:
    def __init__(self, cfg: LlamaConfig | str, device, micro_batch=1, seq_len=4096, grad_accum=1, lr=3e-4,
                 seed=0, bucket_mb=None, overlap_optimizer=None, shard_optimizer=None,
                 transposed_weights=None, force_collectives=False):
        if isinstance(cfg, str):
            cfg = PRESETS[cfg]
        self.cfg = cfg
        self.device = device
        self.micro_batch = micro_batch
        self.seq_len = seq_len
        self.grad_accum = grad_accum
        # GEMM policy: no stream-K kernels, so collectives can overlap the
        # GEMMs (ops/gemm.py).  Its plans resolve on a helper thread while
        # the weights initialise (~0.47 s of code-object loading that would
        # otherwise sit in the first step, profiles/r3_first).
        from ..ops import gemm as _gemm

        self.gemm_mode = _gemm.resolve_auto()
        self._gemm_prewarm = _gemm.prewarm(device) if torch.device(device).type == "cuda" else None
        with torch.device(device):
            model = Llama(cfg, device=device)
        model.init_weights(seed)
        self.model = model
        names = {id(p): n for n, p in model.named_parameters()}
        self.flat = FlatParams(model.params_backward_order(), names=names, no_decay=model.no_decay)
        self.wt = None
        if transposed_weights is None:
            transposed_weights = enabled_default(device)
        if transposed_weights:  # dgrad on W^T (ops/wt.py): +2 B/param of HBM
            lin = [p for n, p in model.named_parameters() if p.dim() == 2 and not n.startswith("embed.")]
            lin += [model.head_weight()]
            self.wt = TransposedWeights(self.flat, lin)
        broadcast_params(self.flat)
        if shard_optimizer is None:
            shard_optimizer = os.environ.get("TOA_ZERO", "0") == "1"
        # fresh gradients: no zeroing pass, each parameter's first producer of
        # a step overwrites its slice (FlatParams.mark_fresh, ops.grad.take_fresh)
        self.fresh_grads = os.environ.get("TOA_FRESH_GRADS", "1") != "0"
        # force_collectives: run the bucketed collectives even at world 1 (the
        # RCCL world-1 test drives the real reduce-scatter / all-gather path)
        self.bucketer = GradBucketer(self.flat, bucket_bytes=None if bucket_mb is None else int(bucket_mb * 2**20),
                                     shard=shard_optimizer, enabled=True if force_collectives else None)
        self.gather = None
        self.pipeline_tail = os.environ.get("TOA_ZERO_PIPE", "1") != "0"
        if self.bucketer.shard:  # ZeRO-1: reduce-scatter, owned-shard AdamW, in-place all-gather
            # fp32 master / m / v only for the owned shards: 12 B/param x (1 - 1/world) of HBM freed
            self.flat.shard_state(self.bucketer.owned)
            self.bucketer.pull_rs = self._pull_reduce()
            self.opt = FlatAdamW(self.flat, lr=lr, owned=self.bucketer.owned)
            self.gather = ParamGather(self.flat, self.bucketer.buckets, self.bucketer.rank, self.bucketer.world,
                                      on_gathered=self.wt.refresh if self.wt else None, emulator=self.bucketer.emu,
                                      pull=self._pull_gather())
        else:
            if overlap_optimizer is None:
                overlap_optimizer = os.environ.get("TOA_OPT_OVERLAP", "0") == "1"
            self.opt = FlatAdamW(self.flat, lr=lr, overlap=overlap_optimizer, buckets=self.bucketer.buckets,
                                 fuse_zero_grad=not self.fresh_grads,
                                 post_update=self.wt.refresh if self.wt else None)
            if self.wt is not None and os.environ.get("TOA_ADAM_WT", "1") != "0":
                # the update writes the W^T copies itself (ops/optim.py toa_adamw_wt)
                self.opt.fused_wt = self.wt
        self._fused_norm(model)
        if self.opt.overlap or self.gather is not None:
            self._hooks = self._install_param_waits()
        self._closed = False
        self._closed_registered = bool(self._pull_transports())
        if self._closed_registered:
            import atexit

            # registered after the process group's own atexit teardown
            # (train/dist.py init), so it runs BEFORE it (LIFO)
            atexit.register(self.close)
        self.step_idx = 0
        # start-up diagnostics: called with a phase name after the first
        # step's forward / backward / update are issued (host side; the
        # replica runtime's mark, examples/llama_train.py)
        self.on_phase = None

    def _fused_norm(self, model):
        """World 1, unsharded, clipping on, the assembly weight gradients:
        the clipping norm from the partials the weight-gradient kernels write
        (ops/gemm.SumsqSession) instead of a pass over the whole gradient.
        TOA_FUSED_NORM=0 turns it off."""
        from ..ops import _lib
        from ..ops import gemm as _g

        if (os.environ.get("TOA_FUSED_NORM", "1") == "0" or self.flat.device.type != "cuda"
                or not _lib.has("toa_wgrad_asm_set_sumsq") or self.gather is not None
                or self.bucketer.world != 1 or not self.opt.max_grad_norm):
            return
        head = model.head_weight()
        lin = [p for n, p in model.named_parameters() if p.dim() == 2 and not n.startswith("embed.")]
        if not any(head is p for p in lin) and not any(head is p for n, p in model.named_parameters()
                                                        if n.startswith("embed.")):
            lin.append(head)   # an untied head: its gradient has one producer, the weight-gradient GEMM
        sess = self._sumsq = _g.SumsqSession(self.flat, lin)
        self.opt.sumsq = sess
        _g._SESSIONS.add(sess)

    def _phase(self, name):
        if self.on_phase is not None and self.step_idx == 0:
            self.on_phase(name)

    def _wait_bucket(self, b):
        self.opt.wait_bucket(b)
        if self.gather is not None:
            self.gather.wait(b)

    def _install_param_waits(self):
        """Forward pre-hooks: each module waits only for the buckets holding
        its own parameters (FlatAdamW overlap mode; the sharded update's
        parameter all-gather).  The root's direct parameter (the untied
        lm_head) is used right after the final norm, so that wait rides on
        the final norm's hook instead of the root's."""
        hooks = []

        def waiter(buckets):
            def hook(mod, args):
                for b in buckets:
                    self._wait_bucket(b)
            return hook

        root_params = list(self.model.parameters(recurse=False))
        for name, mod in self.model.named_modules():
            ps = list(mod.parameters(recurse=False))
            if mod is self.model:
                continue
            if mod is self.model.norm:
                ps = ps + root_params
            if ps:
                bs = sorted({p._toa_bucket for p in ps})
                hooks.append(mod.register_forward_pre_hook(waiter(bs)))
        return hooks

    def synthetic_batch(self, seed=1234):
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        tok = torch.randint(0, self.cfg.vocab_size, (self.micro_batch, self.seq_len + 1), device=self.device,
                            generator=g)
        return tok[:, :-1].contiguous(), tok[:, 1:].contiguous()

    def step(self, batches):
        """batches: list (len grad_accum) of (tokens, targets)."""
        from ..ops import gemm as _gemm

        with _gemm.first_step(self.step_idx == 0):
            return self._step(batches)

    def _step(self, batches):
        if self.fresh_grads:
            self.flat.mark_fresh()
        elif not self.opt.grads_zeroed:
            self.flat.zero_grad()
        loss_sum = None
        for i, (tok, tgt) in enumerate(batches):
            loss = self.model(tok, tgt)
            self._phase("first_fwd_issued")
            self.opt.wait_all()  # backward writes gradients the update is still zeroing
            if self.gather is not None:
                self.gather.wait_all()  # backward reads every weight (and W^T)
            self.bucketer.armed = i == len(batches) - 1  # reduce once, after the last micro-batch
            (loss / len(batches)).backward()
            self._phase("first_bwd_issued")
            loss_sum = loss.detach() if loss_sum is None else loss_sum + loss.detach()
        if self.fresh_grads:
            self.flat.zero_stale()  # parameters no producer wrote this step
        self.bucketer.armed = True
        self.bucketer.finish()
        if self.gather is not None and self.pipeline_tail:
            # ZeRO-1 tail, bucket by bucket in forward-need order: each
            # bucket's all-gather starts as soon as its shard is updated
            self.opt.step(grad_scale=self.bucketer.grad_scale, bucket_order=self.gather.order(),
                          after_bucket=self.gather.launch_one, before_bucket=self._emulated_fused_reduce)
        else:
            self.opt.step(grad_scale=self.bucketer.grad_scale)
            if self.gather is not None:
                self.gather.launch()
        self._phase("first_update_issued")
        if self.gather is not None and self.gather.pull is not None:
            self.gather.pull.poll()   # a peer that never published surfaces one step later
        self.step_idx += 1
        return loss_sum / len(batches)

    def _pull_gather(self):
        """TOA_ZERO_AG=sdma on a one-node GPU job (every rank on this node):
        the weight all-gather as copy-engine pulls (parallel/pull_gather.py)."""
        from ..parallel import pull_gather

        bk = self.bucketer
        if pull_gather.mode_from_env() != "sdma" or bk.world < 2 or bk.emu is not None:
            return None
        return self._build_pull_gather()

    def _build_pull_gather(self):
        from ..parallel import pull_gather

        bk = self.bucketer
        if self.flat.param.device.type != "cuda" or int(os.environ.get("LOCAL_WORLD_SIZE", "0")) != bk.world:
            raise RuntimeError("TOA_ZERO_AG=sdma needs a GPU job whose ranks share one node "
                               "(LOCAL_WORLD_SIZE == world: the operator's node-local layout)")
        t = pull_gather.GpuIpcTransport(self.flat.param, bk.rank, bk.world, len(bk.buckets), group=bk.group,
                                        timeout_ms=pull_gather.timeout_ms_from_env())
        return pull_gather.PullGather(t, [(b[0], b[1]) for b in bk.buckets], bk.rank, bk.world)

    def _pull_reduce(self):
        """TOA_ZERO_RS=sdma on a one-node GPU job: the gradient
        reduce-scatter as copy-engine pulls plus an owner-side sum
        (parallel/pull_gather.PullReduceScatter)."""
        from ..parallel import pull_gather

        bk = self.bucketer
        if pull_gather.rs_mode_from_env() != "sdma" or bk.world < 2 or bk.emu is not None:
            return None
        return self._build_pull_reduce()

    def _build_pull_reduce(self):
        from ..parallel import pull_gather

        if not self.fresh_grads:
            # the zeroing pass at the start of step t+1 runs on the compute
            # stream before any wait, and nothing orders it after the owners'
            # pulls of this rank's step-t slices: an owner could sum zeroed
            # gradients.  Fresh gradients (the default) have no such pass --
            # the next backward's first write to a bucket comes after the
            # forward waited for that bucket's updated shard, i.e. after the pull.
            raise RuntimeError("TOA_ZERO_RS=sdma needs fresh gradients (TOA_FRESH_GRADS=1, the default)")
        bk = self.bucketer
        if (self.flat.grad.device.type != "cuda" or self.flat.grad.dtype != torch.bfloat16
                or int(os.environ.get("LOCAL_WORLD_SIZE", "0")) != bk.world):
            raise RuntimeError("TOA_ZERO_RS=sdma needs bf16 gradients on a GPU job whose ranks share one node "
                               "(LOCAL_WORLD_SIZE == world: the operator's node-local layout)")
        t = pull_gather.GpuIpcTransport(self.flat.grad, bk.rank, bk.world, len(bk.buckets), group=bk.group,
                                        what="reduce-scatter", timeout_ms=pull_gather.timeout_ms_from_env())
        return pull_gather.PullReduceScatter(t, [(b[0], b[1]) for b in bk.buckets], bk.rank, bk.world)

    # ---- ZeRO-1 collective transport, switchable between steps (bench A/B)
    def collective_transport(self) -> str | None:
        """"rccl" | "sdma" for a sharded trainer (both halves on the same
        transport), "mixed" when only one half pulls, None unsharded."""
        if self.gather is None:
            return None
        ag, rs = self.gather.pull is not None, self.bucketer.pull_rs is not None
        return "sdma" if ag and rs else ("rccl" if not (ag or rs) else "mixed")

    def set_collective_transport(self, kind: str):
        """Switch both ZeRO-1 collectives (the weight all-gather and the
        gradient reduce-scatter) to RCCL or to the copy-engine pulls between
        two steps.  Collective: every rank calls it at the same step.  The
        switch drains first -- every outstanding gather waited (and its W^T
        refresh run), the device synchronised, a barrier -- so no rank pulls
        across the boundary.  The pull transports are built once, on the
        first switch to "sdma", and kept (``close`` frees them)."""
        if self.gather is None:
            raise RuntimeError("collective transport: the trainer is not sharded (ZeRO-1 off)")
        if kind not in ("rccl", "sdma"):
            raise ValueError(kind)
        self.opt.wait_all()
        self.gather.wait_all()
        torch.cuda.synchronize()
        self._group_barrier()
        ag, rs = getattr(self, "_pulls", (None, None))
        ag, rs = ag or self.gather.pull, rs or self.bucketer.pull_rs
        if kind == "sdma":
            # built in the same order on every rank (both constructors are collective)
            ag = ag or self._build_pull_gather()
            rs = rs or self._build_pull_reduce()
            if not self._closed_registered:
                import atexit

                atexit.register(self.close)
                self._closed_registered = True
            self.gather.pull, self.bucketer.pull_rs = ag, rs
        else:
            self.gather.pull, self.bucketer.pull_rs = None, None
        self._pulls = (ag, rs)

    def _pull_transports(self):
        cur = [(self.gather.pull if self.gather is not None else None), getattr(self.bucketer, "pull_rs", None)]
        out = []
        for x in cur + list(getattr(self, "_pulls", ())):
            if x is not None and all(x is not y for y in out):
                out.append(x)
        return out

    def _group_barrier(self):
        import torch.distributed as dist

        group = self.bucketer.group
        if not dist.is_initialized():
            return
        if dist.get_backend(group) == "nccl":
            dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=group)
        torch.cuda.synchronize()

    def close(self, timeout_s: float = 60.0):
        """Orderly teardown of the copy-engine transports: this rank's pulls
        are drained and the device synchronised, then a barrier over the
        group (every peer has finished pulling from this rank's exported
        parameter / gradient / flag memory), and only then the IPC mappings
        are closed and the flag memory freed.  Idempotent; registered at
        exit.  After a failure (a peer may be gone) the barrier is bounded
        and the memory is left to process exit."""
        pulls = self._pull_transports()
        if self._closed or not pulls:
            return
        self._closed = True
        from . import dist as _dist

        try:
            self.opt.wait_all()
            if self.gather is not None:
                self.gather.wait_all()
            torch.cuda.synchronize()
        except Exception:  # noqa: BLE001 - a failed run still frees nothing a peer may read
            return
        if _dist._FAILED or _dist._EXIT_STATUS or not _dist._bounded(self._group_barrier, timeout_s):
            return
        for p in pulls:
            p.close()

    def _emulated_fused_reduce(self, b):
        """TOA_EMULATE_RS=sdma (parallel/emulate.py): price the reduction an
        AdamW summing the copy-engine-pulled gradient slices would do."""
        emu = self.bucketer.emu
        if emu is not None:
            lo, hi = self.gather.ranges[b]
            emu.fused_reduce(self.flat.grad[lo:hi])

    def tokens_per_step(self, world=1):
        return self.micro_batch * self.seq_len * self.grad_accum * world


def timed_steps(trainer: LlamaTrainer, batches, n, sync=True):
    t0 = time.perf_counter()
    loss = None
    for _ in range(n):
        loss = trainer.step(batches)
    if sync and torch.cuda.is_available():
        torch.cuda.synchronize()
    return time.perf_counter() - t0, loss


def rng_state(device) -> dict:
    """This process's CPU RNG state and, on a GPU, the device generator's
    (uint8 tensors)."""
    out = {"cpu": torch.get_rng_state()}
    if torch.device(device).type == "cuda":
        out["cuda"] = torch.cuda.get_rng_state(torch.device(device))
    return out


def set_rng_state(st: dict | None, device):
    if not st:
        return
    if st.get("cpu") is not None:
        torch.set_rng_state(st["cpu"].cpu().to(torch.uint8))
    if st.get("cuda") is not None and torch.device(device).type == "cuda":
        torch.cuda.set_rng_state(st["cuda"].cpu().to(torch.uint8), torch.device(device))


def trainer_state(tr: LlamaTrainer, data=None):
    """This rank's share of the training state: the fp32 master / moment
    shards it holds (all of them without ZeRO) plus where they belong in the
    flat buffer, the step, this rank's RNG states and (given the data
    stream) its cursor.  NOT a collective -- every rank saves its own share
    (train/sharded_ckpt.py), and the shares of any world size re-shard on
    load (:func:`load_trainer_state`)."""
    tr.opt.wait_all()
    if tr.gather is not None:
        tr.gather.wait_all()
    tr.bucketer.verify()  # never persist an update built from a failed one-shot all-reduce / pulled reduce-scatter
    if tr.gather is not None and tr.gather.pull is not None:
        tr.gather.pull.check()  # ... or from weights a copy-engine all-gather never completed
    return {"flat": tr.flat.state_dict(), "opt": tr.opt.state_dict(), "step": tr.step_idx,
            "rank": tr.bucketer.rank, "world": tr.bucketer.world, "rng": rng_state(tr.device),
            "data": data.state_dict() if data is not None else None}


def load_trainer_state(tr: LlamaTrainer, st, data=None):
    """Restore from one state (``trainer_state`` of an unsharded run) or a
    list of per-rank shares of any world size.  Collective when this
    trainer shards its optimizer: the restored weights are all-gathered.
    RNG states and the data cursor come from the share this rank saved
    (same rank index; rank 0's when the world grew)."""
    shards = st if isinstance(st, (list, tuple)) else [st]
    mine = next((s for s in shards if int(s.get("rank", 0)) == tr.bucketer.rank), shards[0])
    tr.opt.wait_all()
    if tr.gather is not None:
        tr.gather.wait_all()
    full = not tr.flat.state_sharded
    tr.flat.load_state_shards([s["flat"] for s in shards], set_params="all" if full else "held")
    if tr.gather is not None:  # held shards -> every rank's bf16 weights
        tr.gather.launch()
        tr.gather.wait_all()
    tr.flat.params_changed()
    tr.opt.load_state_dict(shards[0]["opt"])
    tr.step_idx = int(shards[0]["step"])
    set_rng_state(mine.get("rng"), tr.device)
    if data is not None and mine.get("data"):
        data.load_state_dict(mine["data"])
