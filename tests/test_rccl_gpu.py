"""The RCCL (``nccl`` backend) data-parallel path on a real MI355X at world 1.

The 8-GPU run is the driver's; what can be proven on one GPU is that the
collectives the trainer issues work on RCCL exactly as on gloo:
* ZeRO-1 (parallel/zero.py): in-place ``reduce_scatter_tensor`` on slices
  of the flat gradient buffer fired from backward hooks, an owned-shard
  AdamW over COMPACT fp32 state, in-place ``all_gather_into_tensor`` of the
  bf16 weights waited for per bucket by forward pre-hooks;
* plain DP: bucketed async ``all_reduce``.
At world 1 both are identities: the all-reduce trainer must match the
trainer with no collectives bit for bit; the sharded one sums the clipping
norm per owned range (a different fp32 summation order), so it matches to
rounding."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    try:
        from tf_operator_amd.train.llm import LlamaTrainer

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
        res = {}
        for name, kw in (("none", {}), ("zero", dict(shard_optimizer=True, force_collectives=True)),
                         ("allreduce", dict(shard_optimizer=False, force_collectives=True))):
            tr = LlamaTrainer("llama-tiny", dev, micro_batch=2, seq_len=128, lr=1e-3, bucket_mb=0.25, **kw)
            if name == "zero":
                assert tr.bucketer.shard and tr.gather is not None and len(tr.bucketer.buckets) > 2
                assert tr.flat.state_ranges == [tuple(r) for r in tr.bucketer.owned]
            if name == "allreduce":
                assert tr.bucketer.enabled and not tr.bucketer.shard
            b = tr.synthetic_batch()
            losses = [float(tr.step([b])) for _ in range(4)]
            if tr.gather is not None:
                tr.gather.wait_all()
            torch.cuda.synchronize()
            res[name] = (losses, tr.flat.param.detach().float().cpu(), tr.flat.master.detach().cpu())
        dist.destroy_process_group()
        ok = [("allreduce", res["allreduce"][0] == res["none"][0], torch.equal(res["allreduce"][1], res["none"][1]),
               torch.equal(res["allreduce"][2], res["none"][2]))]
        l0, p0, m0 = res["none"]
        l1, p1, m1 = res["zero"]
        ok.append(("zero", max(abs(a - b) for a, b in zip(l0, l1)) < 1e-3,
                   float((p0 - p1).abs().max()) <= 1e-2 * float(p0.abs().max()),
                   float((m0 - m1).abs().max()) <= 1e-3 * float(m0.abs().max())))
        q.put((ok, res["none"][0], None))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((None, None, traceback.format_exc()))


@pytest.mark.timeout(300)
def test_rccl_world1_zero_and_allreduce_match_no_collectives():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    ok, losses, err = q.get(timeout=280)
    p.join(60)
    assert err is None, err
    assert losses[-1] < losses[0]
    for name, same_loss, same_param, same_master in ok:
        assert same_loss and same_param and same_master, (name, same_loss, same_param, same_master)


def _pipe_worker(pipe, out, q):
    """One process per arm (the trainer reads TOA_ZERO_PIPE at init): rank 0
    of an emulated world-2 ZeRO-1 step on the GPU (TOA_EMULATE_WORLD=2, no
    traffic) -- the HIP AdamW over rank 0's shards, bucket by bucket
    (pipelined) or all at once.  Results go to a file (a queue would hand
    the parent shared memory its exiting producer frees)."""
    os.environ.update(TOA_ZERO="1", TOA_EMULATE_WORLD="2", TOA_EMULATE_BYTES="0", TOA_ZERO_PIPE=str(pipe))
    try:
        from tf_operator_amd.train.llm import LlamaTrainer

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.manual_seed(0)
        tr = LlamaTrainer("llama-tiny128", dev, micro_batch=2, seq_len=256)
        assert tr.gather is not None and tr.pipeline_tail == bool(pipe)
        batch = [tr.synthetic_batch()]
        losses = [float(tr.step(batch)) for _ in range(3)]
        tr.gather.wait_all()
        torch.cuda.synchronize()
        torch.save({"losses": losses, "param": tr.flat.param.detach().cpu(), "master": tr.flat.master.detach().cpu()},
                   out)
        q.put((pipe, None))
    except Exception as e:  # pragma: no cover
        q.put((pipe, repr(e)))


@pytest.mark.timeout(300)
def test_zero_pipelined_tail_bit_identical_on_gpu(tmp_path):
    """the pipelined ZeRO-1 tail on the GPU path (HIP AdamW writing
    the bf16 weights of each owned shard, the all-gather launched per bucket)
    gives the same losses, weights and fp32 master shards bit for bit as the
    whole-update-first tail."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    res = {}
    for pipe in (0, 1):
        out = str(tmp_path / f"pipe{pipe}.pt")
        p = ctx.Process(target=_pipe_worker, args=(pipe, out, q))
        p.start()
        _, err = q.get(timeout=250)
        p.join(timeout=30)
        assert err is None, err
        res[pipe] = torch.load(out, weights_only=True)
    a, b = res[0], res[1]
    assert a["losses"] == b["losses"]
    assert torch.equal(a["param"].view(torch.int16), b["param"].view(torch.int16))
    assert torch.equal(a["master"], b["master"])
