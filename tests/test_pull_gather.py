"""The copy-engine ZeRO-1 weight all-gather's pull protocol
(parallel/pull_gather.py) on the CPU: gloo ranks pull their peers' shards
through file-backed shared memory (ShmTransport, the GPU transport's
protocol: publish epoch -> wait for every peer's epoch -> copy the peers'
shards) and the result is compared bit for bit with
dist.all_gather_into_tensor of the same shards, over several steps, at
world 2, 4 and 8 (the headline job's size), bf16 and fp32, with buckets of different sizes."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tag, dtype, q):
    import torch.distributed as dist

    from tf_operator_amd.parallel import zero
    from tf_operator_amd.parallel.pull_gather import PullGather, ShmTransport

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    t = None
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        sizes = [64 * world * k for k in (3, 1, 7, 2)]          # bucket lengths (multiples of 8 world)
        ranges, lo = [], 0
        for n in sizes:
            ranges.append((lo, lo + n))
            lo += n
        numel = lo
        t = ShmTransport(tag, rank, world, numel, dtype, len(ranges))
        pg = PullGather(t, ranges, rank, world)
        ok = True
        for step in range(4):
            g = torch.Generator().manual_seed(1000 * step + rank)
            # this rank's "updated" shards (owned ranges), other ranges stale
            t.buf.copy_(torch.full((numel,), -1.0).to(dtype))
            for (s, e) in zero.owned_ranges([(a, b) for a, b in ranges], world, rank):
                t.buf[s:e].copy_(torch.randn(e - s, generator=g).to(dtype))
            ref = t.buf.clone()
            pg.new_step()
            for b in reversed(range(len(ranges))):    # ParamGather.order(): forward-need order
                pg.launch_one(b).wait()
            # reference: RCCL's (here gloo's) all-gather of the same shards
            for (s, e) in ranges:
                n = (e - s) // world
                out = torch.empty(e - s, dtype=dtype)
                dist.all_gather_into_tensor(out, ref[s + rank * n:s + (rank + 1) * n].clone())
                ok = ok and torch.equal(out.view(torch.int16 if dtype == torch.bfloat16 else torch.int32),
                                        t.buf[s:e].clone().view(torch.int16 if dtype == torch.bfloat16 else torch.int32))
        q.put((rank, ok, None))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(e)))
    finally:
        if t is not None:
            t.close()
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world,dtype", [(2, torch.bfloat16), (4, torch.float32), (8, torch.bfloat16)])
def test_pull_gather_matches_all_gather(world, dtype):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, tag = _port(), f"t{os.getpid()}_{world}"
    procs = [ctx.Process(target=_worker, args=(r, world, port, tag, dtype, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for rank, ok, err in res:
        assert err is None, (rank, err)
        assert ok, rank
    leftovers = [f for f in os.listdir("/dev/shm") if f.startswith(f"toa_pull_{tag}")]
    assert not leftovers, leftovers


def test_zero_ag_mode_env(monkeypatch):
    from tf_operator_amd.parallel import pull_gather

    monkeypatch.delenv("TOA_ZERO_AG", raising=False)
    assert pull_gather.mode_from_env() == "rccl"
    monkeypatch.setenv("TOA_ZERO_AG", "sdma")
    assert pull_gather.mode_from_env() == "sdma"
    monkeypatch.setenv("TOA_ZERO_AG", "bogus")
    with pytest.raises(ValueError):
        pull_gather.mode_from_env()


def _rs_worker(rank, world, port, tag, q):
    """The copy-engine reduce-scatter protocol (PullReduceScatter) over
    ShmTransport: each rank's shard of every bucket must equal the fp32 sum
    (own slice first, then the peers in rank order, rounded once) of every
    rank's gradients; the rest of the buffer keeps this rank's own values."""
    import torch.distributed as dist

    from tf_operator_amd.parallel import zero
    from tf_operator_amd.parallel.pull_gather import PullReduceScatter, ShmTransport

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    t = None
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        sizes = [64 * world * k for k in (5, 1, 3, 2)]
        ranges, lo = [], 0
        for n in sizes:
            ranges.append((lo, lo + n))
            lo += n
        t = ShmTransport(tag, rank, world, lo, torch.bfloat16, len(ranges))
        rs = PullReduceScatter(t, ranges, rank, world)
        ok = True
        for step in range(3):
            grads = [torch.randn(lo, generator=torch.Generator().manual_seed(77 * step + r)).to(torch.bfloat16)
                     for r in range(world)]
            t.buf.copy_(grads[rank])
            dist.barrier()   # stand-in for the previous step's all-gather ordering
            works = [(b, rs.launch_one(b)) for b in reversed(range(len(ranges)))]   # backward order
            for b, w in works:
                w.wait()
                rs.reduce(b)
            rs.new_step()
            want = grads[rank].clone()
            for s, e in zero.owned_ranges(ranges, world, rank):
                acc = grads[rank][s:e].float()
                for r in range(world):
                    if r != rank:
                        acc += grads[r][s:e].float()
                want[s:e] = acc.to(torch.bfloat16)
            ok = ok and torch.equal(t.buf.clone().view(torch.int16), want.view(torch.int16))
            dist.barrier()
        q.put((rank, ok, None))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(e)))
    finally:
        if t is not None:
            t.close()
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_pull_reduce_scatter_matches_sum(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, tag = _port(), f"rs{os.getpid()}_{world}"
    procs = [ctx.Process(target=_rs_worker, args=(r, world, port, tag, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for rank, ok, err in res:
        assert err is None, (rank, err)
        assert ok, rank
    leftovers = [f for f in os.listdir("/dev/shm") if f.startswith(f"toa_pull_{tag}")]
    assert not leftovers, leftovers


def test_zero_rs_mode_env(monkeypatch):
    from tf_operator_amd.parallel import pull_gather

    monkeypatch.delenv("TOA_ZERO_RS", raising=False)
    assert pull_gather.rs_mode_from_env() == "rccl"
    monkeypatch.setenv("TOA_ZERO_RS", "sdma")
    assert pull_gather.rs_mode_from_env() == "sdma"
    monkeypatch.setenv("TOA_ZERO_RS", "ring")
    with pytest.raises(ValueError):
        pull_gather.rs_mode_from_env()


def _lost_peer_worker(rank, world, port, tag, lost, q):
    """World-8 protocol with one peer (`lost`) that never publishes: every
    other rank's pull must fail within the transport's timeout, naming the
    lost rank, instead of hanging the step."""
    import time

    import torch.distributed as dist

    from tf_operator_amd.parallel.pull_gather import PullGather, ShmTransport

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    t = None
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ranges = [(0, 64 * world), (64 * world, 192 * world)]
        t = ShmTransport(tag, rank, world, 192 * world, torch.bfloat16, len(ranges), timeout_s=2.0)
        pg = PullGather(t, ranges, rank, world)
        pg.new_step()
        if rank == lost:
            t.publish = lambda idx, epoch: None      # stalled: never publishes its shards
        t0 = time.monotonic()
        try:
            for b in reversed(range(len(ranges))):
                pg.launch_one(b).wait()
            q.put((rank, "ok", time.monotonic() - t0))
        except RuntimeError as e:
            q.put((rank, str(e), time.monotonic() - t0))
    except Exception as e:  # pragma: no cover
        q.put((rank, "setup: " + repr(e), 0.0))
    finally:
        for p in (getattr(t, "paths", [None])[rank:rank + 1] + getattr(t, "fpaths", [None])[rank:rank + 1]):
            if p:
                try:
                    os.unlink(p)
                except FileNotFoundError:
                    pass


@pytest.mark.timeout(180)
def test_pull_gather_world8_lost_peer_fails_every_rank_in_time():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, lost = 8, 5
    port, tag = _port(), f"lost{os.getpid()}"
    procs = [ctx.Process(target=_lost_peer_worker, args=(r, world, port, tag, lost, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (msg, dt) for r, msg, dt in (q.get(timeout=150) for _ in range(world))}
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    for r in range(world):
        msg, dt = res[r]
        if r == lost:
            continue   # it pulls from live peers; its own failure shows up as theirs
        assert f"rank {lost} never published" in msg, (r, msg)
        assert dt < 10.0, (r, dt)


def test_sdma_reduce_scatter_refuses_accumulated_grads():
    """TOA_ZERO_RS=sdma with TOA_FRESH_GRADS=0: the next step's zeroing pass is
    not ordered after the owners' pulls of this rank's gradient slices, so the
    trainer refuses the combination before anything is built (advice r5)."""
    import types

    from tf_operator_amd.train.llm import LlamaTrainer

    stub = types.SimpleNamespace(fresh_grads=False, bucketer=None, flat=None)
    with pytest.raises(RuntimeError, match="needs fresh gradients"):
        LlamaTrainer._build_pull_reduce(stub)
