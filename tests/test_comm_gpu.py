"""One-shot IPC all-reduce (csrc/hip/comm.hip) with 2 processes on the one
GPU of the test box: handles exchanged over a gloo group, results vs the
exact sum, 2-slot ring reuse over many calls, bf16 and fp32, odd sizes."""
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


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from tf_operator_amd.parallel.ipc import IpcAllReduce

        ar = IpcAllReduce(slot_bytes=4 << 20, timeout_ms=20000)
        worst = 0.0
        for it in range(24):
            for n, dt in ((1000, torch.bfloat16), (262147, torch.float32), (1 << 20, torch.bfloat16)):
                g = torch.Generator(device="cpu").manual_seed(1000 * it + n)
                parts = [torch.randn(n, generator=g) for _ in range(world)]
                t = parts[rank].to(dt).cuda()
                ar(t)
                want = sum(p.to(dt).float() for p in parts)
                worst = max(worst, float((t.float().cpu() - want).abs().max() / (want.abs().max() + 1e-6)))
        torch.cuda.synchronize()
        ar.check()
        ar.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, worst, None))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(e)))


@pytest.mark.timeout(240)
def test_ipc_oneshot_allreduce_two_processes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for rank, worst, err in res:
        assert err is None, (rank, err)
        assert worst < 1e-2, (rank, worst)


def _dp_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TOA_IPC_ALLREDUCE="1",
                      LOCAL_WORLD_SIZE=str(world))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from tf_operator_amd.models.vision import MnistMLP
        from tf_operator_amd.ops.llm import cross_entropy
        from tf_operator_amd.train import simple
        from tf_operator_amd.train.data import SyntheticMNIST
        from tf_operator_amd.train.runtime import Runtime

        torch.manual_seed(0)
        model = MnistMLP(100, dtype=torch.float32, device="cuda")
        rt = Runtime()
        rt.info = type("I", (), {"rank": rank, "world": world})()
        tr = simple.DPTrainer(model, lambda o, y: cross_entropy(o, y), rt, lr=1e-3)
        assert tr.bucketer.ipc is not None
        data = SyntheticMNIST(100, rank, world, device="cuda")
        for _ in range(20):
            tr.step(*data.next())
        torch.cuda.synchronize()
        tr.bucketer.ipc.check()
        flat = tr.flat.param.detach().float().cpu()
        out = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(out, flat)
        q.put((rank, bool(torch.equal(out[0], out[1])), None))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, None, repr(e)))


@pytest.mark.timeout(240)
def test_dp_trainer_over_ipc_allreduce():
    """GradBucketer routes a small model's buckets through the one-shot IPC
    path; the replicas stay identical."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
    for rank, same, err in res:
        assert err is None, (rank, err)
        assert same, rank


def _lost_peer_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from tf_operator_amd.parallel.ipc import IpcAllReduce

        ar = IpcAllReduce(slot_bytes=1 << 20, timeout_ms=300)
        raised = None
        if rank == 0:  # rank 1 never joins this all-reduce: a lost peer
            ar(torch.ones(1024, device="cuda"))
            try:
                for _ in range(3):  # poll() looks at the copy queued one step earlier
                    torch.cuda.synchronize()
                    ar.poll()
            except RuntimeError as e:
                raised = str(e)
        dist.barrier()
        ar.close()
        dist.destroy_process_group()
        q.put((rank, raised, None))
    except Exception as e:  # pragma: no cover
        q.put((rank, None, repr(e)))


@pytest.mark.timeout(120)
def test_ipc_lost_peer_raises_from_poll():
    """A peer that never arrives sets the sticky error word after the bounded
    spin; GradBucketer.finish()'s per-step poll() turns it into an exception
    instead of letting stale peer slots be summed into the gradient."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_lost_peer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (m, e)) for r, m, e in (q.get(timeout=100) for _ in range(2)))
    for p in procs:
        p.join(timeout=30)
    assert res[0][1] is None and res[1][1] is None, res
    assert res[0][0] and "rank" in res[0][0] and "1" in res[0][0], res


def _operator_env_worker(rank, world, port, env, q):
    """One replica with exactly the env the operator's node-local layout
    injects (core.gen_env), no TOA_IPC_ALLREDUCE: GradBucketer must pick the
    one-shot path by itself, per bucket by size."""
    import torch.distributed as dist

    os.environ.pop("TOA_IPC_ALLREDUCE", None)
    os.environ.update(env, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=int(env["RANK"]), world_size=int(env["WORLD_SIZE"]))
        from tf_operator_amd.models.vision import MnistMLP
        from tf_operator_amd.ops.llm import cross_entropy
        from tf_operator_amd.train import simple
        from tf_operator_amd.train.data import SyntheticMNIST
        from tf_operator_amd.train.runtime import Runtime

        torch.manual_seed(0)
        # hid.weight 784 x 3000 fp32 = 9.4 MB: above the one-shot size; the
        # 12 KB-120 KB tensors below it
        model = MnistMLP(3000, dtype=torch.float32, device="cuda")
        rt = Runtime()
        rt.info = type("I", (), {"rank": rank, "world": world})()
        tr = simple.DPTrainer(model, lambda o, y: cross_entropy(o, y), rt, lr=1e-3, bucket_mb=0.05)
        reason = tr.bucketer.ipc_reason
        data = SyntheticMNIST(100, rank, world, device="cuda")
        for _ in range(5):
            tr.step(*data.next())
        torch.cuda.synchronize()
        tr.bucketer.verify()
        flat = tr.flat.param.detach().float().cpu()
        out = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(out, flat)
        q.put((rank, (tr.bucketer.ipc is not None, reason, dict(tr.bucketer.path_counts),
                      bool(torch.equal(out[0], out[1]))), None))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, None, repr(e)))


@pytest.mark.timeout(240)
def test_oneshot_under_operator_env():
    """The node-local env of a Worker=2 TFJob makes the job one-shot
    eligible (LOCAL_WORLD_SIZE = world).  On this one-GPU box both replicas
    share the device over gloo, so automatic selection declines (it needs an
    RCCL group, one GPU per rank -- ADVICE r3) and the path is forced here:
    small buckets go one-shot, the big one stays on the process group, and
    the replicas stay identical.  The automatic RCCL case is the pure
    decision in tests/test_core_controller.py::test_oneshot_selection_under_operator_env."""
    from tf_operator_amd import core

    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
           "metadata": {"name": "nl", "namespace": "default", "annotations": {"amd.com/node-local": "true"}},
           "spec": {"tfReplicaSpecs": {"Worker": {"replicas": 2, "template": {"spec": {"containers": [
               {"name": "tensorflow", "image": "x", "resources": {"limits": {"amd.com/gpu": 1}}}]}}}}}}
    keep = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "TOA_NODE_LOCAL")
    envs = [{e["name"]: e["value"] for e in core.gen_env(job, "Worker", i) if e["name"] in keep} for i in range(2)]
    assert [e["LOCAL_WORLD_SIZE"] for e in envs] == ["2", "2"]
    for e in envs:
        e["TOA_IPC_ALLREDUCE"] = "1"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_operator_env_worker, args=(r, 2, port, envs[r], q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
    for rank, got, err in res:
        assert err is None, (rank, err)
        selected, reason, counts, same = got
        assert selected and reason.startswith("forced"), (rank, reason)
        assert counts["oneshot"] > 0 and counts["collective"] > 0, (rank, counts)
        assert same, rank


def test_emulate_xfer_moves_bytes_at_the_paced_rate():
    """parallel/emulate.py's stand-in for an RCCL ring kernel: copies every
    byte, and paced to G GB/s on 32 workgroups it takes about bytes / G
    (the property the overlap emulation relies on); unpaced it runs at HBM
    speed."""
    from tf_operator_amd.ops import _lib

    src = torch.randint(0, 255, (64 << 20,), dtype=torch.uint8, device="cuda")
    dst = torch.zeros_like(src)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = {}
    # warm-up launch (code-object load) outside the timed calls
    _lib.call("toa_emulate_xfer", _lib.ptr(src), _lib.ptr(dst), 1 << 20, 32, 0.0, _lib.stream(src))
    for gbps in (0.0, 100.0):
        dst.zero_()
        torch.cuda.synchronize()
        ev[0].record()
        _lib.call("toa_emulate_xfer", _lib.ptr(src), _lib.ptr(dst), src.numel(), 32, gbps, _lib.stream(src))
        ev[1].record()
        torch.cuda.synchronize()
        times[gbps] = ev[0].elapsed_time(ev[1])
        assert torch.equal(src, dst), gbps
    want_ms = src.numel() / 100e9 * 1e3  # 0.67 ms at 100 GB/s
    assert 0.9 * want_ms <= times[100.0] <= 1.6 * want_ms, times
    assert times[0.0] < 0.5 * want_ms, times


def _pull_worker(rank, world, port, q):
    """Copy-engine weight all-gather (parallel/pull_gather.py) between two
    processes on the one GPU: IPC-mapped flat buffers, flag publish / wait
    kernels, SDMA copies; each step's result vs the exact concatenation."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from tf_operator_amd.parallel import zero
        from tf_operator_amd.parallel.pull_gather import GpuIpcTransport, PullGather

        sizes = [64 * world * k for k in (4096, 1, 333, 2048)]   # 1 MiB .. bf16 buckets
        ranges, lo = [], 0
        for n in sizes:
            ranges.append((lo, lo + n))
            lo += n
        buf = torch.zeros(lo, device="cuda", dtype=torch.bfloat16)
        t = GpuIpcTransport(buf, rank, world, len(ranges), timeout_ms=20000)
        pg = PullGather(t, ranges, rank, world)
        ok = True
        for step in range(6):
            want = torch.empty(lo, dtype=torch.bfloat16)
            for r in range(world):
                g = torch.Generator().manual_seed(100 * step + r)
                vals = torch.randn(lo, generator=g).to(torch.bfloat16)
                for (s, e) in zero.owned_ranges(ranges, world, r):
                    want[s:e] = vals[s:e]
                if r == rank:
                    mine = vals.cuda()
            buf.fill_(-7)
            for (s, e) in zero.owned_ranges(ranges, world, rank):   # "AdamW" on the compute stream
                buf[s:e].copy_(mine[s:e])
            pg.new_step()
            works = [pg.launch_one(b) for b in reversed(range(len(ranges)))]
            for w in works:
                w.wait()
            got = buf.cpu()
            ok = ok and torch.equal(got.view(torch.int16), want.view(torch.int16))
            dist.barrier()   # the test's own stand-in for the next step's reduce-scatter ordering
        torch.cuda.synchronize()
        t.check()
        pg.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ok, None))
    except Exception as e:  # pragma: no cover
        q.put((rank, None, repr(e)))


@pytest.mark.timeout(240)
def test_pull_gather_copy_engine_two_processes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _port()
    procs = [ctx.Process(target=_pull_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for rank, ok, err in res:
        assert err is None, (rank, err)
        assert ok, rank


def _rs_pull_worker(rank, world, port, q):
    """Copy-engine reduce-scatter (PullReduceScatter over GpuIpcTransport)
    between two processes on the one GPU: each shard must equal the fp32 sum
    (own slice first, peers in rank order, one rounding) of both ranks'
    gradients, the rest of the buffer untouched."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from tf_operator_amd.parallel import zero
        from tf_operator_amd.parallel.pull_gather import GpuIpcTransport, PullReduceScatter

        sizes = [64 * world * k for k in (4096, 1, 333, 2048)]
        ranges, lo = [], 0
        for n in sizes:
            ranges.append((lo, lo + n))
            lo += n
        buf = torch.zeros(lo, device="cuda", dtype=torch.bfloat16)
        t = GpuIpcTransport(buf, rank, world, len(ranges), timeout_ms=20000, what="reduce-scatter")
        rs = PullReduceScatter(t, ranges, rank, world)
        ok = True
        for step in range(5):
            grads = [torch.randn(lo, generator=torch.Generator().manual_seed(31 * step + r)).to(torch.bfloat16)
                     for r in range(world)]
            buf.copy_(grads[rank].cuda())            # "backward" on the compute stream
            works = [(b, rs.launch_one(b)) for b in reversed(range(len(ranges)))]
            for b, w in works:
                w.wait()
                rs.reduce(b)
            rs.new_step()
            want = grads[rank].clone()
            for s_, e in zero.owned_ranges(ranges, world, rank):
                acc = grads[rank][s_:e].float()
                for r in range(world):
                    if r != rank:
                        acc += grads[r][s_:e].float()
                want[s_:e] = acc.to(torch.bfloat16)
            ok = ok and torch.equal(buf.cpu().view(torch.int16), want.view(torch.int16))
            dist.barrier()   # the test's stand-in for the all-gather that orders the next backward
        torch.cuda.synchronize()
        t.check()
        rs.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ok, None))
    except Exception as e:  # pragma: no cover
        q.put((rank, None, repr(e)))


def test_pull_reduce_scatter_copy_engine_two_processes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 2, _port()
    procs = [ctx.Process(target=_rs_pull_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for rank, ok, err in res:
        assert err is None, (rank, err)
        assert ok, rank


def _zero_sdma_trainer_worker(rank, world, port, out, sdma):
    """llama-tiny ZeRO-1 steps, both ranks on the one GPU and the same batch.
    sdma: the weight all-gather AND the gradient reduce-scatter by copy-engine
    pulls (no collective on either path; the process group is gloo and
    carries only the norm); world 1 (rank 0 only): the unsharded reference."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    if sdma:
        os.environ.update(TOA_ZERO_AG="sdma", TOA_ZERO_RS="sdma")
    try:
        torch.cuda.set_device(0)
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        from tf_operator_amd.models.llama import PRESETS
        from tf_operator_amd.train.llm import LlamaTrainer

        tr = LlamaTrainer(PRESETS["llama-tiny"], torch.device("cuda", 0), micro_batch=2, seq_len=128, lr=1e-3,
                          bucket_mb=0.25, shard_optimizer=world > 1)
        if world > 1:
            assert tr.bucketer.pull_rs is not None and tr.gather.pull is not None
            assert len(tr.bucketer.buckets) > 2
        b = tr.synthetic_batch()
        losses = [float(tr.step([b])) for _ in range(5)]
        if tr.gather is not None:
            tr.gather.wait_all()
        torch.cuda.synchronize()
        if world > 1:
            tr.bucketer.pull_rs.check()
            tr.gather.pull.check()
        torch.save({"losses": losses, "param": tr.flat.param.float().cpu()}, f"{out}.{world}.{rank}")
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        torch.save({"err": repr(e)}, f"{out}.{world}.{rank}")


def test_zero_trainer_both_collectives_by_copy_engine(tmp_path):
    """TOA_ZERO_AG=sdma + TOA_ZERO_RS=sdma end to end: two ranks on the same
    batch must train like one unsharded rank (the sum of two equal bf16
    gradients halves back exactly; only the norm's summation order differs)."""
    ctx = mp.get_context("spawn")
    out = str(tmp_path / "res")
    ref = ctx.Process(target=_zero_sdma_trainer_worker, args=(0, 1, _port(), out, False))
    ref.start()
    ref.join(timeout=300)
    port = _port()
    procs = [ctx.Process(target=_zero_sdma_trainer_worker, args=(r, 2, port, out, True)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    r1 = torch.load(f"{out}.1.0", weights_only=True)
    assert "err" not in r1, r1
    for r in range(2):
        r2 = torch.load(f"{out}.2.{r}", weights_only=True)
        assert "err" not in r2, (r, r2)
        assert max(abs(a - b) for a, b in zip(r1["losses"], r2["losses"])) < 2e-3, (r1["losses"], r2["losses"])
        d = (r1["param"] - r2["param"]).abs().max()
        assert float(d) <= 2e-2 * float(r1["param"].abs().max()), float(d)


def _zero8_worker(rank, world, port, out, lost, preset="llama-tiny", seq=128):
    """llama-tiny ZeRO-1 on `world` processes sharing the one GPU, both
    collectives by copy-engine pulls (gloo carries nothing else: clipping is
    off, so no norm all-reduce either), every rank on the same batch.
    lost >= 0: that rank never publishes its shards (a stalled peer); every
    rank must then leave non-zero within the pull timeout.  Results go to a
    file; the process ends with os._exit (0 = trained, 1 = raised)."""
    import time

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    if world > 1:
        os.environ.update(TOA_ZERO_AG="sdma", TOA_ZERO_RS="sdma", TOA_PULL_TIMEOUT_MS="3000")
    code, t0 = 1, time.monotonic()
    try:
        torch.cuda.set_device(0)
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        from tf_operator_amd.models.llama import PRESETS
        from tf_operator_amd.train.llm import LlamaTrainer

        tr = LlamaTrainer(PRESETS[preset], torch.device("cuda", 0), micro_batch=2, seq_len=seq, lr=1e-3,
                          bucket_mb=0.25, shard_optimizer=world > 1)
        tr.opt.max_grad_norm = 0.0   # no clipping: the sharded run must match the unsharded one bit for bit
        if world > 1:
            assert tr.collective_transport() == "sdma" and len(tr.bucketer.buckets) > 2
            if rank == lost:
                for x in tr._pull_transports():
                    x.t.publish = lambda idx, epoch: None
        b = tr.synthetic_batch()
        losses = [float(tr.step([b])) for _ in range(6)]
        if tr.gather is not None:
            tr.gather.wait_all()
        torch.cuda.synchronize()
        for x in tr._pull_transports():
            x.check()
        torch.save({"losses": losses, "param": tr.flat.param.cpu().view(torch.int16),
                    "s": time.monotonic() - t0}, f"{out}.{world}.{rank}")
        tr.close()
        code = 0
    except Exception as e:  # noqa: BLE001 - recorded, then a non-zero exit
        torch.save({"err": repr(e)[:2000], "s": time.monotonic() - t0}, f"{out}.{world}.{rank}")
    os._exit(code)


def _run_zero8(tmp_path, world, lost, preset="llama-tiny", seq=128):
    ctx = mp.get_context("spawn")
    out = str(tmp_path / f"z{lost}_{preset}_{seq}")
    port = _port()
    procs = [ctx.Process(target=_zero8_worker, args=(r, world, port, out, lost, preset, seq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    alive = [r for r, p in enumerate(procs) if p.is_alive()]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not alive, f"ranks {alive} still running after 240 s"
    return [p.exitcode for p in procs], [torch.load(f"{out}.{world}.{r}", weights_only=True) for r in range(world)]


@pytest.mark.timeout(600)
def test_zero1_eight_processes_copy_engine_bit_exact(tmp_path):
    """World 8 on the one GPU (the headline job's size, verdict r5): llama-tiny
    ZeRO-1 with the weight all-gather AND the gradient reduce-scatter by
    copy-engine pulls trains bit for bit like one unsharded rank (eight equal
    bf16 gradients sum exactly and the 1/8 scale undoes it)."""
    codes, ref = _run_zero8(tmp_path, 1, -1)
    assert codes == [0], ref
    codes, res = _run_zero8(tmp_path, 8, -1)
    assert codes == [0] * 8, [r.get("err") for r in res]
    for r in range(8):
        assert res[r]["losses"] == ref[0]["losses"], (r, res[r]["losses"], ref[0]["losses"])
        assert torch.equal(res[r]["param"], ref[0]["param"]), r


@pytest.mark.timeout(600)
def test_zero1_eight_processes_lost_peer_every_rank_exits_nonzero(tmp_path):
    """The same world-8 job with rank 5 never publishing: the pullers' bounded
    waits mark it lost, poll() raises on the following steps, and every rank
    -- the stalled one included, once its peers are gone -- exits non-zero
    well inside the pull timeout budget instead of hanging."""
    codes, res = _run_zero8(tmp_path, 8, 5)
    assert all(c != 0 for c in codes), (codes, [r.get("err") for r in res])
    assert any("rank" in (r.get("err") or "") and "5" in (r.get("err") or "") for r in res), res
    assert max(r["s"] for r in res) < 120, [r["s"] for r in res]


@pytest.mark.timeout(600)
def test_zero1_four_processes_fused_epilogues_bit_exact(tmp_path):
    """The fused paths of the flagship step under ZeRO-1 (llama-tiny128 at
    seq 512: the QKV GEMM's RoPE epilogue, the output projection's delta
    epilogue, the residual adds in the output / down projections' epilogues
    with their presummed norms -- whose module hooks carry the gather waits --,
    the weight-gradient kernels) with both collectives by
    copy-engine pulls: four ranks train bit for bit like one unsharded rank
    (whose update also writes the W^T copies, toa_adamw_wt)."""
    codes, ref = _run_zero8(tmp_path, 1, -1, "llama-tiny128", 512)
    assert codes == [0], ref
    codes, res = _run_zero8(tmp_path, 4, -1, "llama-tiny128", 512)
    assert codes == [0] * 4, [r.get("err") for r in res]
    for r in range(4):
        assert res[r]["losses"] == ref[0]["losses"], (r, res[r]["losses"], ref[0]["losses"])
        assert torch.equal(res[r]["param"], ref[0]["param"]), r
