"""Per-rank sharded asynchronous checkpoints (train/sharded_ckpt.py) and
ZeRO-1 re-sharding on load, on CPU/gloo.

Reference behaviour being matched: every worker of the reference's Keras job
checkpoints and the job resumes after preemption
(multi_worker_strategy-with-keras.py:92-109); the elastic policy needs the
resume to work at a different world size (BASELINE config #5)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tf_operator_amd.parallel import zero
from tf_operator_amd.parallel.flat import FlatParams
from tf_operator_amd.train import sharded_ckpt
from tf_operator_amd.train.llm import LlamaTrainer, load_trainer_state, trainer_state


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flat(seed=0, n=(300, 77, 1000)):
    g = torch.Generator().manual_seed(seed)
    ps = [torch.nn.Parameter(torch.randn(k, generator=g)) for k in n]
    f = FlatParams(ps)
    f.exp_avg = torch.randn(f.numel, generator=g)
    f.exp_avg_sq = torch.rand(f.numel, generator=g)
    return f


def _state(f):
    return {"flat": f.state_dict(), "opt": {"step": 5, "lr": 1e-3}, "step": 5}


def test_compact_state_roundtrip_any_world(tmp_path):
    """A world-2 save (each rank its own compact shards) restores into a
    world-1 layout and into a world-3 sharding, element for element."""
    full = _flat()
    ref = {k: getattr(full, k).clone() for k in sharded_ckpt.STATE_KEYS}
    n = full.numel
    cut = (n // 2) // 64 * 64
    shards2 = [[(0, 64), (cut, n - 64)], [(64, cut), (n - 64, n)]]
    cks = []
    for r, rg in enumerate(shards2):  # both ranks' saves in flight at once (rank 0 commits)
        f = _flat()
        f.shard_state(rg)
        assert f.master.numel() == sum(b - a for a, b in rg)
        ck = sharded_ckpt.Checkpointer(str(tmp_path), rank=r, world=2, commit_timeout=60)
        ck.save(5, _state(f))
        cks.append(ck)
    for ck in cks:
        ck.wait()
    assert open(tmp_path / "latest").read() == "step_00000005"
    shares = sharded_ckpt.load_latest(str(tmp_path))
    assert [s["rank"] for s in shares] == [0, 1] and shares[0]["world"] == 2

    g = _flat(seed=1)  # different values everywhere
    g.load_state_shards([s["flat"] for s in shares], set_params="all")
    for k in sharded_ckpt.STATE_KEYS:
        assert torch.equal(getattr(g, k), ref[k]), k
    assert torch.equal(g.param, ref["master"].to(g.param.dtype))

    thirds = [(0, n // 3), (n // 3, 2 * n // 3), (2 * n // 3, n)]
    for lo, hi in thirds:
        h = _flat(seed=2)
        h.shard_state([(lo, hi)])
        h.load_state_shards([s["flat"] for s in shares], set_params="held")
        for k in sharded_ckpt.STATE_KEYS:
            assert torch.equal(getattr(h, k), ref[k][lo:hi]), (k, lo)


def test_replicated_shares_restore_once(tmp_path):
    """Without ZeRO every rank of a world-2 job saves the WHOLE state: a
    resume (any world size) takes each range once instead of rejecting the
    doubled coverage."""
    from tf_operator_amd.parallel.flat import _uncovered

    assert _uncovered(0, 10, []) == [(0, 10)]
    assert _uncovered(0, 10, [(2, 4), (6, 12)]) == [(0, 2), (4, 6)]
    assert _uncovered(3, 5, [(0, 10)]) == []
    full = _flat()
    ref = {k: getattr(full, k).clone() for k in sharded_ckpt.STATE_KEYS}
    cks = []
    for r in range(2):
        ck = sharded_ckpt.Checkpointer(str(tmp_path), rank=r, world=2, commit_timeout=60)
        ck.save(7, _state(_flat()))
        cks.append(ck)
    for ck in cks:
        ck.wait()
    shares = sharded_ckpt.load_latest(str(tmp_path))
    assert len(shares) == 2 and all(s["flat"]["state_ranges"] == [[0, full.numel]] or
                                    [tuple(x) for x in s["flat"]["state_ranges"]] == [(0, full.numel)]
                                    for s in shares)
    g = _flat(seed=1)
    g.load_state_shards([s["flat"] for s in shares], set_params="all")
    for k in sharded_ckpt.STATE_KEYS:
        assert torch.equal(getattr(g, k), ref[k]), k
    n = full.numel
    h = _flat(seed=2)
    h.shard_state([(64, n // 2 // 64 * 64)])
    h.load_state_shards([s["flat"] for s in shares], set_params="held")
    assert torch.equal(h.master, ref["master"][64:n // 2 // 64 * 64])


def test_uncommitted_step_is_not_latest(tmp_path):
    """Only rank 0 of a world-2 save finished: no manifest, the previous
    committed step stays `latest` (a crash mid-save loses nothing)."""
    f = _flat()
    ck = sharded_ckpt.Checkpointer(str(tmp_path), rank=0, world=1)
    ck.save(1, _state(f), block=True)
    ck2 = sharded_ckpt.Checkpointer(str(tmp_path), rank=1, world=2)  # rank 0 of step 2 never shows up
    ck2.save(2, _state(f), block=True)
    assert sharded_ckpt.latest_dir(str(tmp_path)).endswith("step_00000001")
    assert sharded_ckpt.load_latest(str(tmp_path))[0]["step"] == 1


def test_checkpoint_files_hold_no_pickle(tmp_path):
    f = _flat()
    ck = sharded_ckpt.Checkpointer(str(tmp_path), rank=0, world=1)
    ck.save(3, _state(f), block=True)
    d = sharded_ckpt.latest_dir(str(tmp_path))
    names = sorted(os.listdir(d))
    assert names == ["manifest.json", "rank00000.exp_avg.f32", "rank00000.exp_avg_sq.f32", "rank00000.json",
                     "rank00000.master.f32"]
    assert os.path.getsize(os.path.join(d, "rank00000.master.f32")) == 4 * f.numel
    assert ck.last_timing["bytes"] == 12 * f.numel


def _ckpt_worker(rank, world, port, root, phase, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = LlamaTrainer("llama-tiny", torch.device("cpu"), micro_batch=2, seq_len=32, lr=1e-3, seed=rank,
                          bucket_mb=0.01, shard_optimizer=world > 1)
        g = torch.Generator().manual_seed(7)
        batches = [(torch.randint(0, tr.cfg.vocab_size, (2, 33), generator=g)) for _ in range(world * 6)]
        batches = [(b[:, :-1].contiguous(), b[:, 1:].contiguous()) for b in batches]
        mine = batches[rank::world]
        ck = sharded_ckpt.Checkpointer(root, rank, world)
        res = {}
        if phase == "save":
            for i in range(3):
                tr.step([mine[i]])
            ck.save(tr.step_idx, trainer_state(tr))  # asynchronous ...
            res["cont"] = [float(tr.step([mine[3 + i]])) for i in range(2)]  # ... training continues
            ck.wait()
        else:
            shares = sharded_ckpt.load_latest(root)
            load_trainer_state(tr, shares)
            assert tr.step_idx == 3
            if world == 2:
                res["cont"] = [float(tr.step([mine[3 + i]])) for i in range(2)]
        full = zero.gather_full_state(tr.flat, world) if world > 1 else {
            k: getattr(tr.flat, k) for k in ("master", "exp_avg", "exp_avg_sq")}
        res["master"] = full["master"].clone()
        res["param"] = tr.flat.param.float().clone()
        if rank == 0:
            torch.save(res, out)
    finally:
        dist.destroy_process_group()


def test_zero_checkpoint_resume_and_reshard(tmp_path):
    """World 2 with ZeRO-1 saves asynchronously while it keeps training; a
    fresh world-2 job resumes and reproduces the continuation exactly; a
    world-1 (and a world-4) job re-shard the same checkpoint to the saved
    state."""
    root = str(tmp_path / "ck")
    a = str(tmp_path / "a.pt")
    mp.spawn(_ckpt_worker, args=(2, _free_port(), root, "save", a), nprocs=2, join=True)
    saved = torch.load(a, weights_only=True)
    b = str(tmp_path / "b.pt")
    mp.spawn(_ckpt_worker, args=(2, _free_port(), root, "load", b), nprocs=2, join=True)
    resumed = torch.load(b, weights_only=True)
    assert resumed["cont"] == saved["cont"]
    assert torch.equal(resumed["master"], saved["master"])
    shares = sharded_ckpt.load_latest(root)
    ref_master = torch.zeros_like(saved["master"])
    for s in shares:
        off = 0
        for lo, hi in s["flat"]["state_ranges"]:
            ref_master[lo:hi] = torch.from_numpy(s["flat"]["master"][off:off + hi - lo].copy())
            off += hi - lo
    for w in (1, 4):
        c = str(tmp_path / f"c{w}.pt")
        mp.spawn(_ckpt_worker, args=(w, _free_port(), root, "load", c), nprocs=w, join=True)
        got = torch.load(c, weights_only=True)
        assert torch.equal(got["master"], ref_master), w
        assert torch.equal(got["param"], ref_master.to(torch.bfloat16).float()), w


@pytest.mark.parametrize("world,zero", [(2, "auto"), (2, "0")])
def test_llama_train_zero_checkpoint_every(tmp_path, world, zero):
    """The operator payload with ZeRO on (its default for world > 1) or off,
    and --checkpoint-every, runs to completion on every rank (no chief-only
    collective), leaves a committed world-2 checkpoint and resumes from it."""
    root = str(tmp_path / "ck")
    port = _free_port()
    import subprocess
    import sys

    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world),
                   TOA_CHECKPOINT_DIR=root, TOA_NO_GPU="1", OMP_NUM_THREADS="1")
    def run(steps):
        procs = []
        for r in range(world):
            env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                       WORLD_SIZE=str(world), TOA_CHECKPOINT_DIR=root, TOA_NO_GPU="1", OMP_NUM_THREADS="1")
            procs.append(subprocess.Popen([sys.executable, "-m", "tf_operator_amd.examples.llama_train", "--steps",
                                           str(steps), "--seq-len", "32", "--checkpoint-every", "2", "--zero", zero],
                                          env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs = [p.communicate(timeout=300)[0].decode() for p in procs]
        assert all(p.returncode == 0 for p in procs), outs

    run(4)
    shares = sharded_ckpt.load_latest(root)
    assert shares[0]["step"] == 4 and shares[0]["world"] == world and len(shares) == world
    n = shares[0]["flat"]["numel"]
    per_rank = sum(hi - lo for s in shares for lo, hi in s["flat"]["state_ranges"])
    assert per_rank == (n if zero == "auto" else world * n)
    port = _free_port()
    run(6)  # resumes at step 4 from the world-2 shares, runs to 6
    assert sharded_ckpt.load_latest(root)[0]["step"] == 6


def test_stale_partial_of_crashed_attempt_never_commits(tmp_path):
    """A crashed attempt left ``step_N.partial`` with both ranks' markers.
    Saving step N again, rank 0 must NOT take the old markers as this
    attempt's: it waits for rank 1's new share, then commits the new data
    (stale markers satisfied the wait while peers rewrote)."""
    root = str(tmp_path)
    # the crashed attempt: rank 1's share and marker, never committed (its
    # rank 0 died before the commit)
    stale = sharded_ckpt.Checkpointer(root, rank=1, world=2, attempt="old", commit_timeout=1.0)
    stale.save(4, _state(_flat(seed=11)), block=True)
    assert os.path.exists(os.path.join(root, "step_00000004.partial", "rank00001.json"))
    new = [_flat(seed=20), _flat(seed=21)]
    ck0 = sharded_ckpt.Checkpointer(root, rank=0, world=2, attempt="new", commit_timeout=1.0)
    ck0.save(4, _state(new[0]))
    with pytest.raises(RuntimeError):  # times out: rank 1's marker is the old attempt's
        ck0.wait()
    assert sharded_ckpt.latest_dir(root) is None
    ck0 = sharded_ckpt.Checkpointer(root, rank=0, world=2, attempt="new", commit_timeout=60)
    ck1 = sharded_ckpt.Checkpointer(root, rank=1, world=2, attempt="new", commit_timeout=60)
    ck0.save(4, _state(new[0]))
    ck1.save(4, _state(new[1]))
    ck0.wait()
    ck1.wait()
    shares = sharded_ckpt.load_latest(root)
    assert [s["rank"] for s in shares] == [0, 1]
    for r in range(2):
        assert torch.equal(torch.from_numpy(shares[r]["flat"]["master"].copy()), new[r].master)


def _stream_worker(rank, world, port, root, phase, out):
    """Synthetic token stream + RNG across a checkpoint (gloo, ZeRO-1)."""
    from tf_operator_amd.train.data import SyntheticTokens

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = LlamaTrainer("llama-tiny", torch.device("cpu"), micro_batch=2, seq_len=32, lr=1e-3, seed=0,
                          bucket_mb=0.01, shard_optimizer=True)
        data = SyntheticTokens(2, 32, tr.cfg.vocab_size, rank=rank)
        ck = sharded_ckpt.Checkpointer(root, rank, world)
        ck.sync_attempt()
        res = {"loss": []}
        torch.manual_seed(1000 + rank)
        if phase == "full":
            for i in range(5):
                res["loss"].append(float(tr.step([data.next()])))
                torch.rand(3 + i)  # the step's own (here: stand-in) RNG use
        elif phase == "save":
            for i in range(3):
                res["loss"].append(float(tr.step([data.next()])))
                torch.rand(3 + i)
            ck.save(tr.step_idx, trainer_state(tr, data), block=True)
        else:
            torch.manual_seed(99)  # a restarted process: different RNG, fresh stream
            load_trainer_state(tr, sharded_ckpt.load_latest(root), data=data)
            assert data.cursor == 3 and tr.step_idx == 3
            for i in range(3, 5):
                res["loss"].append(float(tr.step([data.next()])))
                torch.rand(3 + i)
        res["rand"] = torch.rand(4)
        torch.save(res, f"{out}.{rank}")
    finally:
        dist.destroy_process_group()


def test_resume_reproduces_losses_rng_and_data(tmp_path):
    """3 steps + checkpoint + a fresh world-2 job running 2 more steps gives
    bit-for-bit the losses and the RNG draws of 5 uninterrupted steps (the
    data cursor and every rank's RNG state travel in the checkpoint)."""
    root = str(tmp_path / "ck")
    outs = {}
    for phase in ("full", "save", "load"):
        o = str(tmp_path / phase)
        mp.spawn(_stream_worker, args=(2, _free_port(), root if phase != "full" else str(tmp_path / "x"), phase, o),
                 nprocs=2, join=True)
        outs[phase] = [torch.load(f"{o}.{r}", weights_only=True) for r in range(2)]
    for r in range(2):
        full, a, b = outs["full"][r], outs["save"][r], outs["load"][r]
        assert a["loss"] + b["loss"] == full["loss"], r
        assert torch.equal(b["rand"], full["rand"]), r
