"""Parameter servers over torch.distributed (parallel/ps_collective.py) on
CPU/gloo -- the RCCL path's protocol with W workers + P servers in one
process group.

(1) sync mode (SyncReplicasOptimizer, replicas_to_aggregate = W) equals one
    process applying AdamW to the mean of the workers' gradients, for one
    and for two servers (the flat vector sharded across them), with
    gradient buckets small enough that a bucket straddles a shard boundary;
(2) async mode applies every push as its own update (W x steps updates)
    and every worker ends with weights some server produced;
(3) E2E: a TFJob PS=1 Worker=2 running the ResNet payload (resnet-tiny)
    through the operator and the local kubelet, in both modes."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tf_operator_amd.ops.optim import FlatAdamW
from tf_operator_amd.parallel.flat import FlatParams
from tf_operator_amd.train import simple

STEPS, LR = 4, 1e-2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(16, 48), torch.nn.ReLU(), torch.nn.Linear(48, 40),
                               torch.nn.ReLU(), torch.nn.Linear(40, 8))


def _data(w):
    g = torch.Generator().manual_seed(1000 + w)
    return torch.randn(12, 16, generator=g), torch.randn(12, 8, generator=g)


class _RT:
    rank = 0

    def first_step_done(self):
        pass


def _proc(rank, workers, servers, mode, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=workers + servers)
    try:
        model = _model(seed=rank)  # different inits: the broadcast of worker 0's must win
        loss_fn = torch.nn.functional.mse_loss
        if rank >= workers:
            ps = simple.parameter_server(model, workers, servers, mode=mode, lr=LR, bucket_mb=0.0005)
            ps.serve(STEPS)
            lo, hi = ps.ranges[ps.p]
            res = {"updates": ps.updates, "lo": lo, "hi": hi, "param": ps.flat.param[lo:hi].clone()}
        else:
            tr = simple.PSTrainer(model, loss_fn, _RT(), workers, servers, mode=mode, lr=LR, bucket_mb=0.0005)
            x, y = _data(rank)
            losses = [float(tr.step(x, y)[0]) for _ in range(STEPS)]
            pending = len(tr.ps.pulls)  # sync: the last pull is still in flight when step() returns
            tr.sync_params()
            res = {"param": tr.flat.param.clone(), "nbuckets": len(tr.ps.buckets), "pieces": len(tr.ps.pieces),
                   "losses": losses, "pending_after_step": pending}
        torch.save(res, f"{out}.{rank}")
    finally:
        dist.destroy_process_group()


def _run(tmp_path, workers, servers, mode, tag="r"):
    out = str(tmp_path / tag)
    mp.spawn(_proc, args=(workers, servers, mode, _free_port(), out), nprocs=workers + servers, join=True)
    return [torch.load(f"{out}.{r}", weights_only=True) for r in range(workers + servers)]


def _reference(workers):
    model = _model(seed=0)
    params = [p for p in model.parameters()]
    flat = FlatParams(list(reversed(params)))
    simple.attach_autograd_hooks(flat)
    opt = FlatAdamW(flat, lr=LR, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=0.0)
    for _ in range(STEPS):
        flat.zero_grad()
        for w in range(workers):
            x, y = _data(w)
            torch.nn.functional.mse_loss(model(x), y).backward()
        opt.step(grad_scale=1.0 / workers)
    return flat.param.clone()


@pytest.mark.parametrize("servers", [1, 2])
def test_sync_ps_matches_mean_gradient_adam(tmp_path, servers):
    workers = 2
    res = _run(tmp_path, workers, servers, "sync")
    ref = _reference(workers)
    assert res[0]["nbuckets"] > 2 and res[0]["pieces"] > res[0]["nbuckets"] - 1 + (servers - 1)
    for w in range(workers):
        assert torch.allclose(res[w]["param"], ref, atol=1e-6, rtol=1e-5), (w, (res[w]["param"] - ref).abs().max())
    for s in range(servers):
        r = res[workers + s]
        assert r["updates"] == STEPS
        assert torch.allclose(r["param"], ref[r["lo"]:r["hi"]], atol=1e-6, rtol=1e-5)


def test_sync_ps_async_pull_keeps_loss_trajectory(tmp_path, monkeypatch):
    """PS=1 Worker=2: the parameter pull issued asynchronously and waited
    per bucket by the next forward gives exactly the losses and weights of
    the blocking pull (TOA_PS_BLOCKING_PULL=1), and step() really returns
    with the pull still in flight."""
    workers, servers = 2, 1
    asyn = _run(tmp_path, workers, servers, "sync", tag="a")
    monkeypatch.setenv("TOA_PS_BLOCKING_PULL", "1")
    block = _run(tmp_path, workers, servers, "sync", tag="b")
    for w in range(workers):
        assert asyn[w]["losses"] == block[w]["losses"], w
        assert torch.equal(asyn[w]["param"], block[w]["param"]), w
        assert asyn[w]["pending_after_step"] > 0 and block[w]["pending_after_step"] == 0
    assert asyn[0]["losses"][-1] < asyn[0]["losses"][0]


def test_async_ps_applies_every_push(tmp_path):
    workers, servers = 2, 1
    res = _run(tmp_path, workers, servers, "async")
    ps = res[workers]
    assert ps["updates"] == workers * STEPS
    init = FlatParams(list(reversed(list(_model(seed=0).parameters())))).param
    for w in range(workers):
        assert torch.isfinite(res[w]["param"]).all()
        assert not torch.equal(res[w]["param"], init)
    # the worker served last holds exactly the server's final weights
    assert any(torch.equal(res[w]["param"], ps["param"]) for w in range(workers))


@pytest.mark.parametrize("mode,gpu_ps", [("sync", False), ("async", False), ("sync", True)])
def test_tfjob_ps1_worker2_resnet_e2e(mode, gpu_ps):
    """PS=1 Worker=2 through the operator and the local kubelet.  gpu_ps: every
    replica requests one amd.com/gpu (BASELINE config #2), so the operator puts
    the PS into the world itself (WORLD_SIZE 3, PS rank 2) and the payload only
    checks it; otherwise the CPU PS joins the trainers' gloo world."""
    from tf_operator_amd.sdk import container, pod_template
    from tf_operator_amd.testing.cluster import LocalCluster

    cmd = [sys.executable, "-m", "tf_operator_amd.examples.resnet_train", "--arch", "resnet-tiny", "--image", "32",
           "--batch", "4", "--classes", "10", "--steps", "3", "--warmup", "1", "--ps-mode", mode]
    env = {"OMP_NUM_THREADS": "1", "TOA_NO_GPU": "1", "CUDA_VISIBLE_DEVICES": ""}
    spec = {rt: {"replicas": n, "restartPolicy": "Never",
                 "template": pod_template(container(image="toa/trainer", command=cmd, env=env,
                                                    gpus=1 if gpu_ps else 0))}
            for rt, n in (("PS", 1), ("Worker", 2))}
    name = f"rn-ps-{mode}" + ("-gpu" if gpu_ps else "")
    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
           "spec": {"runPolicy": {"cleanPodPolicy": "None"}, "tfReplicaSpecs": spec}}
    with LocalCluster(gpus=3 if gpu_ps else 0) as c:
        c.client.create(job)
        done = c.client.wait_for_job(name, polling_interval=0.2, timeout_seconds=240)
        conds = [x["type"] for x in done["status"]["conditions"]]
        logs = c.client.get_logs(name, master=False)
        assert conds[-1] == "Succeeded", (conds, logs)
        assert f"[{mode}]" in logs[f"{name}-worker-0"] and "samples/s" in logs[f"{name}-worker-0"], logs
        # the PS applied the optimizer: sync = one update per step, async = one per push
        want = 4 if mode == "sync" else 8
        assert f"ps 0: {want} {mode} updates" in logs[f"{name}-ps-0"], logs
        owner = "operator" if gpu_ps else "payload"
        assert f"ps world ({owner}): 2 trainers + 1 servers, rank 2 of 3" in logs[f"{name}-ps-0"], logs
