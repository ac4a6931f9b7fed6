"""MXJob payload (API parity): the ps-lite ``dist_sync``
kvstore pattern on the operator's MXNet env contract (MX_CONFIG + DMLC_*,
reference pkg/controller.v1/mxnet/mxnet.go:55-233).

* scheduler (DMLC_ROLE=scheduler, listens on DMLC_PS_ROOT_PORT): rendezvous
  and shutdown -- waits for every worker's DONE, then stops the servers;
* server: one contiguous shard of the flat parameters, synchronous update
  of the mean of DMLC_NUM_WORKER pushes (tf_operator_amd.parallel.ps);
* worker: trains the MNIST MLP, push gradients / pull parameters per step.

CPU only (MXNet has no ROCm build here); the MI355X path is all-reduce DP.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import time

import numpy as np
import torch

from tf_operator_amd.models.vision import MnistMLP
from tf_operator_amd.ops.llm import cross_entropy
from tf_operator_amd.ops.mlp import accuracy
from tf_operator_amd.parallel.ps import ParameterServer, PSClient, shard_sizes
from tf_operator_amd.train.data import SyntheticMNIST
from tf_operator_amd.train.dist import own_port, resolve_endpoint


def _cluster():
    cfg = json.loads(os.environ.get("MX_CONFIG", "{}") or "{}")
    return cfg.get("cluster", {}), cfg.get("task", {})


def _flat(model):
    return torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).numpy()


def _load(model, flat):
    off = 0
    with torch.no_grad():
        for p in model.parameters():
            n = p.numel()
            p.copy_(torch.from_numpy(flat[off:off + n]).view_as(p))
            off += n


def _connect(host, port, tries=600):
    for _ in range(tries):
        try:
            return socket.create_connection((host, port), timeout=30)
        except OSError:
            time.sleep(0.1)
    raise SystemExit(f"cannot reach {host}:{port}")


def run_scheduler(n_workers):
    srv = socket.socket()
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind(("0.0.0.0", int(os.environ.get("DMLC_PS_ROOT_PORT", "9091"))))
    srv.listen(64)
    done = 0
    while done < n_workers:
        c, _ = srv.accept()
        if c.recv(16).startswith(b"DONE"):
            done += 1
        c.close()
    print(f"[scheduler] all {n_workers} workers done", flush=True)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--lr", type=float, default=0.01)
    a = ap.parse_args(argv)
    role = os.environ.get("DMLC_ROLE", "worker")
    n_workers = int(os.environ.get("DMLC_NUM_WORKER", "1"))
    n_servers = int(os.environ.get("DMLC_NUM_SERVER", "1"))
    cluster, task = _cluster()
    torch.manual_seed(0)
    model = MnistMLP(100, dtype=torch.float32, device="cpu")
    flat0 = _flat(model)
    sizes = shard_sizes(flat0.size, n_servers)
    if role == "scheduler":
        run_scheduler(n_workers)
        # stop the servers once training is over
        eps = [resolve_endpoint(f"{u['url']}:{u['port']}") for u in cluster.get("server", [])]
        PSClient(eps, sizes).stop_servers()
        return
    if role == "server":
        idx = int(task.get("index", 0))
        off = sum(sizes[:idx])
        ps = ParameterServer(flat0[off:off + sizes[idx]], lr=a.lr, sync_replicas=n_workers,
                             port=own_port(9091))
        print(f"[server {idx}] shard of {sizes[idx]} params, dist_sync over {n_workers} workers", flush=True)
        ps.serve_forever()
        return
    wid = int(os.environ.get("DMLC_WORKER_ID", task.get("index", 0)))
    eps = [resolve_endpoint(f"{u['url']}:{u['port']}") for u in cluster.get("server", [])]
    client = None
    for _ in range(600):
        try:
            client = PSClient(eps, sizes)
            break
        except OSError:
            time.sleep(0.1)
    if client is None:
        raise SystemExit("servers unreachable")
    _load(model, client.pull())
    data = SyntheticMNIST(a.batch, wid, n_workers)
    for s in range(1, a.steps + 1):
        x, y = data.next()
        model.zero_grad(set_to_none=True)
        loss = cross_entropy(model(x), y)
        loss.backward()
        g = np.concatenate([p.grad.float().reshape(-1).numpy() for p in model.parameters()])
        _load(model, client.push(g))
        if s % 50 == 0:
            print(f"[worker {wid}] step {s} loss {float(loss):.4f}", flush=True)
    x, y = SyntheticMNIST(2000, rank=10_000).next()
    with torch.no_grad():
        acc = float(accuracy(model(x), y))
    print(f"[worker {wid}] accuracy {acc:.3f}", flush=True)
    host, port = os.environ.get("DMLC_PS_ROOT_URI", "127.0.0.1"), int(os.environ.get("DMLC_PS_ROOT_PORT", "9091"))
    with _connect(host, port) as c:
        c.sendall(b"DONE")


if __name__ == "__main__":
    main()
