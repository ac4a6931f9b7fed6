"""XGBoostJob payload (API parity): distributed histogram
gradient boosting with a Rabit-style allreduce, on the operator's XGBoost
env contract (MASTER_ADDR/MASTER_PORT/WORLD_SIZE/RANK, reference
pkg/controller.v1/xgboost/xgboost.go:14-135).

Every rank holds a row shard of a synthetic binary-classification matrix.
Per boosting round and tree level each rank builds (gradient, hessian)
histograms over quantised feature bins for every open node; one allreduce
sums them (the Rabit step of XGBoost's ``hist`` method), after which every
rank picks the same best splits, so the trees are identical everywhere
without shipping data.  A "step" = one boosting round.  CPU + gloo.
"""
from __future__ import annotations

import argparse
import os
import time

import numpy as np
import torch
import torch.distributed as dist


def make_data(n, f, rank, seed=7):
    rng = np.random.default_rng(seed + 1000 * rank)
    x = rng.normal(size=(n, f)).astype(np.float32)
    w = np.random.default_rng(seed).normal(size=f)
    logit = x @ w + 0.5 * np.sin(3 * x[:, 0]) * x[:, 1]
    y = (logit + 0.3 * rng.normal(size=n) > 0).astype(np.float32)
    return x, y


def allreduce(a: np.ndarray) -> np.ndarray:
    if dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy()
    return a


class Tree:
    def __init__(self, depth):
        self.depth = depth
        self.feat = np.full(2 ** depth - 1, -1, np.int32)
        self.thr = np.zeros(2 ** depth - 1, np.int32)
        self.leaf = np.zeros(2 ** depth, np.float32)

    def predict_bins(self, xb):
        node = np.zeros(xb.shape[0], np.int64)
        for _ in range(self.depth):
            f = self.feat[node]
            go_right = np.where(f >= 0, xb[np.arange(xb.shape[0]), np.maximum(f, 0)] > self.thr[node], False)
            node = 2 * node + 1 + go_right
        return self.leaf[node - (2 ** self.depth - 1)]


def grow(xb, g, h, depth, nbins, lam=1.0, eta=0.3):
    n, f = xb.shape
    tree = Tree(depth)
    node = np.zeros(n, np.int64)
    for level in range(depth):
        first = 2 ** level - 1
        nodes = 2 ** level
        local = node - first
        hist = np.zeros((nodes, f, nbins, 2), np.float64)
        for j in range(f):
            idx = (local * nbins + xb[:, j]).astype(np.int64)
            hist[:, j, :, 0] = np.bincount(idx, weights=g, minlength=nodes * nbins).reshape(nodes, nbins)
            hist[:, j, :, 1] = np.bincount(idx, weights=h, minlength=nodes * nbins).reshape(nodes, nbins)
        hist = allreduce(hist)  # the Rabit step
        cg, ch = np.cumsum(hist[..., 0], axis=2), np.cumsum(hist[..., 1], axis=2)
        G, Hs = cg[:, :, -1:], ch[:, :, -1:]
        gain = cg ** 2 / (ch + lam) + (G - cg) ** 2 / (Hs - ch + lam) - G ** 2 / (Hs + lam)
        gain[:, :, -1] = -np.inf
        for k in range(nodes):
            j, b = np.unravel_index(np.argmax(gain[k]), gain[k].shape)
            if gain[k, j, b] > 1e-6:
                tree.feat[first + k], tree.thr[first + k] = j, b
        f_of = tree.feat[node]
        right = np.where(f_of >= 0, xb[np.arange(n), np.maximum(f_of, 0)] > tree.thr[node], False)
        node = 2 * node + 1 + right
    leaf = node - (2 ** depth - 1)
    gs = allreduce(np.bincount(leaf, weights=g, minlength=2 ** depth))
    hs = allreduce(np.bincount(leaf, weights=h, minlength=2 ** depth))
    tree.leaf[:] = (-eta * gs / (hs + lam)).astype(np.float32)
    return tree


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--rows", type=int, default=20000, help="rows per rank")
    ap.add_argument("--features", type=int, default=16)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--bins", type=int, default=32)
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    x, y = make_data(a.rows, a.features, rank)
    # global quantile bin edges from a small allreduced sample (sketch)
    edges = np.quantile(x[: min(2000, len(x))], np.linspace(0, 1, a.bins + 1)[1:-1], axis=0)
    edges = allreduce(edges) / world
    xb = np.stack([np.searchsorted(edges[:, j], x[:, j]) for j in range(a.features)], 1).astype(np.int32)
    pred = np.zeros(len(y), np.float32)
    t0 = time.time()
    for r in range(1, a.rounds + 1):
        p = 1 / (1 + np.exp(-pred))
        tree = grow(xb, (p - y).astype(np.float64), (p * (1 - p)).astype(np.float64), a.depth, a.bins)
        pred += tree.predict_bins(xb)
        if r % 5 == 0 or r == a.rounds:
            p = 1 / (1 + np.exp(-pred))
            ll = allreduce(np.array([-(y * np.log(p + 1e-9) + (1 - y) * np.log(1 - p + 1e-9)).sum(),
                                     ((p > 0.5) == y).sum(), len(y)]))
            if rank == 0:
                print(f"[xgboost rank 0/{world}] round {r} logloss {ll[0] / ll[2]:.4f} acc {ll[1] / ll[2]:.3f} "
                      f"({(time.time() - t0) / r * 1e3:.1f} ms/round)", flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
