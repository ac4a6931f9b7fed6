"""Synthetic datasets of the reference payloads' shapes (no network, no
downloads): MNIST-shaped images with a learnable labelling (labels = argmax
of a fixed random projection, so accuracy actually rises), CIFAR/ImageNet
shaped tensors for the CNN/ResNet benchmarks, and token streams for Llama.
Every rank draws a disjoint shard (seeded by rank), like a DistributedSampler.
"""
from __future__ import annotations

import torch


class SyntheticMNIST:
    """pool > 0 on a GPU: the whole synthetic training set (`pool` batches,
    e.g. 600 x 100 = one MNIST epoch, 188 MB) is generated once on the
    device and next() hands out views of it, epoch after epoch -- no host
    work or host-to-device copy per step (what a graph-replayed step needs)."""

    def __init__(self, batch, rank=0, world=1, seed=0, device="cpu", image=False, dtype=torch.float32, pool=0):
        g = torch.Generator().manual_seed(1234)
        self.proj = torch.randn(784, 10, generator=g)
        self.batch = batch
        self.gen = torch.Generator().manual_seed(seed * 1000003 + rank)
        self.device = device
        self.image = image
        self.dtype = dtype
        self.pool = None
        if pool > 0 and torch.device(device).type == "cuda":
            gd = torch.Generator(device=device).manual_seed(seed * 1000003 + rank)
            x = torch.rand(pool, batch, 784, generator=gd, device=device)
            y = (x @ self.proj.to(device)).argmax(-1)
            if image:
                x = x.view(pool, batch, 1, 28, 28)
            self.pool = (x.to(dtype), y)
            self.i = 0

    def next(self):
        if self.pool is not None:
            x, y = self.pool[0][self.i], self.pool[1][self.i]
            self.i = (self.i + 1) % self.pool[0].shape[0]
            return x, y
        x = torch.rand(self.batch, 784, generator=self.gen)
        y = (x @ self.proj).argmax(-1)
        if self.image:
            x = x.view(-1, 1, 28, 28)
        return x.to(self.device, self.dtype), y.to(self.device)

    def __iter__(self):
        while True:
            yield self.next()


class SyntheticImages:
    """ImageNet-shaped (3x224x224) random batches with random labels.

    ``fresh_labels=True`` draws new labels every step (on the device, into
    the same buffer): the images stay resident, but the model cannot
    memorise the batch.  With one fixed batch, Adam drives the loss to ~0
    within ~20 steps and then occasionally blows up into a dead network
    (loss stuck at ~ln(#distinct labels)), with PyTorch's or the fused HIP
    BatchNorm alike (profiles/r2_resnet/divergence_*.log) -- a property of
    memorising random labels, not of the kernels."""

    def __init__(self, batch, shape=(3, 224, 224), classes=1000, rank=0, device="cpu", dtype=torch.bfloat16,
                 channels_last=True, fresh_labels=False):
        g = torch.Generator(device=device).manual_seed(77 + rank)
        self.x = torch.randn(batch, *shape, generator=g, device=device).to(dtype)
        if channels_last:
            self.x = self.x.contiguous(memory_format=torch.channels_last)
        self.y = torch.randint(0, classes, (batch,), generator=g, device=device)
        self.classes, self.fresh, self.g = classes, fresh_labels, g

    def next(self):
        if self.fresh:
            torch.randint(0, self.classes, self.y.shape, generator=self.g, device=self.y.device, out=self.y)
        return self.x, self.y


class SyntheticBinary:
    """keras_model_to_estimator.py:26-33: 1024 x 10 random features, 0/1 labels."""

    def __init__(self, n=1024, batch=32, rank=0, device="cpu"):
        g = torch.Generator().manual_seed(5 + rank)
        self.x = torch.rand(n, 10, generator=g)
        w = torch.randn(10, generator=torch.Generator().manual_seed(9))
        self.y = ((self.x - 0.5) @ w > 0).float()
        self.batch, self.i, self.device = batch, 0, device

    def next(self):
        n = self.x.shape[0]
        idx = torch.arange(self.i, self.i + self.batch) % n
        self.i = (self.i + self.batch) % n
        return self.x[idx].to(self.device), self.y[idx].to(self.device)


class SyntheticTokens:
    """Llama token stream with a resumable position: batch i of rank r is a
    pure function of (seed, r, i), drawn on the device, so ``state_dict()``
    (the cursor) is the whole data state a checkpoint needs -- a resumed run
    reads exactly the batches the uninterrupted run would have read next.

    ``fixed=True`` hands out batch 0 every time (the benchmark's resident
    batch: no generation work inside the timed step)."""

    def __init__(self, micro_batch, seq_len, vocab, rank=0, seed=100, device="cpu", fixed=False):
        self.micro_batch, self.seq_len, self.vocab = micro_batch, seq_len, vocab
        self.rank, self.seed, self.device, self.fixed = rank, seed, torch.device(device), fixed
        self.cursor = 0
        self._fixed = None

    def _draw(self, i):
        g = torch.Generator(device=self.device)
        g.manual_seed((self.seed * 1000003 + self.rank) * 1000003 + i)
        tok = torch.randint(0, self.vocab, (self.micro_batch, self.seq_len + 1), device=self.device, generator=g)
        return tok[:, :-1].contiguous(), tok[:, 1:].contiguous()

    def next(self):
        if self.fixed:
            if self._fixed is None:
                self._fixed = self._draw(0)
            self.cursor += 1
            return self._fixed
        b = self._draw(self.cursor)
        self.cursor += 1
        return b

    def state_dict(self):
        return {"cursor": int(self.cursor), "seed": int(self.seed), "rank": int(self.rank)}

    def load_state_dict(self, sd):
        if sd:
            self.cursor = int(sd.get("cursor", 0))
