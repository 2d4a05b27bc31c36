"""HBM-resident dataset + device-side batch index stream.

Replaces ``DataSet.next_batch`` (construct_distribute.py:526-569): epoch-shuffled batches
that wrap across epoch ends.  The index stream is the concatenation of per-epoch
permutations, cut into ``[chunk, B]`` rows; a device int64 ``cursor`` selects the row,
so the gather + cursor increment live INSIDE the captured HIP graph and a replay needs
no host work.  The host only refills the stream every ``chunk`` steps.

In data parallel each rank draws a disjoint shard of every epoch permutation (rank r
takes positions r, r+W, ...), i.e. a DistributedSampler over the resident dataset.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .datasets import ArrayDataset


class DeviceDataset:
    def __init__(self, ds: ArrayDataset, device):
        self.n = len(ds)
        self.images = torch.from_numpy(np.ascontiguousarray(ds.images)).to(device)       # uint8 [N,784]
        self.labels = torch.from_numpy(np.ascontiguousarray(ds.labels)).to(device)       # int64 [N]
        self.labels32 = self.labels.to(torch.int32)
        self.device = torch.device(device)

    def batch(self, idx: torch.Tensor):
        x = self.images.index_select(0, idx).to(torch.float32).mul_(1.0 / 255.0)
        return x, self.labels.index_select(0, idx)


class BatchStream:
    def __init__(self, n: int, batch: int, device, seed: int = 0, chunk: int = 512,
                 rank: int = 0, world: int = 1):
        if n <= 0:
            raise ValueError("empty dataset")
        self.n, self.batch, self.chunk = n, batch, chunk
        self.rank, self.world = rank, world
        self.seed = seed
        self.rng = np.random.default_rng(seed)   # identical on every rank -> same permutations
        self.pending = np.zeros(0, np.int64)
        self.rows = torch.zeros(chunk, batch, dtype=torch.int64, device=device)
        self.cursor = torch.zeros(1, dtype=torch.int64, device=device)
        self.used = chunk  # forces a refill on first use
        self.epochs = 0

    def _next_indices(self, count: int) -> np.ndarray:
        need = count * self.world
        parts = [self.pending]
        have = len(self.pending)
        while have < need:
            p = self.rng.permutation(self.n)
            self.epochs += 1
            parts.append(p)
            have += len(p)
        allidx = np.concatenate(parts)
        take, self.pending = allidx[:need], allidx[need:]
        return take[self.rank::self.world]

    def seek(self, step: int) -> None:
        """Position the stream so the next step is global step ``step`` of an unbroken
        run (exact resume): step s always consumes positions [s*B*W, (s+1)*B*W) of the
        permutation sequence, so replay the generator and drop what was consumed."""
        self.rng = np.random.default_rng(self.seed)
        self.pending = np.zeros(0, np.int64)
        self.epochs = 0
        skip = step * self.batch * self.world
        while skip > 0:
            p = self.rng.permutation(self.n)
            self.epochs += 1
            if skip < len(p):
                self.pending = p[skip:]
                break
            skip -= len(p)
        self.used = self.chunk            # next before_step() refills from here

    def refill(self) -> None:
        idx = self._next_indices(self.chunk * self.batch).reshape(self.chunk, self.batch)
        self.rows.copy_(torch.from_numpy(idx), non_blocking=False)
        self.cursor.zero_()
        self.used = 0

    def before_step(self) -> None:
        """Host-side bookkeeping; call once per step before launching/replaying it."""
        if self.used >= self.chunk:
            self.refill()
        self.used += 1

    def current(self) -> torch.Tensor:
        """Device op (graph-capturable): this step's [B] indices, then cursor += 1."""
        idx = self.rows.index_select(0, self.cursor).view(-1)
        self.cursor.add_(1)
        return idx
