"""HBM-resident dataset + device-side batch index stream.

Replaces ``DataSet.next_batch`` (construct_distribute.py:526-569): epoch-shuffled batches
that wrap across epoch ends.  The index stream is the concatenation of per-epoch
permutations, cut into rows of B indices; a device int64 ``cursor`` selects the row, so
the gather + cursor increment live INSIDE the captured HIP graph and a replay needs no
host work.

The row table is double-buffered: ``rows`` holds two halves of ``chunk`` rows and the
device cursor wraps modulo ``2 * chunk``.  While the device consumes one half the host
refills the other from pinned memory with a non-blocking copy, issued only once an event
says the device has finished with that half, so the training loop never waits for the
GPU to drain (a synchronous pageable copy every ``chunk`` steps did).

In data parallel each rank draws a disjoint shard of every epoch permutation (rank r
takes positions r, r+W, ...), i.e. a DistributedSampler over the resident dataset.
"""
from __future__ import annotations

from typing import List, Optional

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
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.rows = torch.zeros(2 * chunk, batch, dtype=torch.int64, device=device)
        self.cursor = torch.zeros(1, dtype=torch.int64, device=device)
        self.wrap = 2 * chunk           # the device cursor runs modulo this
        pin = self.cuda and torch.cuda.is_available()
        self._stage = [torch.zeros(chunk, batch, dtype=torch.int64, pin_memory=pin) for _ in range(2)]
        self._done_ev: List[Optional[torch.cuda.Event]] = [None, None]   # device finished half h
        self._filled = [False, False]
        self.refills = 0
        self.on_reset = None
        self.seek(0)

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
        self.rng = np.random.default_rng(self.seed)   # identical on every rank -> same permutations
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
        if self.cuda:
            torch.cuda.synchronize(self.device)      # nothing in flight reads the halves
        self._done_ev = [None, None]
        self._fill(0)
        self._fill(1)
        self.cursor.zero_()
        self.half, self.used = 0, 0
        if self.on_reset is not None:
            self.on_reset()              # device-side consumers of the cursor (batch staging)

    def _fill(self, h: int) -> None:
        idx = self._next_indices(self.chunk * self.batch).reshape(self.chunk, self.batch)
        st = self._stage[h]
        ev = self._done_ev[h]
        if ev is not None:
            ev.synchronize()             # the previous copy out of this staging buffer is done
        st.copy_(torch.from_numpy(idx))
        self.rows[h * self.chunk:(h + 1) * self.chunk].copy_(st, non_blocking=self.cuda)
        self._filled[h] = True
        self.refills += 1

    def can_group(self, k: int) -> bool:
        """Can the next ``k`` steps be enqueued as ONE launch (a multi-step graph)?  Yes
        when they stay inside one half of the row table, so every before_step() call the
        group makes up front marks and refills exactly what per-step calls would."""
        pos = 0 if self.used >= self.chunk else self.used
        return 1 <= k <= self.chunk and pos + k <= self.chunk

    def before_step(self) -> None:
        """Host-side bookkeeping; call once per step before launching/replaying it."""
        if self.used >= self.chunk:
            # this step enters the other half; the device finishes the old one once every
            # step issued so far has run: mark that point, refill the old half later
            old = self.half
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
                self._done_ev[old] = ev
            self._filled[old] = False
            self.half, self.used = 1 - old, 0
            if not self._filled[self.half]:      # host ran a whole half ahead: wait for it
                self._refill_now(self.half)
        other = 1 - self.half
        if not self._filled[other]:
            ev = self._done_ev[other]
            # the last step of a half already reads the next half's first row (the HIP
            # program stages the NEXT step's batch at the end of each step): that half
            # must be filled before this step is enqueued
            if ev is None or ev.query() or self.used == self.chunk - 1:
                self._refill_now(other)
        self.used += 1

    def _refill_now(self, h: int) -> None:
        ev = self._done_ev[h]
        if ev is not None:
            ev.synchronize()
        self._fill(h)

    def current(self) -> torch.Tensor:
        """Device op (graph-capturable): this step's [B] indices, then cursor += 1 (mod)."""
        idx = self.rows.index_select(0, self.cursor).view(-1)
        self.cursor.add_(1).remainder_(self.wrap)
        return idx
