"""Data-parallel gradient synchronisation strategies over RCCL/xGMI.

Reference: asynchronous between-graph replication through a parameter server —
``replica_device_setter`` puts every variable on ``/job:ps`` and each worker pulls
vars / pushes grads over gRPC per ``sess.run`` (construct_distribute.py:355-357, 413;
SURVEY.md §2.3).  On one MI355X node that becomes:

* ``allreduce`` (default) — synchronous DP: every rank holds the params; the flat fp32
  gradient buffer is summed with RCCL all-reduce in a few large buckets (xGMI ring
  collectives are per-link bound, so few large messages beat many small ones).  The
  1/world averaging factor is folded into the loss-gradient seed, so the all-reduced
  SUM is already the mean and no extra scaling pass is needed.
* ``ps`` — the parameter-server capability, sharded and synchronous (ZeRO-1 style):
  reduce-scatter gradients to each rank's owned shard, the owner applies the fused
  optimizer to its shard only (optimizer slots exist only for the shard, the PS
  analogue of accumulators living on ``/job:ps``), then all-gather the new params.
* ``lowrank`` — exact sync DP for the dense layers at small per-rank batch: a dense
  weight gradient is ``Xᵀ·dY`` with K = per-rank batch, so instead of all-reducing the
  [in, out] gradient we all-gather the [B, in] activations and [B, out] output grads
  and every rank forms the global ``Xᵀ·dY`` locally (K = world·B).  For the sample
  config fc1 that is 0.9 MB gathered per rank instead of an 8 MB all-reduce.

All strategies are written against ``torch.distributed`` so the identical code runs on
gloo (CPU tests) and RCCL (MI355X).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from .dist import DistContext

DEFAULT_BUCKET_BYTES = 32 << 20   # one bucket covers the sample model's 9.1 MB gradient


class GradSync:
    def __init__(self, ctx: DistContext, numel: int, strategy: str = "allreduce",
                 bucket_bytes: int = DEFAULT_BUCKET_BYTES):
        if strategy not in ("allreduce", "ps", "lowrank"):
            raise ValueError(f"unknown DP strategy {strategy!r}")
        self.ctx, self.numel, self.strategy = ctx, numel, strategy
        if strategy == "ps" and ctx.enabled and numel % ctx.world:
            raise ValueError("ps strategy needs the flat buffer padded to a multiple of world")
        self.shard = numel // ctx.world if ctx.enabled else numel
        self.bucket_elems = max(1, bucket_bytes // 4)
        # grouped RCCL launches for the multi-tensor lowrank collectives (opt-in: a grouped
        # collective inside HIP-graph capture crashed capture_end on ROCm 7 / torch 2.10)
        self.coalesce = ctx.backend == "nccl" and os.environ.get("CSA_COALESCE", "0") == "1"

    @property
    def grad_scale(self) -> float:
        """Factor folded into dL/dlogits so that SUM-reduced grads are the global mean."""
        return 1.0 / self.ctx.world if self.ctx.enabled else 1.0

    def shard_range(self) -> Tuple[int, int]:
        if self.strategy != "ps" or not self.ctx.enabled:
            return 0, self.numel
        r = self.ctx.rank
        return r * self.shard, (r + 1) * self.shard

    def buckets(self, lo: int = 0, hi: Optional[int] = None) -> List[Tuple[int, int]]:
        hi = self.numel if hi is None else hi
        out, o = [], lo
        while o < hi:
            out.append((o, min(hi, o + self.bucket_elems)))
            o = out[-1][1]
        return out

    # ---- allreduce ----
    def allreduce(self, flat_grad: torch.Tensor, lo: int = 0, hi: Optional[int] = None) -> None:
        if not self.ctx.enabled:
            return
        for a, b in self.buckets(lo, hi):
            dist.all_reduce(flat_grad[a:b])

    # ---- ps (sharded) ----
    def reduce_scatter(self, flat_grad: torch.Tensor, shard_out: torch.Tensor) -> None:
        if not self.ctx.enabled:
            shard_out.copy_(flat_grad)
            return
        dist.reduce_scatter_tensor(shard_out, flat_grad)

    def all_gather_params(self, flat_param: torch.Tensor) -> None:
        if not self.ctx.enabled:
            return
        lo, hi = self.shard_range()
        dist.all_gather_into_tensor(flat_param, flat_param[lo:hi].clone()
                                    if self.ctx.backend == "gloo" else flat_param[lo:hi])

    # ---- lowrank ----
    def all_gather_rows(self, local: torch.Tensor, out: torch.Tensor) -> None:
        """[B, n] per rank -> [world*B, n] (rank-major)."""
        if not self.ctx.enabled:
            out.copy_(local)
            return
        dist.all_gather_into_tensor(out, local.contiguous())

    def all_gather_rows_many(self, pairs) -> None:
        """Several ``all_gather_rows`` issued as ONE grouped RCCL launch where the backend
        supports coalescing (each separate collective pays its own fixed latency)."""
        if not self.ctx.enabled:
            for local, out in pairs:
                out.copy_(local)
            return
        if self.coalesce and len(pairs) > 1:
            with dist._coalescing_manager(async_ops=False):
                for local, out in pairs:
                    dist.all_gather_into_tensor(out, local.contiguous())
            return
        for local, out in pairs:
            dist.all_gather_into_tensor(out, local.contiguous())

    def allreduce_ranges(self, flat: torch.Tensor, ranges) -> None:
        """Sum-all-reduce the given [lo, hi) slices of ``flat`` (one grouped launch on RCCL)."""
        if not self.ctx.enabled or not ranges:
            return
        if self.coalesce and len(ranges) > 1:
            with dist._coalescing_manager(async_ops=False):
                for lo, hi in ranges:
                    dist.all_reduce(flat[lo:hi])
            return
        for lo, hi in ranges:
            dist.all_reduce(flat[lo:hi])

    def broadcast_params(self, flat_param: torch.Tensor) -> None:
        """Initial sync from rank 0 (reference: chief runs init_op, construct_distribute.py:379)."""
        if self.ctx.enabled:
            dist.broadcast(flat_param, src=0)
