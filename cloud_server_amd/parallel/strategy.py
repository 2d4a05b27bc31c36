"""Start-up choice of the data-parallel strategy for a job, by measurement.

Two strategies move the sample CNN's dense gradients very differently:

* ``allreduce`` — every rank forms its own weight gradients (K = B) and the whole 9.1 MB
  gradient is all-reduced (RCCL, or the xGMI one-/two-shot peer-buffer kernels picked per
  bucket by ``GradSync``'s tuner);
* ``lowrank`` — the dense layers' GEMM operands (X [B, in], dY [B, out]: 0.9 MB) are
  all-gathered instead, and every rank forms the GLOBAL weight gradient itself with
  K = world x B — W x the fc1 weight-gradient FLOPs, but ~10x fewer bytes on the links.

Which wins depends on world size, link bandwidth and the GEMM's cost, so instead of a
rule this module times a few real training steps of each candidate (HIP graph replays,
max over ranks — every rank gets the same answer) and returns the fastest.  Reference:
the PS push/pull of the whole gradient every step (construct_distribute.py:355-357, 413).
"""
from __future__ import annotations

import time
from typing import Dict, Sequence, Tuple

import torch

from .dist import DistContext, all_reduce_max, barrier


def time_strategy(cfg, ds, ctx: DistContext, strategy: str, steps: int = 30, warmup: int = 5,
                  backend: str = "auto") -> float:
    """Seconds per step of ``strategy`` (max over ranks)."""
    from ..runtime.engine import TrainEngine
    eng = TrainEngine(cfg, ds, device=ctx.device, ctx=ctx, backend=backend, strategy=strategy)
    for _ in range(warmup):
        eng.step()
    eng.sync_device()
    barrier(ctx)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    eng.sync_device()
    dt = (time.perf_counter() - t0) / steps
    if eng.sync is not None:
        eng.sync.check()
        if eng.sync.xgmi is not None:      # free this engine's peer buffers on every rank
            barrier(ctx)
            eng.sync.xgmi.close()
    del eng
    if ctx.device.type == "cuda":
        torch.cuda.empty_cache()
    return all_reduce_max(ctx, dt)


def pick_strategy(cfg, ds, ctx: DistContext, candidates: Sequence[str] = ("lowrank", "allreduce"),
                  steps: int = 30, backend: str = "auto") -> Tuple[str, Dict[str, float]]:
    """(fastest strategy, {strategy: ms per step}) — identical on every rank."""
    if not ctx.enabled:
        return "allreduce", {}
    times = {s: time_strategy(cfg, ds, ctx, s, steps=steps, backend=backend) * 1e3 for s in candidates}
    best = min(candidates, key=lambda s: (times[s], candidates.index(s)))
    return best, {k: round(v, 4) for k, v in times.items()}
