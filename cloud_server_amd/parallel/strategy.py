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
from typing import Dict, Optional, Sequence, Tuple

import torch

from .dist import DistContext, all_reduce_max, barrier


def time_strategy(cfg, ds, ctx: DistContext, strategy: str, steps: int = 30, warmup: int = 5,
                  backend: str = "auto") -> float:
    """Seconds per step of ``strategy`` (max over ranks); ``inf`` for a ":hf" trial whose
    engine did not come out as the :hf program (no HIP program, or its hfuse / tail-fold
    preconditions failed) — it would only time a duplicate of the plain strategy."""
    from ..runtime.engine import TrainEngine
    eng = TrainEngine(cfg, ds, device=ctx.device, ctx=ctx, backend=backend, strategy=strategy)
    if strategy.endswith(":hf"):
        built = bool(getattr(getattr(eng, "program", None), "dp_hf", False))
        if all_reduce_max(ctx, 0.0 if built else 1.0) > 0.0:   # the same answer on every rank
            if eng.sync is not None and eng.sync.xgmi is not None:
                barrier(ctx)
                eng.sync.xgmi.close()
            del eng
            return float("inf")
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


# Rough MI355X rates for the start-up pruning below (measured in profiles/: the dense
# weight-gradient kernels reach 27-35 TFLOP/s of f32 MFMA on these shapes; one xGMI link
# moves ~153 GB/s and a fully connected node's peer-buffer collectives use all W - 1 links)
F32_GEMM_FLOPS = 30e12
XGMI_LINK_BPS = 153e9


def lowrank_worth_trying(cfg, world: int) -> bool:
    """False when lowrank's extra weight-gradient FLOPs — every rank forms the GLOBAL dense
    gradient with K = world x B instead of B — already cost more than moving the dense
    gradient bytes over the links would (2 (W-1)/W of it per rank, spread over W-1 links),
    so a W-GPU job does not pay a 30-step trial for a strategy that cannot win.  At B = 50
    on the sample CNN that keeps lowrank at W = 2 (7 us of extra GEMM vs 52 us on one
    link) and drops it at W = 8 (47 us vs 13 us)."""
    from ..models.cnn import build_model
    if world <= 1:
        return False
    B = cfg.batch_size
    plan = build_model(cfg).plan
    dense = [lp for lp in plan.layers if type(lp.spec).__name__ == "DenseSpec"]
    extra_flops = sum(2.0 * (world - 1) * B * lp.in_shape.numel * lp.spec.hidden for lp in dense)
    grad_bytes = sum(4.0 * lp.in_shape.numel * lp.spec.hidden for lp in dense)
    t_gemm = extra_flops / F32_GEMM_FLOPS
    t_links = 2.0 * (world - 1) / world * grad_bytes / ((world - 1) * XGMI_LINK_BPS)
    return t_gemm <= t_links


def default_candidates(cfg, world: int, gpu: bool = False) -> Tuple[str, ...]:
    """lowrank where it can win, allreduce, and ps (the parameter-server capability:
    bucketed reduce-scatter to owner shards overlapped with the backward, owner-side
    optimizer, xGMI all-gather — construct_distribute.py:355-357, 413), each also as its
    ":hf" program: the one-GPU step's structure (dense weight gradients inside the pair
    backward launch, fewer and shorter launches) at the price of one exchange after the
    backward instead of buckets overlapped with it — which wins depends on the link time
    (``gpu``: the ":hf" programs exist on the HIP program only)."""
    base = ("allreduce", "allreduce:hf", "ps", "ps:hf") if gpu else ("allreduce", "ps")
    return (("lowrank",) + base) if lowrank_worth_trying(cfg, world) else base


def pick_strategy(cfg, ds, ctx: DistContext, candidates: Optional[Sequence[str]] = None,
                  steps: int = 30, backend: str = "auto") -> Tuple[str, Dict[str, float]]:
    """(fastest strategy, {strategy: ms per step}) — identical on every rank.  Default
    candidates: ``default_candidates`` (lowrank only where it can win)."""
    if not ctx.enabled:
        return "allreduce", {}
    if candidates is None:
        candidates = default_candidates(cfg, ctx.world, gpu=ctx.device.type == "cuda")
    candidates = tuple(candidates)
    if len(candidates) == 1:
        return candidates[0], {}
    times = {s: time_strategy(cfg, ds, ctx, s, steps=steps, backend=backend) * 1e3 for s in candidates}
    best = min(candidates, key=lambda s: (times[s], candidates.index(s)))
    # (a skipped ":hf" trial is reported as null)
    return best, {k: (round(v, 4) if v != float("inf") else None) for k, v in times.items()}
