#!/usr/bin/env python3
"""Headline benchmark: training throughput of the reference sample config.

Metric: training samples/s of the API.md:306-332 sample CNN
(conv[2,2,10] -> conv[2,2,20] -> pool -> norm -> sigmoid -> fc512 -> fc512 -> fc10,
2,276,218 params, fp32) at the reference batch of 50 per worker with Adagrad (the
optimizer the reference actually runs, construct_distribute.py:372).  Reference:
≈352 samples/s (B=50 / 0.14209 s mean step, API.md:462-507).

Weak scaling: every rank trains B=50 per step on its own shard of a synthetic
MNIST-shaped dataset resident in HBM; gradients are all-reduced over RCCL/xGMI every
step (synchronous DP), so ``value`` is the whole-job samples/s.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        (N>1: torchrun --nproc-per-node N ... bench.py --gpus N)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_SAMPLES_PER_S = 50 / 0.14209   # API.md:462-507 (mean of logged durations)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    # auto: "lowrank" data parallelism when world > 1 (dense weight gradients from
    # all-gathered GEMM operands instead of an 8 MB all-reduce; parallel/dp.py), else plain
    ap.add_argument("--strategy", default="auto", choices=["auto", "allreduce", "ps", "lowrank"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--optimizer", default="AdagradOptimizer")
    args = ap.parse_args()

    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cloud_server_amd.data.datasets import synthetic_mnist
    from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
    from cloud_server_amd.parallel.dist import all_reduce_max, barrier, init_distributed, shutdown
    from cloud_server_amd.runtime.engine import TrainEngine

    ctx = init_distributed("cuda" if torch.cuda.is_available() else "cpu")
    if args.strategy == "auto":
        args.strategy = "lowrank" if ctx.world > 1 else "allreduce"
    cfg_json = dict(SAMPLE_CONFIG)
    cfg_json["optimizer_name"] = args.optimizer
    cfg_json["learning_rate"] = 1e-4 if args.optimizer == "AdagradOptimizer" else 0.01
    cfg_json["options"] = {"batch_size": args.batch}
    cfg = parse_train_config(cfg_json)
    ds = synthetic_mnist(60000, seed=0)   # MNIST-shaped synthetic data (no network here)
    eng = TrainEngine(cfg, ds, device=ctx.device, ctx=ctx, backend=args.backend,
                      use_graph=not args.no_graph, strategy=args.strategy)

    for _ in range(args.warmup):
        eng.step()
    eng.sync_device()
    barrier(ctx)
    eng.sync_device()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step()
    eng.sync_device()
    barrier(ctx)
    eng.sync_device()
    dt = time.perf_counter() - t0
    dt = all_reduce_max(ctx, dt)
    if eng.sync is not None:
        eng.sync.check()   # a timed-out xGMI peer wait invalidates the run: fail loudly
    m = eng.metrics_since(eng.host_step - min(args.steps, 100))

    total = args.batch * ctx.world * args.steps / dt
    if ctx.rank == 0:
        out = {
            "metric": "train_samples_per_s",
            "value": round(total, 1),
            "unit": "samples/s",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt * 1e3 / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(total / BASELINE_SAMPLES_PER_S, 2),
            "dtype": "fp32",
            "data": "synthetic (MNIST-shaped 28x28 uint8, 60k samples, HBM-resident)",
            "config": {
                "model": "reference sample CNN (API.md:306-332), 2,276,218 params",
                "global_batch": args.batch * ctx.world,
                "seq_len": None,
                "per_gpu_batch": args.batch,
                "optimizer": cfg.effective_optimizer,
                "parallelism": f"dp{ctx.world}" + ("" if args.strategy == "allreduce" else f"-{args.strategy}"),
                "backend": eng.backend,
                "hip_graph": eng.use_graph,
                # per call site: xGMI peer-buffer kernel or RCCL, and (CSA_XGMI=auto) the
                # start-up timings that decided it
                "collectives": {t: ("xgmi" if c is not None else "rccl") for t, c in eng.sync._choice.items()}
                               or ("rccl" if ctx.world > 1 else "none"),
                "xgmi": eng.sync.xgmi_reason,
                "collective_tuning_us": eng.sync.xgmi_tuning,
            },
            "final_loss": round(m["loss"], 4),
            "final_batch_accuracy": round(m["accuracy"], 4),
        }
        print(json.dumps(out), flush=True)
    shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
