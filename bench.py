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
        (N>1: bench.py starts ``torch.distributed.run --nproc-per-node N`` on itself as a
        child process; under an outer torchrun WORLD_SIZE must equal N)

Multi-tenant (one GPU, K independent sample-config jobs; value = aggregate samples/s):
        python bench.py --jobs K --pack graph   # one process, one graph with K branches
        python bench.py --jobs K --pack procs   # K processes, one graph each
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_SAMPLES_PER_S = 50 / 0.14209   # API.md:462-507 (mean of logged durations)


def _sample_cfg(args):
    from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
    cfg_json = dict(SAMPLE_CONFIG)
    cfg_json["optimizer_name"] = args.optimizer
    cfg_json["learning_rate"] = 1e-4 if args.optimizer == "AdagradOptimizer" else 0.01
    cfg_json["options"] = {"batch_size": args.batch}
    return parse_train_config(cfg_json)


def _proc_job(rank, args, barrier, out_q):
    """One packed job as its own process (own HIP context + graph)."""
    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cloud_server_amd.data.datasets import synthetic_mnist
    from cloud_server_amd.runtime.engine import TrainEngine
    cfg = _sample_cfg(args)
    cfg.seed = rank
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    eng = TrainEngine(cfg, synthetic_mnist(60000, seed=rank), device=dev, backend=args.backend,
                      use_graph=not args.no_graph)
    for _ in range(args.warmup):
        eng.step()
    eng.sync_device()
    barrier.wait()
    for _ in range(args.steps):
        eng.step()
    eng.sync_device()
    barrier.wait()
    out_q.put((rank, eng.backend, eng.metrics_since(eng.host_step - min(args.steps, 100))["loss"]))


def bench_packed(args) -> int:
    """K independent jobs on ONE GPU; value = aggregate samples/s of all jobs."""
    if args.gpus != 1:
        raise SystemExit("--jobs packs jobs onto one GPU; run it with --gpus 1")
    K = args.jobs
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if args.pack == "procs":
        import multiprocessing as mp
        ctx = mp.get_context("spawn")        # the parent never touches the GPU
        barrier, out_q = ctx.Barrier(K + 1), ctx.Queue()
        procs = [ctx.Process(target=_proc_job, args=(r, args, barrier, out_q)) for r in range(K)]
        for p in procs:
            p.start()
        barrier.wait()
        t0 = time.perf_counter()
        barrier.wait()
        dt = time.perf_counter() - t0
        res = [out_q.get(timeout=600) for _ in range(K)]
        for p in procs:
            p.join()
        if any(p.exitcode != 0 for p in procs):
            raise SystemExit("a packed job process failed")
        backend = res[0][1]
        loss = sum(r[2] for r in res) / K
    else:
        import torch
        from cloud_server_amd.data.datasets import synthetic_mnist
        from cloud_server_amd.runtime.engine import TrainEngine
        from cloud_server_amd.runtime.multijob import PackedJobs
        dev = "cuda:0" if torch.cuda.is_available() else "cpu"
        engs = []
        for r in range(K):
            cfg = _sample_cfg(args)
            cfg.seed = r
            engs.append(TrainEngine(cfg, synthetic_mnist(60000, seed=r), device=dev,
                                    backend=args.backend, use_graph=not args.no_graph, packed=True))
        pack = PackedJobs(engs)
        pack.step()                       # capture + first step
        pack.prepare_group_graph()        # multi-step graph captured + replayed once, state restored
        pack.run_steps(max(args.warmup - 1, 0))
        pack.sync_device()
        t0 = time.perf_counter()
        pack.run_steps(args.steps)
        pack.sync_device()
        dt = time.perf_counter() - t0
        backend = engs[0].backend
        loss = sum(e.metrics_since(e.host_step - min(args.steps, 100))["loss"] for e in engs) / K
    total = args.batch * K * args.steps / dt
    out = {
        "metric": "train_samples_per_s",
        "value": round(total, 1),
        "unit": "samples/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 5),     # one step of EVERY job
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(total / BASELINE_SAMPLES_PER_S, 2),
        "dtype": "fp32",
        "data": "synthetic (MNIST-shaped 28x28 uint8, 60k samples per job, HBM-resident)",
        "config": {
            "model": "reference sample CNN (API.md:306-332), 2,276,218 params",
            "jobs": K,
            "pack": args.pack,
            "per_job_batch": args.batch,
            "global_batch": args.batch * K,
            "seq_len": None,
            "optimizer": args.optimizer,
            "parallelism": f"{K} independent jobs / 1 GPU",
            "backend": backend,
        },
        "final_loss": round(loss, 4),
    }
    print(json.dumps(out), flush=True)
    return 0


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch_ranks(args):
    """``--gpus N`` means N ranks however bench.py is started.

    * under ``torch.distributed.run`` (``WORLD_SIZE`` set): it must equal ``--gpus``, else
      the run would be mislabelled — exit non-zero;
    * plain ``python bench.py --gpus N`` with N > 1: start ``torch.distributed.run
      --nproc-per-node N`` on this same script as a CHILD process (127.0.0.1 rendezvous on
      a free port) and exit with its return code; the child's rank 0 prints the one JSON
      line on the inherited stdout.  This process has made no GPU call at that point (torch
      is not even imported), so nothing initialised here outlives the hand-off;
    * ``--gpus 1`` without ``WORLD_SIZE``: ``None`` — the single-process path, unchanged.

    Reference: the cluster is the host lists the launcher writes into the worker's flags
    (construct_distribute.py:37-40, :344-346; cmd.py:54-70)."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus:
            print(f"bench.py: WORLD_SIZE={world_env} but --gpus {args.gpus}; launch "
                  f"--nproc-per-node {args.gpus} or pass --gpus {world_env}", file=sys.stderr)
            return 2
        return None
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if args.gpus == 1:
        return None
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, cwd=os.path.dirname(os.path.abspath(__file__))).returncode


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    # auto: "lowrank" data parallelism when world > 1 (dense weight gradients from
    # all-gathered GEMM operands instead of an 8 MB all-reduce; parallel/dp.py), else plain
    ap.add_argument("--strategy", default="auto",
                    choices=["auto", "allreduce", "allreduce:hf", "ps", "ps:hf", "lowrank"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--optimizer", default="AdagradOptimizer")
    ap.add_argument("--jobs", type=int, default=1, help="independent jobs packed on one GPU")
    ap.add_argument("--pack", default="graph", choices=["graph", "procs"])
    args = ap.parse_args()
    if args.jobs > 1:
        return bench_packed(args)
    rc = _launch_ranks(args)
    if rc is not None:
        return rc

    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from cloud_server_amd.data.datasets import synthetic_mnist
    from cloud_server_amd.parallel.dist import all_reduce_max, barrier, init_distributed, shutdown
    from cloud_server_amd.runtime.engine import TrainEngine

    ctx = init_distributed("cuda" if torch.cuda.is_available() else "cpu")
    cfg = _sample_cfg(args)
    ds = synthetic_mnist(60000, seed=0)   # MNIST-shaped synthetic data (no network here)
    tuning = {}
    if args.strategy == "auto":
        # N > 1: time lowrank (all-gather the dense GEMM operands, W x fc1 wgrad FLOPs) vs
        # allreduce (9.1 MB gradient, one-/two-shot xGMI or RCCL per bucket) on a few real
        # steps and keep the faster (parallel/strategy.py; same answer on every rank)
        from cloud_server_amd.parallel.strategy import pick_strategy
        args.strategy, tuning = pick_strategy(cfg, ds, ctx, backend=args.backend)
    eng = TrainEngine(cfg, ds, device=ctx.device, ctx=ctx, backend=args.backend,
                      use_graph=not args.no_graph, strategy=args.strategy)

    # run_steps: exactly K steps; on one GPU groups of CSA_GRAPH_STEPS steps replay one
    # multi-step graph and the remainder the k/2, k/4, .. 2-step graphs (runtime/engine.py)
    eng.step()                          # capture + first step (the single-step graph's first replay)
    if args.steps <= 64 and os.environ.get("CSA_BENCH_ONE_GRAPH", "1") == "1":
        # a short timed loop (the driver's K = 20) is ONE K-step graph replay: no gaps
        # between graph launches inside the timed region (K real steps either way)
        eng.extra_group_sizes = [args.steps]
    eng.prepare_group_graph()           # every multi-step graph captured AND replayed once
                                        # (state restored): no first launch in the timed loop
    eng.run_steps(max(args.warmup - 1, 0))
    eng.sync_device()
    barrier(ctx)
    eng.sync_device()
    t0 = time.perf_counter()
    eng.run_steps(args.steps)
    eng.sync_device()
    barrier(ctx)
    eng.sync_device()
    dt = time.perf_counter() - t0
    dt = all_reduce_max(ctx, dt)
    dt_train = None
    if eng.extra_group_sizes:
        # the same K steps again through the graph sizes training's run_steps uses (32, 16,
        # .., 2: no K-step graph) — reported beside the headline
        eng.extra_group_sizes = []
        barrier(ctx)
        eng.sync_device()
        t1 = time.perf_counter()
        eng.run_steps(args.steps)
        eng.sync_device()
        barrier(ctx)
        eng.sync_device()
        dt_train = all_reduce_max(ctx, time.perf_counter() - t1)
    # a timed-out xGMI peer wait or in-kernel tail wait (skipped updates) invalidates the
    # run: fail loudly (agreed by every rank under data parallelism)
    eng.check_health()
    m = eng.metrics_since(eng.host_step - min(args.steps, 100))

    total = args.batch * ctx.world * args.steps / dt
    pg = "none"
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        pg = torch.distributed.get_backend()
        pg = "rccl" if pg == "nccl" else pg          # the "nccl" backend IS RCCL on ROCm
    if ctx.rank == 0:
        out = {
            "metric": "train_samples_per_s",
            "value": round(total, 1),
            "unit": "samples/s",
            "n_gpus": ctx.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt * 1e3 / args.steps, 5),
            # the same K steps replayed as training's graph sizes (null: K > 64, already so)
            "ms_per_step_training_graphs": None if dt_train is None else round(dt_train * 1e3 / args.steps, 5),
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
                "collectives": {t: ("xgmi" if c is not None else pg) for t, c in eng.sync._choice.items()}
                               or (pg if ctx.world > 1 else "none"),
                "xgmi": eng.sync.xgmi_reason,
                "collective_tuning_us": eng.sync.xgmi_tuning,
                "strategy_tuning_ms_per_step": tuning,
                # CSA_DIST_SHARED_GPU=1 (parallel/dist.py): every rank on ONE GPU over a gloo
                # group — a rehearsal of the N-rank code path, NOT an N-GPU measurement
                **({"rehearsal": f"{ctx.world} ranks sharing one GPU (CSA_DIST_SHARED_GPU=1): not a multi-GPU number"}
                   if os.environ.get("CSA_DIST_SHARED_GPU") == "1" and ctx.world > 1 else {}),
            },
            "final_loss": round(m["loss"], 4),
            "final_batch_accuracy": round(m["accuracy"], 4),
        }
        print(json.dumps(out), flush=True)
    shutdown(ctx)
    return 0


if __name__ == "__main__":
    sys.exit(main())
