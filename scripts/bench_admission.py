#!/usr/bin/env python3
"""Packed-host admission / retirement stall on one GPU (VERDICT r2 "cheap admission").

K sample-config jobs run packed (``PackedJobs``, the ``gpu_host`` loop's data path) in
8-step graph launches.  Then, like ``gpu_host.serve`` does between launches:
  * admission: a (K+1)-th job is built (engine + HBM dataset), the pack is rebuilt and the
    next launch re-captures (only the NEW engine warms up);
  * retirement: one job leaves, the pack is rebuilt, the next launch re-captures.
Printed per event: engine build, first packed step (warm-up + single-step capture), first
8-step launch (multi-step capture), and the steady 8-step launch for comparison — the
stall every other tenant sees is the sum of the first two columns beyond steady state.

Usage: python scripts/bench_admission.py [--jobs 4] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from cloud_server_amd.data.datasets import synthetic_mnist
    from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
    from cloud_server_amd.runtime.engine import TrainEngine
    from cloud_server_amd.runtime.multijob import PackedJobs

    os.environ.setdefault("CSA_GRAPH_STEPS", "8")
    dev = "cuda:0"

    def cfg(seed):
        c = dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-4,
                 options={"batch_size": 50})
        p = parse_train_config(c)
        p.seed = seed
        return p

    def build(seed):
        t0 = time.perf_counter()
        e = TrainEngine(cfg(seed), synthetic_mnist(60000, seed=seed), device=dev, backend="hip", use_graph=True,
                        packed=True)
        torch.cuda.synchronize()
        return e, (time.perf_counter() - t0) * 1e3

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    engines = [build(i)[0] for i in range(a.jobs)]
    pack = PackedJobs(engines)
    pack.step()
    pack.run_steps(8)
    steady = min(timed(lambda: pack.run_steps(8)) for _ in range(20))
    rows = []
    seed = 100
    for rep in range(a.reps):
        for event in ("admit", "retire"):
            if event == "admit":
                e, t_build = build(seed)
                seed += 1
                engines.append(e)
            else:
                engines.pop(0)
                t_build = 0.0
            pack = PackedJobs(engines)                       # what gpu_host does on a change
            t_first = timed(pack.step)                       # warm-up (new engine only) + capture
            t_group = timed(lambda: pack.run_steps(8))       # multi-step graph capture + 8 steps
            t_steady = min(timed(lambda: pack.run_steps(8)) for _ in range(5))
            rows.append({"event": event, "jobs": len(engines), "build_ms": round(t_build, 2),
                         "first_step_ms": round(t_first, 2), "first_group_ms": round(t_group, 2),
                         "steady_group_ms": round(t_steady, 3),
                         "stall_ms": round(t_first + t_group - t_steady, 2)})
            print(json.dumps(rows[-1]), flush=True)
    import gc
    t0 = time.perf_counter(); gc.collect(); t_gc = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"gc_collect_ms": round(t_gc, 2), "steady_group_ms_K": round(steady, 3), "jobs": a.jobs,
                      "mean_stall_ms_admit": round(sum(r["stall_ms"] for r in rows if r["event"] == "admit") / a.reps, 2),
                      "mean_stall_ms_retire": round(sum(r["stall_ms"] for r in rows if r["event"] == "retire") / a.reps, 2)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
