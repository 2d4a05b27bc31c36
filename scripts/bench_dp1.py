#!/usr/bin/env python3
"""Data-parallel code path on ONE GPU: a world-1 RCCL process group with a context that
reports DP as enabled (as tests/test_gpu_dp_overlap.py), timed like bench.py.  Measures
what the DP program costs over the 1-GPU program at the same config (the driver's
N-GPU runs add only the collectives' link time on top of this).

    python scripts/bench_dp1.py [--strategy lowrank|allreduce|ps] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--strategy", default="lowrank")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--xgmi", default="auto")
    a = ap.parse_args()
    os.environ["CSA_XGMI"] = a.xgmi
    import torch
    import torch.distributed as dist
    from cloud_server_amd.data.datasets import synthetic_mnist
    from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
    from cloud_server_amd.parallel.dist import DistContext
    from cloud_server_amd.runtime.engine import TrainEngine

    class DPContext(DistContext):
        @property
        def enabled(self) -> bool:
            return True

    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    from cloud_server_amd.parallel.dist import rccl_env_defaults
    rccl_env_defaults()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-4,
                                      options={"batch_size": 50}))
        ctx = DPContext(rank=0, world=1, local_rank=0, backend="nccl", device=dev)
        eng = TrainEngine(cfg, synthetic_mnist(60000, seed=0), device=dev, ctx=ctx, backend="hip",
                          strategy=a.strategy)
        eng.step()
        eng.prepare_group_graph()
        eng.run_steps(a.warmup - 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run_steps(a.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        eng.sync.check()
        print(json.dumps({"strategy": a.strategy, "ms_per_step": round(dt * 1e3 / a.steps, 5),
                          "samples_per_s": round(50 * a.steps / dt, 1), "group_steps": eng.group_steps(),
                          "collectives": {t: ("xgmi" if c is not None else "rccl") for t, c in eng.sync._choice.items()},
                          "lr_update": [bool(getattr(u, "lr_update", False)) for u in eng.program.lr_units],
                          "loss": round(eng.metrics_since(eng.host_step - 100)["loss"], 4)}), flush=True)
    finally:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
