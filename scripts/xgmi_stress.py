#!/usr/bin/env python3
"""Stress of the overlapped xGMI data-parallel step with W ranks sharing ONE GPU — the
configuration in which round 4 lost peer flags — recording the per-block diagnostics of
every channel when a peer wait times out (profiles/r5_notes.md).

    python scripts/xgmi_stress.py --world 2 --steps 300 [--strategy allreduce|ps]

Variants come from the environment: CSA_XGMI_BLOCKS (co-resident cap; 0 = none),
CSA_KERNEL_LIB (a kernel-library variant, e.g. round 4's xGMI kernels).  Prints one JSON
line: per rank {"ok", "timeouts": {channel: diag summary}, "ms_per_step"}."""
import argparse
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, steps, strategy, q, chunk=25):
    import torch
    import torch.distributed as dist
    os.environ.update(CSA_XGMI="1", LOCAL_WORLD_SIZE=str(world), HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from cloud_server_amd.data.datasets import synthetic_mnist
        from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
        from cloud_server_amd.parallel.dist import DistContext
        from cloud_server_amd.runtime.engine import TrainEngine
        cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-3,
                                      options={"batch_size": 50}))
        ctx = DistContext(rank=rank, world=world, local_rank=0, backend="nccl", device=dev)
        eng = TrainEngine(cfg, synthetic_mnist(4000, seed=0), device="cuda:0", ctx=ctx, backend="hip",
                          strategy=strategy)
        if strategy == "async_ps":
            assert eng.aps is not None and type(eng.aps).__name__ == "AsyncPSDevice"
        else:
            assert eng.sync.xgmi is not None, eng.sync.xgmi_reason
            assert eng.program.overlap or os.environ.get("CSA_DP_OVERLAP") == "0"

        def poisoned() -> bool:
            if eng.aps is not None:
                return bool(eng.aps.error())
            return any(c.error() for c in eng.sync.xgmi.channels.values())
        eng.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        done = 1
        bad = False
        import faulthandler
        os.makedirs("gpurun_out", exist_ok=True)
        hang_fh = open(f"gpurun_out/xgmi_stress_host_{world}_{rank}.txt", "w")
        slow_host = []                       # (step, host call, seconds) of calls > 0.1 s
        chunks = []                          # ms per step of each 25-step chunk
        while done < steps:
            n = min(chunk, steps - done)
            tc = time.perf_counter()
            for i in range(n):
                # a host call that blocks > 0.5 s leaves its Python stack in the dump file
                faulthandler.dump_traceback_later(0.5, file=hang_fh)
                th = time.perf_counter()
                eng.step()
                faulthandler.cancel_dump_traceback_later()
                w = time.perf_counter() - th
                if w > 0.1:
                    slow_host.append((done + i, "step", round(w, 3)))
            done += n
            faulthandler.dump_traceback_later(0.5, file=hang_fh)
            th = time.perf_counter()
            torch.cuda.synchronize()
            faulthandler.cancel_dump_traceback_later()
            if time.perf_counter() - th > 0.1:
                slow_host.append((done, "sync", round(time.perf_counter() - th, 3)))
            chunks.append(round((time.perf_counter() - tc) * 1e3 / n, 3))
            if poisoned():
                bad = True
                break
        dt = time.perf_counter() - t0
        res = {"ok": not bad, "steps": done, "ms_per_step": round(dt * 1e3 / max(done - 1, 1), 3),
               "chunk_ms": chunks, "slow_host": slow_host}
        if eng.aps is not None:
            res.update(staleness=eng.staleness(), aps_blocks=eng.aps.nb)
            eng.finish_async()
            eng.close()
            dist.destroy_process_group()
            q.put((rank, res))
            return
        res["blocks"] = {t: c.blocks_for(c.slot_bytes) for t, c in eng.sync.xgmi.channels.items()}
        if bad:
            res["timeouts"] = {t: c.diag_summary() for t, c in eng.sync.xgmi.channels.items()}
            os.makedirs("gpurun_out", exist_ok=True)
            with open(f"gpurun_out/xgmi_stress_diag_{world}_{rank}.json", "w") as fh:
                json.dump({t: c.diag() for t, c in eng.sync.xgmi.channels.items()}, fh)
        eng.close()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:
        import traceback
        q.put((rank, {"exception": traceback.format_exc()[-2000:]}))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--strategy", default="allreduce")
    ap.add_argument("--chunk", type=int, default=25, help="steps enqueued between host syncs")
    ap.add_argument("--rank", type=int, default=-1,
                    help="run ONE rank in this process (with --port), e.g. each under its own profiler")
    ap.add_argument("--port", type=int, default=0)
    a = ap.parse_args()
    if a.rank >= 0:
        class _Q:
            def put(self, item):
                print(json.dumps({"rank": item[0], "res": item[1]}), flush=True)
        worker(a.rank, a.world, a.port, a.steps, a.strategy, _Q(), a.chunk)
        return 0
    import torch.multiprocessing as mp
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, a.steps, a.strategy, q, a.chunk)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(a.world):
            r, d = q.get(timeout=300)
            res[r] = d
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    print(json.dumps({"world": a.world, "steps": a.steps, "strategy": a.strategy,
                      "blocks_cap": os.environ.get("CSA_XGMI_BLOCKS", "0"),
                      "lib": os.path.basename(os.environ.get("CSA_KERNEL_LIB", "") or "default"),
                      "ranks": res}), flush=True)
    return 0 if all(d.get("ok") for d in res.values()) and len(res) == a.world else 1


if __name__ == "__main__":
    sys.exit(main())
