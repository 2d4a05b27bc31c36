#!/usr/bin/env python3
"""Do two processes sharing ONE GPU run their kernels concurrently?  (profiles/r5_notes.md)

Each probe: both ranks open an xGMI channel (3 s bounded waits), line up on the host, then
one rank delays its call by --delay seconds while the other calls at once and spins on the
peer's flag.  The per-block records (one device-wide 100 MHz clock for both processes) give
when each rank's kernel started and whether the early rank's wait ended by the peer's
arrival or by the timeout.  Variants: `--busy MS` keeps a compute kernel running on a
second stream of the LATE rank during its delay (a rank busy in its own backward)."""
import argparse
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, delay, busy_ms, reps, q):
    import torch
    import torch.distributed as dist
    os.environ.update(HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from cloud_server_amd.parallel import xgmi as X
        from cloud_server_amd.ops import fused as K
        K.load(required=True)
        ch = X.XgmiChannel(rank, world, 4096, dev, timeout_s=3.0)
        v = torch.ones(1024, device=dev)
        o = torch.empty(world * 1024, device=dev)
        a = torch.randn(2048, 2048, device=dev)
        out = []
        for rep in range(reps):
            late = rep % world                     # who delays, alternating
            torch.cuda.synchronize()
            dist.barrier()
            if rank == late:
                if busy_ms > 0:                    # own compute kernels during the delay
                    st = torch.cuda.Stream(dev)
                    with torch.cuda.stream(st):
                        t0 = time.perf_counter()
                        while (time.perf_counter() - t0) * 1e3 < busy_ms:
                            a = a @ a * 1e-3
                time.sleep(delay)
            t_host = time.time()
            ch.all_gather([(v, o)])
            torch.cuda.synchronize()
            d = ch.diag()
            out.append({"rep": rep, "late": late, "t_host": t_host, "t_start": min(r["t_start"] for r in d),
                        "t_wait": max(r["t_wait"] for r in d), "status": sorted({r["status"] for r in d}),
                        "err": ch.error()})
            if ch.error():
                break
        ch.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception:
        import traceback
        q.put((rank, {"exception": traceback.format_exc()[-1500:]}))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--delay", type=float, default=1.0)
    ap.add_argument("--busy", type=float, default=0.0)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, a.delay, a.busy, a.reps, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(a.world):
            r, d = q.get(timeout=120)
            res[r] = d
    finally:
        for p in ps:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
    rows = []
    if all(isinstance(res.get(r), list) for r in range(a.world)):
        for i in range(min(len(res[r]) for r in range(a.world))):
            late = res[0][i]["late"]
            early = [r for r in range(a.world) if r != late]
            t0 = min(res[r][i]["t_start"] for r in early)
            rows.append({"rep": i, "late_rank": late,
                         "late_start_after_early_s": round((res[late][i]["t_start"] - t0) / 1e8, 4),
                         "early_wait_s": round((max(res[r][i]["t_wait"] for r in early) - t0) / 1e8, 4),
                         "status": {r: res[r][i]["status"] for r in range(a.world)}})
    print(json.dumps({"world": a.world, "delay_s": a.delay, "busy_ms": a.busy, "probes": rows,
                      "raw": res if not rows else None}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
