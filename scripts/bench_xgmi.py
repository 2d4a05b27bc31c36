"""Latency of the xGMI peer-buffer collectives (csrc/comm/xgmi.hip), 2 processes.

On the 1-GPU box both ranks share the GPU (peer buffers are then local HBM, so this
measures the protocol + kernel cost, not link bandwidth).  Per size: 50 calls captured
in one HIP graph, replayed; reports us/call.  Usage: python scripts/bench_xgmi.py [world]"""
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, op, bytes): op 0 all-gather, 1 one-shot all-reduce, 2 two-shot all-reduce
SIZES = [("lowrank remainder AR one-shot", 1, 25 * 1024), ("lowrank remainder AR two-shot", 2, 25 * 1024),
         ("lowrank gather (fc1+fc2 rows)", 0, 886000),
         ("AR bucket 1 MB one-shot", 1, 1 << 20), ("AR bucket 1 MB two-shot", 2, 1 << 20),
         ("AR full grad 9.1 MB one-shot", 1, 9104880), ("AR full grad 9.1 MB two-shot", 2, 9104880)]


def worker(rank, world, port, q):
    import torch.distributed as dist
    from cloud_server_amd.parallel import xgmi as X
    from cloud_server_amd.utils.graphs import capture
    torch.cuda.set_device(0 if torch.cuda.device_count() == 1 else rank)
    dev = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = X.XgmiComm(rank, world, dev)
    lines = []
    for name, op, nbytes in SIZES:
        n = nbytes // 16 * 4
        x = torch.randn(n, device=dev)
        out = torch.empty(world * n, device=dev)
        ch = comm.channel(name.rsplit(" ", 1)[0], x.nbytes)
        if op == 0:
            call = lambda: ch.all_gather([(x, out)])
        else:
            call = lambda: ch.all_reduce([x], protocol="oneshot" if op == 1 else "twoshot")
        st = torch.cuda.Stream(dev)
        with torch.cuda.stream(st):
            for _ in range(3):
                call()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with capture(g):
            for _ in range(50):
                call()
        g.replay(); torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / 500 * 1e6
        lines.append(f"{name:34s} {x.nbytes / 1e6:7.3f} MB/rank  {us:8.2f} us/call")
    ch_err = sum(c.error() for c in comm.channels.values())
    comm.close()
    dist.destroy_process_group()
    q.put((rank, lines, ch_err))


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r, (l, e)) for r, l, e in (q.get(timeout=200) for _ in range(world)))
    for p in ps:
        p.join(timeout=30)
    print(f"xGMI peer-buffer collectives, world={world}, GPUs visible={torch.cuda.device_count()}")
    for line in res[0][0]:
        print(line)
    print("channel errors:", sum(e for _, e in res.values()))
