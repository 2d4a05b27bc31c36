"""xGMI peer-buffer collectives (csrc/comm/xgmi.hip) with two real processes.

Both ranks run on the box's one MI355X (the IPC mapping, flag protocol, double
buffering and device-side epoch are the same whether the peer's buffer sits on this
GPU or across an xGMI link); handles travel over a gloo group.  Checked against exact
host-side expectations: multi-segment all-gather, fp32 all-reduce, 60 back-to-back calls
alternating buffer parity, calls captured in a HIP graph and replayed, and the bounded
wait (a missing peer poisons the channel instead of hanging the GPU)."""
import os
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _worker(rank: int, world: int, port: int, q) -> None:
    import torch.distributed as dist
    from cloud_server_amd.parallel import xgmi as X
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        comm = X.XgmiComm(rank, world, dev)
        res = {"self_test": X.self_test(comm)}

        # multi-segment all-gather (the lowrank [B, in] + [B, out] pair shape)
        a = torch.randn(50, 3920, device=dev, generator=torch.Generator(dev).manual_seed(rank))
        b = torch.randn(50, 512, device=dev, generator=torch.Generator(dev).manual_seed(100 + rank))
        oa = torch.empty(world * 50, 3920, device=dev)
        ob = torch.empty(world * 50, 512, device=dev)
        g = comm.channel("g", a.nbytes + b.nbytes)
        g.all_gather([(a, oa), (b, ob)])
        ra = [torch.randn(50, 3920, device=dev, generator=torch.Generator(dev).manual_seed(r)) for r in range(world)]
        rb = [torch.randn(50, 512, device=dev, generator=torch.Generator(dev).manual_seed(100 + r)) for r in range(world)]
        torch.cuda.synchronize()
        res["gather"] = torch.equal(oa, torch.cat(ra)) and torch.equal(ob, torch.cat(rb))

        # all-reduce, two segments, fixed rank order
        s = comm.channel("s", 2 * 4 * 6400)
        x1 = torch.full((6400,), float(rank + 1), device=dev)
        x2 = torch.arange(6400, dtype=torch.float32, device=dev) * (rank + 1)
        s.all_reduce([x1, x2])
        torch.cuda.synchronize()
        tot = sum(r + 1 for r in range(world))
        res["allreduce"] = torch.equal(x1, torch.full_like(x1, float(tot))) and \
            torch.equal(x2, torch.arange(6400, dtype=torch.float32, device=dev) * tot)

        # 60 back-to-back calls without host sync (parity alternation, epoch counter)
        ok = True
        outs = []
        for i in range(60):
            v = torch.full((4096,), float(i * 10 + rank), device=dev)
            o = torch.empty(world * 4096, device=dev)
            g.all_gather([(v, o)])
            outs.append((i, o))
        torch.cuda.synchronize()
        for i, o in outs:
            ok &= all(torch.all(o[r * 4096:(r + 1) * 4096] == i * 10 + r).item() for r in range(world))
        res["sequence"] = ok

        # captured in a HIP graph, replayed with new inputs
        inp = torch.zeros(8192, device=dev)
        red = torch.zeros(8192, device=dev)
        gout = torch.empty(world * 8192, device=dev)
        gr = comm.channel("graph", inp.nbytes)
        st = torch.cuda.Stream(dev)
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):           # warm-up (channel 'graph_ar' created off-graph)
            gr.all_gather([(inp, gout)])
            comm.channel("graph_ar", red.nbytes).all_reduce([red])
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            gr.all_gather([(inp, gout)])
            red.copy_(inp)
            comm.channel("graph_ar", red.nbytes).all_reduce([red])
        ok = True
        for it in range(20):
            inp.fill_(float(it * 100 + rank))
            graph.replay()
            torch.cuda.synchronize()
            for r in range(world):
                ok &= bool(torch.all(gout[r * 8192:(r + 1) * 8192] == it * 100 + r).item())
            ok &= bool(torch.all(red == sum(it * 100 + r for r in range(world))).item())
        res["graph"] = ok
        res["errors"] = sum(ch.error() for ch in comm.channels.values())

        # bounded wait: rank 0 calls alone on a short-timeout channel
        t = X.XgmiChannel(rank, world, 4096, dev, timeout_s=0.5)
        dist.barrier()
        if rank == 0:
            v = torch.ones(1024, device=dev)
            o = torch.empty(world * 1024, device=dev)
            t0 = time.time()
            t.all_gather([(v, o)])
            torch.cuda.synchronize()
            first = time.time() - t0
            t0 = time.time()
            t.all_gather([(v, o)])       # poisoned: returns at once
            torch.cuda.synchronize()
            res["timeout"] = (t.error() == 1, first, time.time() - t0)
        dist.barrier()
        t.close()
        comm.close()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, {"exception": traceback.format_exc()}))


def test_xgmi_two_processes():
    if os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY") is None:
        os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, d = q.get(timeout=100)
            res[r] = d
    finally:
        for p in ps:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
    for r in range(2):
        assert "exception" not in res[r], res[r].get("exception")
        for k in ("self_test", "gather", "allreduce", "sequence", "graph"):
            assert res[r][k], (r, k, res[r])
        assert res[r]["errors"] == 0, res[r]
    poisoned, first, second = res[0]["timeout"]
    assert poisoned and 0.3 < first < 5.0 and second < 0.5, res[0]["timeout"]
