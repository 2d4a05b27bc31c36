"""SyncBN on the HIP program with two real ranks (both on the box's one MI355X, gloo
process group, eager steps): the forward statistic slabs, the backward statistic slabs
and the BN parameter gradients must follow the global batch.  Reference: the PyTorch
path of the same 2-rank job, whose SyncBN is pinned against the single-process full
batch on CPU (tests/test_distributed.py::test_sync_bn_equals_full_batch)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NETS = {
    "sample": None,
    "norm_before_conv": [
        {"layer": "conv", "filter": [2, 2, 6]},
        {"layer": "norm"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [3, 3, 12], "isBias": "True"},
        {"layer": "active"},
        {"layer": "pool", "kernel": [3, 3], "stride": [2, 2]},
        {"layer": "norm"},
        {"layer": "connect", "hidden": 100},
        {"layer": "active", "active_func": "sigmoid"},
    ],
}


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from cloud_server_amd.data.datasets import synthetic_mnist
    from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
    from cloud_server_amd.parallel.dist import DistContext
    from cloud_server_amd.runtime.engine import TrainEngine
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        ctx = DistContext(rank, world, 0, "gloo", torch.device("cuda", 0))
        ds = synthetic_mnist(400, seed=3)
        res = {}
        for name, layers in NETS.items():
            raw = dict(SAMPLE_CONFIG, optimizer_name="GradientDescentOptimizer", learning_rate=0.5,
                       options={"batch_size": 25, "sync_bn": True})
            if layers is not None:
                raw["net_config"] = {"middle_layer": layers}
            cfg = parse_train_config(raw)
            out = {}
            for backend in ("hip", "torch"):
                eng = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend=backend, use_graph=False)
                assert eng.backend == backend, eng.fallback_reason
                assert eng.model.sync_bn
                w0 = eng.flat.clone()
                eng.step()
                eng.sync_device()               # (lands a deferred dense update)
                out[backend] = (eng, w0, eng.flat.clone())
            eh, w0h, w1h = out["hip"]
            et, w0t, w1t = out["torch"]
            worst = 0.0
            for k in eh.model.state.shapes:
                a = eh.model.state.view(k, (w0h - w1h) / 0.5)
                b = et.model.state.view(k, (w0t - w1t) / 0.5)
                scale = b.abs().max().item() + 1e-6
                worst = max(worst, (a - b).abs().max().item() / scale)
            bufs = all(torch.allclose(x, y, atol=1e-5, rtol=1e-4)
                       for (_, x), (_, y) in zip(eh.model.named_buffers(), et.model.named_buffers()))
            res[name] = (worst, bufs)
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, {"exception": traceback.format_exc()}))


def test_sync_bn_hip_matches_torch_two_ranks():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, d = q.get(timeout=110)
            res[r] = d
    finally:
        for p in ps:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
    for r in range(2):
        assert "exception" not in res[r], res[r]["exception"]
        for name, (worst, bufs) in res[r].items():
            assert worst <= 2e-3, (r, name, worst)
            assert bufs, (r, name, "running BN statistics differ")
