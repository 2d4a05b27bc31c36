"""Multi-process data parallel on CPU (gloo, world_size 2) — the same code paths the
MI355X node runs over RCCL/xGMI.

Pins: (1) the collective building blocks; (2) sync DP with 2 ranks x B equals one
process with 2B on the same samples (no BN => order-independent batch mean); (3) the
sharded "ps" strategy (reduce-scatter -> owner optimizer -> all-gather, the reference's
parameter-server capability) produces the same weights as all-reduce;
(4) a distributed training job writes the reference result.txt from rank 0 only and
checkpoints/resumes with sharded optimizer state."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import parse_train_config

CFG = {"iter": 12, "learning_rate": 0.05, "ratio": 0.8, "loss_name": "entropy",
       "optimizer_name": "AdagradOptimizer",
       "options": {"log_every": 4, "ckpt_every": 4, "batch_size": 8},
       "net_config": {"middle_layer": [{"layer": "conv", "filter": [3, 3, 4], "isBias": "True"},
                                       {"layer": "active", "active_func": "relu"},
                                       {"layer": "pool"},
                                       {"layer": "connect", "hidden": 24},
                                       {"layer": "active", "active_func": "sigmoid"}]}}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    torch.set_num_threads(1)            # world 8 on an 8-CPU box: no oversubscription
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from cloud_server_amd.parallel.dist import init_distributed
    return init_distributed("cpu", timeout_s=120)


def _collectives(rank, world, port, out):
    import torch.distributed as dist
    from cloud_server_amd.parallel.dp import GradSync
    ctx = _init(rank, world, port)
    n = 64 * world
    gs = GradSync(ctx, n, "ps", bucket_bytes=40)
    g = torch.arange(n, dtype=torch.float32) * (rank + 1)
    shard = torch.zeros(n // world)
    gs.reduce_scatter(g, shard)
    lo, hi = gs.shard_range()
    exp = torch.arange(n, dtype=torch.float32)[lo:hi] * sum(range(1, world + 1))
    ok = torch.allclose(shard, exp)
    p = torch.zeros(n)
    p[lo:hi] = rank + 1.0
    gs.all_gather_params(p)
    ok &= torch.equal(p, torch.repeat_interleave(torch.arange(1.0, world + 1), n // world))
    ga = GradSync(ctx, n, "allreduce", bucket_bytes=40)       # 10-element buckets
    assert len(ga.buckets()) == -(-n // 10)
    g2 = torch.ones(n) * (rank + 1)
    ga.allreduce(g2)
    ok &= torch.allclose(g2, torch.full((n,), float(sum(range(1, world + 1)))))
    rows = torch.full((3, 5), float(rank))
    allrows = torch.zeros(3 * world, 5)
    ga.all_gather_rows(rows, allrows)
    ok &= all(torch.equal(allrows[3 * r:3 * r + 3], torch.full((3, 5), float(r))) for r in range(world))
    # lowrank identity: sum_r X_r^T dY_r == X_all^T dY_all with rank-major gathered rows
    gen = torch.Generator().manual_seed(rank)
    x, dy = torch.randn(4, 6, generator=gen), torch.randn(4, 3, generator=gen)
    xa, dya = torch.zeros(4 * world, 6), torch.zeros(4 * world, 3)
    ga.all_gather_rows_many([(x, xa), (dy, dya)])
    g_ar = x.t() @ dy
    dist.all_reduce(g_ar)
    ok &= torch.allclose(xa.t() @ dya, g_ar, atol=1e-5)
    # bucketed reduce-scatter to owners: suffix ranges (as the backward produces them)
    # cover the buffer and end as the whole-buffer reduce-scatter
    g3 = torch.arange(n, dtype=torch.float32) * (rank + 1) + 0.5
    sh3 = torch.zeros(n // world)
    for lo, hi in ((n - 7 * 4, n), (20, n - 7 * 4), (0, 20)):
        gs.reduce_scatter_range(g3, sh3, lo, hi)
    ref3 = torch.zeros(n // world)
    gs.reduce_scatter(g3.clone(), ref3)
    ok &= torch.allclose(sh3, ref3)
    flat = torch.arange(12, dtype=torch.float32) * (rank + 1)
    ga.allreduce_ranges(flat, [(0, 3), (8, 12)])
    s = float(sum(range(1, world + 1)))
    ok &= torch.equal(flat[:3], torch.arange(3.0) * s) and torch.equal(flat[8:], torch.arange(8.0, 12.0) * s)
    ok &= torch.equal(flat[3:8], torch.arange(3.0, 8.0) * (rank + 1))
    out[rank] = bool(ok)
    dist.destroy_process_group()


def _train(rank, world, port, strategy, steps, out):
    from cloud_server_amd.parallel.dist import shutdown
    from cloud_server_amd.runtime.engine import TrainEngine
    ctx = _init(rank, world, port)
    cfg = parse_train_config(CFG)
    eng = TrainEngine(cfg, synthetic_mnist(256, seed=1), device="cpu", ctx=ctx, strategy=strategy)
    for _ in range(steps):
        eng.step()
    out[rank] = eng.flat.clone()
    shutdown(ctx)


def _spawn(fn, world, *args):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(fn, args=(world, _port(), *args, out), nprocs=world, join=True)
    return dict(out)


def _share_gpu(rank, world, port, buses, out):
    """ranks_share_gpu with faked device properties: each rank reports PCI bus buses[rank]."""
    from types import SimpleNamespace
    from cloud_server_amd.parallel import dist as D
    ctx = _init(rank, world, port)
    props = SimpleNamespace(pci_domain_id=0, pci_bus_id=buses[rank], pci_device_id=0, uuid=f"gpu{buses[rank]}")
    torch.cuda.get_device_properties = lambda dev=None: props
    out[rank] = D.ranks_share_gpu(ctx, torch.device("cuda", 0))
    D.shutdown(ctx)


@pytest.mark.parametrize("buses,want", [((3, 3), True), ((3, 4), False)])
def test_ranks_share_gpu_compares_pci_locations(buses, want):
    """The shared-GPU launch profile (profiles/r5_notes.md) is chosen only when another
    rank of the job drives the SAME physical GPU: ranks all-gather their PCI locations."""
    out = _spawn(_share_gpu, 2, buses)
    assert out == {0: want, 1: want}


def test_collectives_world2():
    out = _spawn(_collectives, 2)
    assert out == {0: True, 1: True}


def test_allreduce_dp_equals_single_process_big_batch():
    out = _spawn(_train, 2, "allreduce", 6)
    torch.testing.assert_close(out[0], out[1], rtol=0, atol=0)          # replicas identical
    # single process, batch 2B over the same per-step sample sets
    from cloud_server_amd.runtime.engine import TrainEngine
    cfg = parse_train_config(dict(CFG, options=dict(CFG["options"], batch_size=16)))
    eng = TrainEngine(cfg, synthetic_mnist(256, seed=1), device="cpu")
    n = eng.flat.numel()
    torch.testing.assert_close(eng.flat, _init_flat()[:n])     # same seed -> same init as rank 0
    for _ in range(6):
        eng.step()
    torch.testing.assert_close(out[0][:n], eng.flat, rtol=2e-4, atol=2e-5)


def _init_flat():
    from cloud_server_amd.models.cnn import build_model
    return build_model(parse_train_config(CFG)).flat.detach()


def test_ps_strategy_matches_allreduce():
    a = _spawn(_train, 2, "allreduce", 5)
    b = _spawn(_train, 2, "ps", 5)
    torch.testing.assert_close(b[0], b[1], rtol=0, atol=0)
    n = min(a[0].numel(), b[0].numel())
    torch.testing.assert_close(a[0][:n], b[0][:n], rtol=1e-5, atol=1e-6)


def test_collectives_world4():
    """More ranks than the 2-rank default: bucket, reduce-scatter, gather and range
    collectives at world 4 (the 8-GPU path, rehearsed on CPU)."""
    out = _spawn(_collectives, 4)
    assert out == {r: True for r in range(4)}


def test_ps_matches_allreduce_world4():
    a = _spawn(_train, 4, "allreduce", 3)
    b = _spawn(_train, 4, "ps", 3)
    for r in range(1, 4):
        torch.testing.assert_close(a[0], a[r], rtol=0, atol=0)
        torch.testing.assert_close(b[0], b[r], rtol=0, atol=0)
    n = min(a[0].numel(), b[0].numel())
    torch.testing.assert_close(a[0][:n], b[0][:n], rtol=1e-5, atol=1e-6)


def _job(rank, world, port, mdir, cfg, out):
    from cloud_server_amd.parallel.dist import shutdown
    from cloud_server_amd.runtime.trainer import run_job
    ctx = _init(rank, world, port)
    ds = synthetic_mnist(300, seed=2)
    res = run_job(mdir, cfg, device="cpu", ctx=ctx, backend="torch", data=ds.split(0.8))
    out[rank] = res["step"]
    shutdown(ctx)


def test_distributed_job_rank0_writes_and_ps_resume(tmp_path):
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    cfg = dict(CFG, options=dict(CFG["options"], strategy="ps"))
    out = _spawn(_job, 2, mdir, cfg)
    assert out == {0: 12, 1: 12}
    lines = open(os.path.join(mdir, "result.txt")).read().splitlines()
    assert [l.split(",")[0] for l in lines[:4]] == ["step:0", "step:4", "step:8", "step:12"]   # one writer
    assert lines[4].startswith("final_accuracy:")
    from cloud_server_amd.runtime import checkpoint as ckpt
    obj = ckpt.load(ckpt.latest(mdir)[1])
    full = obj["slots"]
    assert full.dim() == 2
    half = full.shape[1] // 2
    assert (full[:, :half] > 0).all() and (full[:, half:] > 0).all()   # both ranks' shards saved
    out = _spawn(_job, 2, mdir, dict(cfg, iter=16))
    assert out == {0: 16, 1: 16}


BN_CFG = {"iter": 4, "learning_rate": 0.01, "ratio": 0.8, "loss_name": "entropy",
          "optimizer_name": "AdamOptimizer", "options": {"batch_size": 6, "sync_bn": True},
          "net_config": {"middle_layer": [{"layer": "conv", "filter": [3, 3, 4], "isBias": "True"},
                                          {"layer": "norm"},
                                          {"layer": "active", "active_func": "relu"},
                                          {"layer": "pool"},
                                          {"layer": "connect", "hidden": 16}]}}


def _sync_bn(rank, world, port, out):
    _sync_bn_w(rank, world, port, out)


def _sync_bn_w(rank, world, port, out):
    """SyncBN: each rank normalises its half of the batch with the GLOBAL statistics; the
    forward equals the single-process full batch and the all-reduced mean gradient
    equals the full-batch gradient."""
    import torch.distributed as dist
    from cloud_server_amd.models.cnn import build_model, loss_fn
    _init(rank, world, port)
    cfg = parse_train_config(BN_CFG)
    assert cfg.sync_bn
    g = torch.Generator().manual_seed(7)
    X = torch.rand(6 * world, 28, 28, 1, generator=g)
    Y = torch.randint(0, 10, (6 * world,), generator=g)
    ref = build_model(cfg)
    ref.train()
    lr = ref(X)
    loss_fn("entropy", lr, Y).backward()
    net = build_model(cfg)
    net.train()
    net.sync_bn = True
    sl = slice(rank * 6, (rank + 1) * 6)
    logits = net(X[sl])
    (loss_fn("entropy", logits, Y[sl]) / world).backward()
    dist.all_reduce(net.flat.grad)
    rm = [n for n, _ in net.named_buffers() if n.endswith("_mean")][0]
    out[rank] = (torch.allclose(logits, lr[sl].detach(), atol=1e-5),
                 float((net.flat.grad - ref.flat.grad).abs().max()),
                 float(ref.flat.grad.abs().max()),
                 torch.allclose(getattr(net, rm), getattr(ref, rm), atol=1e-6))


def test_sync_bn_equals_full_batch():
    out = _spawn(_sync_bn, 2)
    for r in range(2):
        fwd_ok, gdiff, gmax, run_ok = out[r]
        assert fwd_ok, r
        assert gdiff <= 1e-5 * max(1.0, gmax), (r, gdiff, gmax)
        assert run_ok, r


def _agreed_error(rank, world, port, out):
    """a peer-buffer timeout seen by ONE rank (here a fake poisoned channel on
    rank 1) must raise on EVERY rank together, after the last log step too."""
    from cloud_server_amd.parallel.dp import GradSync
    from cloud_server_amd.parallel.dist import shutdown
    ctx = _init(rank, world, port)
    gs = GradSync(ctx, 16, "allreduce")

    class _Ch:
        def __init__(self, err):
            self.err = err

        def error(self):
            return self.err

    class _Comm:
        channels = {"ar": _Ch(1 if rank == 1 else 0)}

        def check(self):
            pass

    gs.check_agreed()                       # no channels: fine on every rank
    gs.xgmi = _Comm()
    try:
        gs.check_agreed()
        out[rank] = "no-raise"
    except RuntimeError:
        out[rank] = "raised"
    shutdown(ctx)


def test_xgmi_error_agreed_across_ranks():
    out = _spawn(_agreed_error, 2)
    assert out == {0: "raised", 1: "raised"}


# ---------------------------------------------------------------------------------------
# World-8 rehearsal of the 8-GPU node (VERDICT r3 "next" #4): every strategy and SyncBN at
# the width the driver's scaling run uses, on gloo.  Reference: the PS/worker host lists
# (construct_distribute.py:37-40, 344-345) — scaling by adding workers.
W8_CFG = dict(CFG, options=dict(CFG["options"], batch_size=50))


def _named(eng):
    return {k: eng.model.state.view(k, eng.flat).detach().clone() for k in eng.model.state.shapes}


def _train_strategies(rank, world, port, steps, out):
    from cloud_server_amd.parallel.dist import shutdown
    from cloud_server_amd.runtime.engine import TrainEngine
    ctx = _init(rank, world, port)
    cfg = parse_train_config(W8_CFG)
    res = {}
    for strategy in ("allreduce", "ps", "lowrank"):
        eng = TrainEngine(cfg, synthetic_mnist(800, seed=1), device="cpu", ctx=ctx, strategy=strategy)
        for _ in range(steps):
            eng.step()
        res[strategy] = _named(eng)
    out[rank] = res
    shutdown(ctx)


def test_world8_strategies_equal_single_process_400_batch():
    """8 ranks x B=50 with allreduce, ps (reduce-scatter -> owner Adagrad -> all-gather) and
    lowrank each equal ONE process training on the 400-sample global batch (3 steps, across
    an epoch boundary of the 800-sample set); replicas are identical."""
    from cloud_server_amd.runtime.engine import TrainEngine
    out = _spawn(_train_strategies, 8, 3)
    cfg = parse_train_config(dict(W8_CFG, options=dict(W8_CFG["options"], batch_size=400)))
    ref = TrainEngine(cfg, synthetic_mnist(800, seed=1), device="cpu")
    for _ in range(3):
        ref.step()
    want = _named(ref)
    for strategy in ("allreduce", "ps", "lowrank"):
        for r in range(1, 8):
            for k in want:
                torch.testing.assert_close(out[r][strategy][k], out[0][strategy][k], rtol=0, atol=0)
        for k, v in want.items():
            torch.testing.assert_close(out[0][strategy][k], v, rtol=2e-4, atol=2e-5,
                                       msg=lambda m, s=strategy, k=k: f"{s} {k}: {m}")


def test_sync_bn_equals_full_batch_world8():
    out = _spawn(_sync_bn_w, 8)
    for r in range(8):
        fwd_ok, gdiff, gmax, run_ok = out[r]
        assert fwd_ok, r
        assert gdiff <= 1e-5 * max(1.0, gmax), (r, gdiff, gmax)
        assert run_ok, r


def test_collectives_world8():
    out = _spawn(_collectives, 8)
    assert out == {r: True for r in range(8)}


def test_lowrank_candidate_pruned_at_width():
    """lowrank's K = W x B weight gradient outgrows the all-reduce's
    link time on the sample CNN somewhere between 4 and 8 GPUs; an 8-GPU job does not time
    it at start-up."""
    from cloud_server_amd.models.dsl import SAMPLE_CONFIG
    from cloud_server_amd.parallel.strategy import default_candidates
    cfg = parse_train_config(dict(SAMPLE_CONFIG, options={"batch_size": 50}))
    assert default_candidates(cfg, 2) == ("lowrank", "allreduce", "ps")
    assert default_candidates(cfg, 8) == ("allreduce", "ps")


def _train_det(rank, world, port, strategy, steps, out):
    os.environ["CSA_DETERMINISTIC"] = "1"
    from cloud_server_amd.parallel.dist import shutdown
    from cloud_server_amd.runtime.engine import TrainEngine
    ctx = _init(rank, world, port)
    cfg = parse_train_config(CFG)
    res = []
    for _ in range(2):
        eng = TrainEngine(cfg, synthetic_mnist(256, seed=1), device="cpu", ctx=ctx, strategy=strategy)
        assert eng.sync.det
        for _ in range(steps):
            eng.step()
        res.append(eng.flat.clone())
    out[rank] = res
    shutdown(ctx)


@pytest.mark.parametrize("strategy", ["allreduce", "ps"])
def test_deterministic_dp_world4_bitwise(strategy):
    """CSA_DETERMINISTIC=1 under data parallelism: every sum is rank-ordered (exact
    all-gather + fold on gloo; the xGMI kernels on the GPU), so two runs and all four
    replicas are bitwise identical."""
    out = _spawn(_train_det, 4, strategy, 4)
    for r in range(4):
        assert torch.equal(out[r][0], out[r][1]), r
        assert torch.equal(out[r][0], out[0][0]), r


def _train_async(rank, world, port, staleness, steps, out):
    from cloud_server_amd.parallel.dist import shutdown
    from cloud_server_amd.runtime.engine import TrainEngine
    ctx = _init(rank, world, port)
    cfg = parse_train_config(dict(CFG, optimizer_name="AdagradOptimizer", learning_rate=0.05,
                                  options=dict(CFG["options"], batch_size=16, staleness=staleness)))
    ds = synthetic_mnist(512, seed=1)
    eng = TrainEngine(cfg, ds, device="cpu", ctx=ctx, strategy="async_ps")
    assert eng.aps is not None and eng.sync.grad_scale == 1.0
    first = None
    for i in range(steps):
        if rank == 1 and i % 3 == 0:
            import time
            time.sleep(0.01)                # a slower worker: the others run ahead (bounded)
        eng.step()
        if i == 9:
            first = eng.metrics_since(0)["loss"]
    last = eng.metrics_since(eng.host_step - 10)["loss"]
    eng.finish_async()
    out[rank] = (eng.flat.clone(), eng.staleness(), first, last, eng.aps.applied)
    shutdown(ctx)


@pytest.mark.parametrize("world,staleness", [(2, 0), (3, 2), (4, 1)])
def test_async_ps_gloo_converges_with_bounded_staleness(world, staleness):
    """VERDICT r3 missing #1: the asynchronous PS (each rank pushes its gradient shards to
    the owners with no step barrier, owners apply every push on its own as it arrives,
    ranks read parameters at most 2s clocks stale).  The loss falls, the measured
    staleness stays within the bound, every owner applied every push, and after the
    final drain the replicas agree bitwise."""
    steps = 40
    out = _spawn(_train_async, world, staleness, steps)
    for r in range(world):
        flat, stale, first, last, applied = out[r]
        assert stale <= 2 * staleness, (r, stale)         # async_ps.py: max_staleness <= 2s
        assert last < first, (r, first, last)
        assert applied == world * steps, (r, applied)
        torch.testing.assert_close(flat, out[0][0], rtol=0, atol=0)


def test_distributed_job_async_ps(tmp_path):
    """A whole training job (result.txt from rank 0, checkpoints with the sharded slots,
    the final drain before evaluation) under strategy async_ps."""
    mdir = str(tmp_path / "m")
    os.makedirs(mdir)
    cfg = dict(CFG, options=dict(CFG["options"], strategy="async_ps", staleness=1))
    out = _spawn(_job, 2, mdir, cfg)
    assert out == {0: 12, 1: 12}
    lines = open(os.path.join(mdir, "result.txt")).read().splitlines()
    assert [l.split(",")[0] for l in lines[:4]] == ["step:0", "step:4", "step:8", "step:12"]
    assert lines[4].startswith("final_accuracy:")


def _aps_save(rank, world, port, path, out):
    """async_ps mid-run checkpoint: rank 1 is slower, so rank 0's copy of rank 1's shard is
    a stale pull while the saved slots are rank 1's current ones."""
    import time
    from cloud_server_amd.parallel.dist import shutdown
    from cloud_server_amd.runtime import checkpoint as ckpt
    from cloud_server_amd.runtime.engine import TrainEngine
    ctx = _init(rank, world, port)
    cfg = parse_train_config(dict(CFG, options=dict(CFG["options"], batch_size=16, staleness=2)))
    eng = TrainEngine(cfg, synthetic_mnist(512, seed=1), device="cpu", ctx=ctx, strategy="async_ps")
    for _ in range(9):
        if rank == 1:
            time.sleep(0.02)
        eng.step()
    st = ckpt.engine_state(eng)                      # collective
    lo, hi = eng.sync.shard_range()
    out[rank] = (eng.flat[lo:hi].clone(), eng.slots.clone(), (lo, hi), eng.flat.clone())
    if rank == 0:
        ckpt.save(path, eng.host_step, st)
    eng.finish_async()
    shutdown(ctx)


def _aps_resume(rank, world, port, path, out):
    from cloud_server_amd.parallel.dist import shutdown
    from cloud_server_amd.runtime import checkpoint as ckpt
    from cloud_server_amd.runtime.engine import TrainEngine
    ctx = _init(rank, world, port)
    cfg = parse_train_config(dict(CFG, options=dict(CFG["options"], batch_size=16, staleness=2)))
    eng = TrainEngine(cfg, synthetic_mnist(512, seed=1), device="cpu", ctx=ctx, strategy="async_ps")
    ckpt.restore_engine(eng, ckpt.load(ckpt.latest(path)[1]))
    out[rank] = (eng.flat.clone(), eng.slots.clone(), eng.host_step)
    eng.finish_async()
    shutdown(ctx)


def test_async_ps_checkpoint_saves_owner_shards_and_resumes(tmp_path):
    """a mid-run async_ps checkpoint holds every OWNER's current shard (gathered,
    as the slots are), not the chief's stale pulled copies; a resume puts the same
    parameters on every rank and each owner's slots back on its shard."""
    from cloud_server_amd.runtime import checkpoint as ckpt
    path = str(tmp_path / "m")
    os.makedirs(path)
    saved = _spawn(_aps_save, 2, path)
    obj = ckpt.load(ckpt.latest(path)[1])
    flat = torch.zeros_like(saved[0][3])
    for name, o, k in obj["layout"]:
        flat[o:o + k] = obj["model"][name].reshape(-1)
    for r in range(2):
        own, slots, (lo, hi), _ = saved[r]
        torch.testing.assert_close(flat[lo:hi], own, rtol=0, atol=0)                  # owner's shard
        torch.testing.assert_close(obj["slots"][:, lo:hi], slots, rtol=0, atol=0)     # owner's slots
    res = _spawn(_aps_resume, 2, path)
    for r in range(2):
        rflat, rslots, step = res[r]
        lo, hi = saved[r][2]
        assert step == 9
        torch.testing.assert_close(rflat, flat, rtol=0, atol=0)
        torch.testing.assert_close(rslots, obj["slots"][:, lo:hi], rtol=0, atol=0)


def _pick_hf(rank, world, port, out):
    from cloud_server_amd.parallel.dist import shutdown
    from cloud_server_amd.parallel.strategy import pick_strategy
    ctx = _init(rank, world, port)
    cfg = parse_train_config(CFG)
    best, times = pick_strategy(cfg, synthetic_mnist(256, seed=1), ctx, candidates=("allreduce", "allreduce:hf"),
                                steps=2, backend="torch")
    out[rank] = (best, times)
    shutdown(ctx)


def test_tuner_skips_hf_trial_without_hf_program():
    """a ':hf' candidate whose engine did not build the :hf program (here the
    eager program) is not timed — it would be a duplicate of the plain strategy."""
    out = _spawn(_pick_hf, 2)
    for r in range(2):
        best, times = out[r]
        assert best == "allreduce" and times["allreduce:hf"] is None and times["allreduce"] > 0
