"""Overlapped, bucketed gradient all-reduce of the HIP program, on one MI355X.

A real RCCL process group of world size 1 (all-reduce = identity) with a context that
reports DP as enabled runs the exact multi-GPU code path — side-stream all-reduces of
the ready gradient suffixes captured into the HIP graph, the main stream joining
before the optimizer — and must give the same weights as the plain single-GPU step."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.parallel.dist import DistContext
from cloud_server_amd.runtime.engine import TrainEngine

pytestmark = pytest.mark.gpu


class _DPContext(DistContext):
    @property
    def enabled(self) -> bool:       # world 1, but take every DP code path
        return True


@pytest.fixture(scope="module")
def pg():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from cloud_server_amd.parallel.dist import rccl_env_defaults
    rccl_env_defaults()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    # the test's engines (and the RCCL works captured into their graphs) die with this
    # group, before the next test's group starts
    import gc
    gc.collect()
    torch.cuda.synchronize()
    dist.destroy_process_group()


def test_overlap_buckets_match_single_gpu(pg, monkeypatch):
    monkeypatch.setenv("CSA_XGMI", "1")      # force the peer-buffer path (world 1: RCCL is a no-op)
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdamOptimizer", learning_rate=1e-3))
    ds = synthetic_mnist(2000, seed=0)
    ctx = _DPContext(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
    a = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend="hip")
    assert a.sync.xgmi is not None, a.sync.xgmi_reason      # buckets on the xGMI peer path
    assert a.program.overlap and len(a.program.bucket_at) >= 2, a.program.bucket_at
    spans = sorted(a.program.bucket_at.values())
    assert spans[0][0] == 0 and spans[-1][1] == a.flat.numel()
    assert all(x[1] == y[0] for x, y in zip(spans, spans[1:]))          # exact tiling
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    for _ in range(20):
        a.step(); b.step()
    a.sync_device(); b.sync_device()   # (lands a deferred dense update)
    torch.testing.assert_close(a.flat, b.flat, rtol=2e-3, atol=2e-5)


def test_lowrank_strategy_matches_single_gpu(pg, monkeypatch):
    """``lowrank`` DP: dense weight gradients from all-gathered GEMM inputs / output
    gradients (K = world·B) on a side stream, the rest all-reduced — captured in the HIP
    graph; world 1 must reproduce the single-GPU step."""
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdamOptimizer", learning_rate=1e-3))
    ds = synthetic_mnist(2000, seed=0)
    ctx = _DPContext(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
    monkeypatch.setenv("CSA_XGMI", "1")
    monkeypatch.setenv("CSA_GRAPH_STEPS", "8")
    a = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend="hip", strategy="lowrank")
    assert a.sync.xgmi is not None, a.sync.xgmi_reason
    assert a.backend == "hip", a.fallback_reason
    names = [u.layer.name for u in a.program.lr_units]
    assert len(names) == 2, names                      # fc1 (materialised BN input) and fc2
    # the gathered global dW is applied inside the weight-gradient launch (no dW buffer,
    # the optimizer launch skips those spans) and the forward GEMMs are register-direct
    assert all(u.lr_update and u.direct for u in a.program.lr_units)
    skipped = {a.model.state.offsets[f"{n}.weight"] for n in names}
    assert not any(lo <= o < hi for lo, hi in a.program.opt_segments for o in skipped), a.program.opt_segments
    # dense-last flat layout: the all-reduced remainder (conv, BN, head) is ONE leading range
    assert len(a.program.lr_ranges) == 1 and a.program.lr_ranges[0][0] == 0, a.program.lr_ranges
    first_dense = min(a.model.state.offsets[f"{n}.weight"] for n in names)
    assert a.program.lr_ranges[0][1] <= first_dense
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    for _ in range(4):
        a.step(); b.step()
    # multi-step graphs under data parallelism: 16 more steps as two 8-step launches
    assert a.group_steps() == 8
    a.run_steps(16); b.run_steps(16)
    assert a.graph_k is not None and a.host_step == b.host_step == 20
    a.sync_device(); b.sync_device()   # (lands a deferred dense update)
    assert a.sync._choice["lr_x"] is not None and a.sync._choice["lr_dy"] is not None, a.sync._choice
    a.sync.check()
    for n in a.model.state.shapes:          # the two flat layouts differ: compare by name
        torch.testing.assert_close(a.model.state.view(n, a.flat), b.model.state.view(n, b.flat),
                                   rtol=2e-3, atol=2e-5)


@pytest.mark.parametrize("strategy,xgmi", [("ps", "0"), ("ps", "1"), ("allreduce", "0")])
def test_ps_and_rccl_programs_match_single_gpu(pg, monkeypatch, strategy, xgmi):
    """The parameter-server capability (``ps``: reduce-scatter -> owner optimizer on its
    shard -> all-gather, the reference's PS placement) and the all-reduce program on plain
    RCCL, on the HIP program with the fused dense backward in gradient mode, the
    row-per-workgroup head and the striped pair gradients; world 1 must reproduce the
    single-GPU step (20 steps, 8-step graphs)."""
    monkeypatch.setenv("CSA_XGMI", xgmi)
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-3))
    ds = synthetic_mnist(2000, seed=0)
    ctx = _DPContext(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
    a = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend="hip", strategy=strategy)
    assert a.backend == "hip", a.fallback_reason
    # the fused dense backward in gradient mode (dW / db stored whole into the flat
    # gradient for the exchange) with the row head's reductions in fc2's epilogue
    assert a.program.fused_grad and all(u.fused for u in a.program.units[2:])
    assert a.program.head_row and not a.program.head_sep
    assert a.program.units[0].row_fold and a.program.units[0].wg_stripes == 16
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    for _ in range(4):
        a.step(); b.step()
    a.run_steps(16); b.run_steps(16)
    a.sync_device(); b.sync_device()   # (lands a deferred dense update)
    assert a.host_step == b.host_step == 20 and int(a.dstep.item()) == 20
    torch.testing.assert_close(a.flat, b.flat, rtol=2e-3, atol=2e-5)
    ma, mb = a.metrics_since(0), b.metrics_since(0)
    assert abs(ma["loss"] - mb["loss"]) < 1e-3 * max(1.0, mb["loss"])
    assert abs(ma["accuracy"] - mb["accuracy"]) <= 3 / (20 * 50) + 1e-9


def test_collective_autotune_records_both_paths(pg, monkeypatch):
    """CSA_XGMI=auto: each call site is timed on both paths (HIP graphs of 10 calls) at
    first use and the choice is recorded; training still matches the single-GPU step."""
    monkeypatch.setenv("CSA_XGMI", "auto")
    # Adam: the step is scale-free, so 20 steps of two summation orders stay within
    # tolerance (SGD/Adagrad at lr 1e-2 drift ~1e-3 between ANY two layouts, allreduce too:
    # scripts/diag_lowrank_opt.py)
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdamOptimizer", learning_rate=1e-3))
    ds = synthetic_mnist(2000, seed=0)
    ctx = _DPContext(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
    a = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend="hip", strategy="lowrank")
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    for _ in range(20):
        a.step(); b.step()
    a.sync_device(); b.sync_device()   # (lands a deferred dense update)
    a.sync.check()
    # gather sites (lr_x, lr_dy) time the xGMI gather; the remainder all-reduce (lr_rem,
    # 16-byte aligned since round 6) times the one-shot protocol — each against RCCL
    assert set(a.sync.xgmi_tuning) >= {"lr_x", "lr_dy", "lr_rem"}, a.sync.xgmi_tuning
    for tag, v in a.sync.xgmi_tuning.items():
        assert v["rccl_us"] > 0 and v["xgmi_us" if tag in ("lr_x", "lr_dy") else "oneshot_us"] > 0, (tag, v)
    print("collective tuning (world 1):", a.sync.xgmi_tuning)
    for n in a.model.state.shapes:          # lowrank uses the dense-last layout: compare by name
        torch.testing.assert_close(a.model.state.view(n, a.flat), b.model.state.view(n, b.flat),
                                   rtol=2e-3, atol=2e-5)


def test_capture_never_finalizes_garbage_graphs_while_capturing():
    """Regression test of the round-2 GPU-suite abort (profiles/r3_gpu_suite_abort.md): a
    CUDAGraph left in a reference cycle by an earlier engine must never be destroyed by a
    garbage collection triggered inside a capture — only outside it."""
    import gc
    import weakref
    from cloud_server_amd.utils.graphs import capture
    x = torch.zeros(8, device="cuda:0")
    old = torch.cuda.CUDAGraph()
    with capture(old):
        x.add_(1)

    class Holder:                       # engine <-> program style reference cycle
        pass
    h = Holder()
    h.graph, h.self_ref = old, h
    seen = []
    weakref.finalize(h, lambda: seen.append(torch.cuda.is_current_stream_capturing()))
    del h, old
    g = torch.cuda.CUDAGraph()
    with capture(g):
        for _ in range(200):
            [object() for _ in range(100)]   # allocations that would trigger a collection
        x.add_(1)
    gc.collect()                      # (the collector is back on after the capture)
    assert seen == [False]            # finalised, and not while capturing
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 1.0         # captures never execute: only the replay added 1


@pytest.mark.parametrize("strategy", ["allreduce", "ps"])
def test_capture_right_after_eager_collectives(pg, monkeypatch, strategy):
    """a DP step whose RCCL collectives are captured into the HIP graph is
    captured IMMEDIATELY after eager collectives on the default group (no device drain,
    no sleep anywhere in ``capture()``): the captured collectives run on the dedicated
    capture group, whose stream never carries an eager work the watchdog is polling."""
    import inspect
    from cloud_server_amd.utils import graphs
    assert "sleep" not in inspect.getsource(graphs.capture)
    monkeypatch.setenv("CSA_XGMI", "0")           # RCCL collectives inside the step graphs
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-3))
    ds = synthetic_mnist(2000, seed=0)
    ctx = _DPContext(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
    a = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend="hip", strategy=strategy)
    assert a.sync.cap_group is not None
    # observed, not timed (None: blocking-wait mode has no watchdog thread to wait for)
    want = None if os.environ.get("TORCH_NCCL_BLOCKING_WAIT", "0") == "1" else True
    assert a.sync.cap_group_retired is want, a.sync.cap_group_retired
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    x = torch.ones(4096, device="cuda:0")
    for _ in range(8):
        dist.all_reduce(x)                       # eager works the watchdog still polls
    a.step(); b.step()                           # warm-up + capture right away
    for _ in range(8):
        dist.all_reduce(x)
    a.prepare_group_graph()                      # every multi-step capture, right away
    b.prepare_group_graph()
    a.run_steps(15); b.run_steps(15)
    a.sync_device(); b.sync_device()   # (lands a deferred dense update)
    assert a.host_step == b.host_step == 16
    torch.testing.assert_close(a.flat, b.flat, rtol=2e-3, atol=2e-5)


@pytest.mark.parametrize("strategy", ["allreduce:hf", "ps:hf"])
def test_hf_programs_match_single_gpu(pg, monkeypatch, strategy):
    """the data-parallel program with the one-GPU step's structure — fc2's
    input gradient in the head launch, fc1's input gradient alone, both dense weight
    gradients formed in GRADIENT mode as extra workgroups of the pair backward (stored whole
    into the flat gradient), the conv stripes folded by that launch's tail — then the
    exchange and the flat optimizer; world 1 must reproduce the single-GPU step."""
    monkeypatch.setenv("CSA_XGMI", "0")
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-3))
    ds = synthetic_mnist(2000, seed=0)
    ctx = _DPContext(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
    a = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend="hip", strategy=strategy)
    assert a.backend == "hip", a.fallback_reason
    p = a.program
    assert p.dp_hf and p.hfuse and p.head_dgrad and p.tail and not p.tail_update and not p.overlap
    assert a.sync.strategy == strategy.split(":")[0]
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    for _ in range(4):
        a.step(); b.step()
    a.run_steps(16); b.run_steps(16)
    a.sync_device(); b.sync_device()   # (lands a deferred dense update)
    assert a.host_step == b.host_step == 20 and int(a.dstep.item()) == 20
    assert p.tail_error() == 0
    torch.testing.assert_close(a.flat, b.flat, rtol=2e-3, atol=2e-5)
    ma, mb = a.metrics_since(0), b.metrics_since(0)
    assert abs(ma["loss"] - mb["loss"]) < 1e-3 * max(1.0, mb["loss"])


def test_carry_flush_is_idempotent_mid_run(pg, monkeypatch):
    """the deferred dense update's pending flag is cleared by the launch right
    after the carrying forward (bn_act_apply), so host flushes between steps (a checkpoint
    every few steps, a second flush right after) never apply the update twice."""
    monkeypatch.setenv("CSA_XGMI", "0")
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name="AdagradOptimizer", learning_rate=1e-3))
    ds = synthetic_mnist(2000, seed=0)
    ctx = _DPContext(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
    a = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend="hip", strategy="allreduce")
    assert a.program.carry is not None, "the allreduce program carries the dense update"
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    for i in range(12):
        a.step(); b.step()
        if i % 3 == 1:
            a.flush_params()
            a.flush_params()                 # a second flush: nothing pending any more
            torch.cuda.synchronize()
            assert int(a.program.carry_pending[0].item()) == 0
    a.sync_device(); b.sync_device()
    torch.testing.assert_close(a.flat, b.flat, rtol=2e-3, atol=2e-5)


@pytest.mark.parametrize("strategy", ["async_ps:flat", "async_ps"])
@pytest.mark.parametrize("opt", ["AdagradOptimizer", "AdamOptimizer"])
def test_async_ps_world1_matches_single_gpu(pg, opt, strategy):
    """async_ps at world 1 (csrc/comm/async_ps.hip): the rank's own push is applied straight
    from its gradient in the step's launch (it never waits on a peer), no publication is
    written (no reader) — the parameters must follow the plain single-GPU step."""
    cfg = parse_train_config(dict(SAMPLE_CONFIG, optimizer_name=opt, learning_rate=1e-3,
                                  options={"batch_size": 50, "staleness": 2}))
    ds = synthetic_mnist(2000, seed=0)
    ctx = _DPContext(rank=0, world=1, local_rank=0, backend="nccl", device=torch.device("cuda", 0))
    a = TrainEngine(cfg, ds, device="cuda:0", ctx=ctx, backend="hip", strategy=strategy)
    assert a.backend == "hip", a.fallback_reason
    assert type(a.aps).__name__ == "AsyncPSDevice"
    # ":hf": the one-GPU step's structure in gradient mode (dense weight gradients inside
    # the pair backward launch, its tail folds the conv stripes), then the push / apply
    assert a.program.dp_hf == (strategy == "async_ps")   # (the default: the :hf program)
    b = TrainEngine(cfg, ds, device="cuda:0", backend="hip")
    for _ in range(12):
        a.step(); b.step()
    a.sync_device(); b.sync_device()
    a.aps.check()
    assert a.aps.applied == 12 and a.staleness() == 0
    torch.testing.assert_close(a.flat, b.flat, rtol=2e-3, atol=2e-5)
    a.finish_async()
    assert a.aps.applied == 12
    a.close()
