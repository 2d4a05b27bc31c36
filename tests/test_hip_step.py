"""Numerics of the HIP training step vs the PyTorch fp32 reference (GPU only).

Each case builds two engines from the same seed and data — one running the
hand-written gfx950 kernels (``HipProgram``), one running eager PyTorch autograd
(``TorchProgram``) — takes one SGD step in each and compares the implied gradients
(g = (w0 - w1) / lr) per named tensor, plus loss and accuracy bookkeeping.
"""
import copy

import numpy as np
import pytest
import torch

from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.runtime.engine import TrainEngine

pytestmark = pytest.mark.gpu


def _cfg(layers, **kw):
    c = copy.deepcopy(SAMPLE_CONFIG)
    c["net_config"]["middle_layer"] = layers
    c["optimizer_name"] = kw.pop("optimizer", "GradientDescentOptimizer")
    c["learning_rate"] = kw.pop("lr", 0.5)
    c["loss_name"] = kw.pop("loss", "entropy")
    c["options"] = dict(batch_size=kw.pop("batch", 50), **kw)
    return parse_train_config(c)


CASES = {
    "sample": SAMPLE_CONFIG["net_config"]["middle_layer"],
    "relu_bias_stride": [
        {"layer": "conv", "filter": [3, 3, 8], "isBias": "True", "stride": [2, 2]},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [2, 2, 16], "padding": "VALID"},
        {"layer": "active", "active_func": "leaky_relu", "param": [0.1]},
        {"layer": "pool"},
        {"layer": "connect", "hidden": 64},
        {"layer": "active", "active_func": "relu"},
    ],
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
    "pair_relu_valid": [
        {"layer": "conv", "filter": [3, 3, 6], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [3, 3, 8], "padding": "VALID", "isBias": "True"},
        {"layer": "active", "active_func": "leaky_relu", "param": [0.1]},
        {"layer": "pool"},
        {"layer": "norm"},
        {"layer": "connect", "hidden": 32},
    ],
    # the MFMA conv-pair family (outside the VALU pair's family): a 4x4 conv B, and a
    # 48-channel conv B whose backward takes the staged (multi-batch) prologue
    "pair_mfma": [
        {"layer": "conv", "filter": [3, 3, 8], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [4, 4, 16]},
        {"layer": "active", "active_func": "relu"},
        {"layer": "pool"},
        {"layer": "norm"},
        {"layer": "connect", "hidden": 32},
    ],
    "pair_mfma_wide": [
        {"layer": "conv", "filter": [2, 2, 8]},
        {"layer": "conv", "filter": [3, 3, 48], "isBias": "True"},
        {"layer": "active", "active_func": "sigmoid"},
        {"layer": "pool"},
        {"layer": "connect", "hidden": 16},
    ],
    # conv A beyond the pair kernels' 16-wide conv-A tile: separate conv units
    "wide_conv_a": [
        {"layer": "conv", "filter": [5, 5, 8], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [3, 3, 16]},
        {"layer": "pool"},
        {"layer": "connect", "hidden": 32},
    ],
    "wide_c1": [
        {"layer": "conv", "filter": [3, 3, 24]},
        {"layer": "conv", "filter": [2, 2, 32], "isBias": "True"},
        {"layer": "active", "active_func": "sigmoid"},
        {"layer": "pool"},
        {"layer": "connect", "hidden": 16},
    ],
    "pair_nopool": [
        {"layer": "conv", "filter": [2, 2, 4]},
        {"layer": "conv", "filter": [3, 3, 8]},
        {"layer": "active", "active_func": "relu"},
        {"layer": "connect", "hidden": 16},
    ],
    "dense_only": [
        {"layer": "connect", "hidden": 128},
        {"layer": "active", "active_func": "relu"},
        {"layer": "connect", "hidden": 64},
    ],
    # standalone units (norm_pool.hip): 2-D BatchNorm after a dense layer and before the
    # head, pool after norm + act, act -> norm -> act, > 128 BN channels, pool first,
    # five biased convs (more striped weight gradients than the optimizer folds)
    "dense_norm_head": [
        {"layer": "conv", "filter": [3, 3, 6], "isBias": "True"},
        {"layer": "pool"},
        {"layer": "connect", "hidden": 64},
        {"layer": "norm"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "connect", "hidden": 32},
        {"layer": "norm"},
    ],
    "pool_after_norm_act": [
        {"layer": "conv", "filter": [3, 3, 8]},
        {"layer": "norm"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "pool"},
        {"layer": "active", "active_func": "sigmoid"},
        {"layer": "norm"},
        {"layer": "active", "active_func": "leaky_relu", "param": [0.2]},
        {"layer": "connect", "hidden": 24},
    ],
    "wide_norm_pool_first": [
        {"layer": "pool"},
        {"layer": "conv", "filter": [3, 3, 16], "isBias": "True"},
        {"layer": "norm"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "pool", "kernel": [3, 3], "stride": [2, 2]},
        {"layer": "connect", "hidden": 160},
        {"layer": "norm"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "connect", "hidden": 16},
    ],
    "five_biased_convs": [
        {"layer": "conv", "filter": [3, 3, 4], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [3, 3, 6], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "pool"},
        {"layer": "conv", "filter": [3, 3, 8], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [3, 3, 8], "isBias": "True"},
        {"layer": "norm"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [3, 3, 10], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "pool"},
        {"layer": "connect", "hidden": 32},
    ],
    # > 128 channels (construct_distribute.py:222-233 takes any filter): implicit-GEMM
    # gconv units with standalone act / pool / norm, next to direct convs
    "wide_conv_192": [
        {"layer": "conv", "filter": [3, 3, 192], "isBias": "True", "stride": [2, 2]},
        {"layer": "active", "active_func": "relu"},
        {"layer": "pool"},
        {"layer": "conv", "filter": [2, 2, 16]},
        {"layer": "norm"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "connect", "hidden": 32},
    ],
    # leaky_relu with alpha = 0 (relu) and alpha < 0 (backward not recoverable from y:
    # lowered as consumer transforms / standalone act units, never fused into a producer)
    "leaky_alpha": [
        {"layer": "conv", "filter": [3, 3, 6], "isBias": "True"},
        {"layer": "active", "active_func": "leaky_relu", "param": [0]},
        {"layer": "conv", "filter": [2, 2, 8]},
        {"layer": "active", "active_func": "leaky_relu", "param": [-0.1]},
        {"layer": "pool"},
        {"layer": "connect", "hidden": 32},
        {"layer": "active", "active_func": "leaky_relu", "param": [-0.1]},
        {"layer": "connect", "hidden": 32},
        {"layer": "active", "active_func": "leaky_relu", "param": [-0.3]},
    ],
    # a 20-layer network (every layer kind, several of each)
    "deep20": [
        {"layer": "conv", "filter": [3, 3, 8], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [3, 3, 8]},
        {"layer": "active", "active_func": "leaky_relu", "param": [0.1]},
        {"layer": "pool"},
        {"layer": "norm"},
        {"layer": "conv", "filter": [3, 3, 12], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "conv", "filter": [2, 2, 12]},
        {"layer": "norm"},
        {"layer": "active"},
        {"layer": "pool"},
        {"layer": "connect", "hidden": 128},
        {"layer": "active", "active_func": "relu"},
        {"layer": "connect", "hidden": 128},
        {"layer": "active", "active_func": "leaky_relu", "param": [-0.2]},
        {"layer": "connect", "hidden": 64},
        {"layer": "active"},
        {"layer": "connect", "hidden": 64},
        {"layer": "active", "active_func": "relu"},
    ],
    # three dense layers with activations between them and before the head: the
    # horizontal-fusion program (three deferred update segments, the head + last-dense
    # input gradient launch with an activation epilogue)
    "dense3_act": [
        {"layer": "conv", "filter": [2, 2, 10]},
        {"layer": "conv", "filter": [2, 2, 20]},
        {"layer": "pool"},
        {"layer": "norm"},
        {"layer": "active"},
        {"layer": "connect", "hidden": 256},
        {"layer": "connect", "hidden": 256},
        {"layer": "connect", "hidden": 128},
        {"layer": "active", "active_func": "leaky_relu", "param": [0.2]},
    ],
    "wide_conv_chain": [
        {"layer": "conv", "filter": [3, 3, 8], "isBias": "True"},
        {"layer": "active", "active_func": "relu"},
        {"layer": "pool"},
        {"layer": "conv", "filter": [3, 3, 160], "padding": "VALID"},
        {"layer": "norm"},
        {"layer": "active", "active_func": "leaky_relu"},
        {"layer": "conv", "filter": [2, 2, 136], "isBias": "True", "stride": [2, 2]},
        {"layer": "active", "active_func": "sigmoid"},
        {"layer": "connect", "hidden": 24},
    ],
}
STANDALONE = {"dense_norm_head": ("bn",), "pool_after_norm_act": ("bn", "pool"),
              "wide_norm_pool_first": ("bn", "pool"), "wide_conv_192": ("gconv", "bn", "pool"),
              "wide_conv_chain": ("gconv", "bn")}


def _run_one(cfg, backend, ds, name=None):
    eng = TrainEngine(cfg, ds, device="cuda", backend=backend, use_graph=False)
    assert eng.backend == backend, eng.fallback_reason
    if backend == "hip" and name in STANDALONE:      # the pattern lowered to standalone units
        kinds = {u.kind for u in eng.program.units}
        assert set(STANDALONE[name]) <= kinds, kinds
    w0 = eng.flat.clone()
    eng.step()
    torch.cuda.synchronize()
    return eng, w0, eng.flat.clone()


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("loss", ["entropy", "mse"])
def test_step_matches_torch(name, loss):
    ds = synthetic_mnist(400, seed=3)
    cfg = _cfg(CASES[name], loss=loss, lr=0.5)
    eh, w0h, w1h = _run_one(cfg, "hip", ds, name)
    et, w0t, w1t = _run_one(cfg, "torch", ds)
    assert torch.equal(w0h, w0t)
    gh = (w0h - w1h) / cfg.effective_lr
    gt = (w0t - w1t) / cfg.effective_lr
    # a gradient that is exactly 0 in exact arithmetic (e.g. a bias followed, through any
    # per-batch-constant path, by a BatchNorm: the batch mean cancels it) is pure fp32
    # summation noise in both programs: bound it against the model's largest gradient
    gmax = gt.abs().max().item()
    for k in eh.model.state.shapes:
        a, b = eh.model.state.view(k, gh), et.model.state.view(k, gt)
        scale = b.abs().max().item() + 1e-6
        err = (a - b).abs().max().item()
        assert err <= 2e-3 * scale + 1e-6 + 1e-5 * gmax, f"{name}/{loss} grad {k}: err {err:.3e} scale {scale:.3e}"
    mh, mt = eh.metrics_since(0), et.metrics_since(0)
    assert abs(mh["loss"] - mt["loss"]) < 1e-4 * max(1, abs(mt["loss"]))
    assert mh["accuracy"] == mt["accuracy"]


@pytest.mark.parametrize("opt", ["AdagradOptimizer", "AdamOptimizer", "AdadeltaOptimizer",
                                 "GradientDescentOptimizer"])
def test_optimizers_match_torch(opt):
    ds = synthetic_mnist(300, seed=5)
    cfg = _cfg(CASES["sample"], optimizer=opt, lr=0.01)
    outs = []
    for backend in ("hip", "torch"):
        eng = TrainEngine(cfg, ds, device="cuda", backend=backend, use_graph=False)
        for _ in range(3):
            eng.step()
        torch.cuda.synchronize()
        outs.append(eng.flat.clone())
    diff = (outs[0] - outs[1]).abs()
    worst = {k: eng.model.state.view(k, diff).max().item() for k in eng.model.state.shapes}
    # Adam / Adadelta normalise each element's step: a gradient that is ~0 in fp32 moves its
    # weight by ~lr whatever its rounding, so a few elements may differ by a fraction of
    # lr * steps; the bulk must agree to fp32 noise
    assert diff.max().item() < 2e-3, f"{opt}: params diverge: {worst}"
    assert torch.quantile(diff[diff > 0].float()[:1 << 24], 0.999).item() < 1e-5 if (diff > 0).any() else True, worst


def test_graph_replay_matches_eager():
    ds = synthetic_mnist(500, seed=7)
    cfg = _cfg(CASES["sample"], optimizer="AdagradOptimizer", lr=0.01)
    a = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=True)
    b = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=False)
    for _ in range(20):
        a.step()
        b.step()
    torch.cuda.synchronize()
    assert (a.flat - b.flat).abs().max().item() < 3e-3   # atomics: run-to-run fp32 order
    assert a.host_step == b.host_step == 20
    assert int(a.dstep.item()) == 20


def test_training_learns_sample_config():
    ds = synthetic_mnist(5000, seed=11)
    cfg = _cfg(CASES["sample"], optimizer="AdamOptimizer", lr=1e-3)
    eng = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=True)
    for _ in range(300):
        eng.step()
    acc = eng.evaluate(ds)
    assert acc > 0.9, acc


@pytest.mark.parametrize("batch", [1, 7, 64, 80, 200])
def test_batch_sizes_match_torch(batch):
    """Odd batch sizes: head MFMA path (<= 64 rows) and generic path, GEMM M tiling."""
    ds = synthetic_mnist(600, seed=13)
    cfg = _cfg(CASES["sample"], lr=0.5, batch=batch)
    eh, w0h, w1h = _run_one(cfg, "hip", ds)
    et, w0t, w1t = _run_one(cfg, "torch", ds)
    gh = (w0h - w1h) / cfg.effective_lr
    gt = (w0t - w1t) / cfg.effective_lr
    for k in eh.model.state.shapes:
        a, b = eh.model.state.view(k, gh), et.model.state.view(k, gt)
        scale = b.abs().max().item() + 1e-6
        assert (a - b).abs().max().item() <= 3e-3 * scale + 1e-6, f"batch {batch} grad {k}"


def test_fused_update_path_active_and_matches_unfused(monkeypatch):
    """Single-GPU program: the dense layers' backward applies the optimizer in-kernel
    (csa_dense_bwd_update) and the row-per-workgroup head's batch reductions (dWh, dbh,
    metric ring) ride in the last dense layer's fused backward.  Several Adam / Adagrad steps match the unfused program (materialised
    gradients + the flat optimizer) and the metric ring agrees."""
    ds = synthetic_mnist(600, seed=17)
    for opt in ("AdamOptimizer", "AdagradOptimizer"):
        cfg = _cfg(CASES["sample"], optimizer=opt, lr=1e-3)
        monkeypatch.setenv("CSA_FUSED_UPDATE", "1")
        monkeypatch.setenv("CSA_FUSED_DENSE", "1")
        a = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=True)
        monkeypatch.setenv("CSA_FUSED_UPDATE", "0")
        b = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=True)
        assert a.program.fused and a.program.head_row and a.program.head_rg == 0
        assert [u.fused for u in a.program.units if u.kind == "dense"] == [True, True]
        assert not b.program.fused
        for _ in range(5):
            a.step()
            b.step()
        torch.cuda.synchronize()
        d = (a.flat - b.flat).abs().max().item()
        assert d < 2e-4, f"{opt}: fused vs unfused params differ by {d}"
        ma, mb = a.metrics_since(0), b.metrics_since(0)
        assert abs(ma["loss"] - mb["loss"]) < 1e-3 * max(1.0, mb["loss"])
        assert int(a.dstep.item()) == int(b.dstep.item()) == 5


@pytest.mark.parametrize("name,valu", [("sample", True), ("pair_relu_valid", True), ("pair_nopool", True),
                                       ("pair_mfma", False), ("pair_mfma_wide", False)])
def test_conv_pair_fused_active(name, valu):
    """The leading conv pair runs as the fused conv_pair kernels (one forward and one
    backward launch) for these configs, in the VALU family or the MFMA family as expected;
    numerics of every case are pinned by test_step_matches_torch."""
    from cloud_server_amd.ops import fused as FK
    ds = synthetic_mnist(200, seed=3)
    eng = TrainEngine(_cfg(CASES[name]), ds, device="cuda", backend="hip", use_graph=False)
    assert eng.program.pair is not None
    assert bool(eng.program.lib.csa_conv_pair_valu_ok(FK.ints(eng.program.pair))) == valu


@pytest.mark.parametrize("name", ["wide_conv_a", "wide_c1"])
def test_wide_conv_a_lowers_to_separate_units(name):
    """A conv A wider than the pair kernels' conv-A tile (> 16 taps or > 16 channels) is
    not fused into a pair; numerics are pinned by test_step_matches_torch."""
    ds = synthetic_mnist(200, seed=3)
    eng = TrainEngine(_cfg(CASES[name]), ds, device="cuda", backend="hip", use_graph=False)
    assert eng.backend == "hip" and eng.program.pair is None


def test_staged_batch_matches_cursor_path(monkeypatch):
    """CSA_STAGE_BATCH=1: the next step's batch is staged by the optimizer and the cursor is
    advanced by the head — identical training to the cursor-walking kernels, also across
    a seek (checkpoint resume) and graph capture."""
    ds = synthetic_mnist(700, seed=17)
    # plain GD: parameter differences stay proportional to the gradients' atomic-order
    # noise (Adagrad's first steps move every weight by ~lr whatever its gradient's size,
    # so a near-zero gradient's rounding can flip a whole step)
    cfg = _cfg(CASES["sample"], optimizer="GradientDescentOptimizer", lr=0.001)
    outs = []
    for staged in ("0", "1"):
        monkeypatch.setenv("CSA_STAGE_BATCH", staged)
        eng = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=True, stream_chunk=4)
        assert eng.program.staged == (staged == "1")
        for _ in range(13):            # crosses several half boundaries of the row table
            eng.step()
        eng.stream.seek(5)             # resume-style cursor move: the program re-stages
        for _ in range(6):
            eng.step()
        torch.cuda.synchronize()
        outs.append((eng.flat.clone(), eng.metrics_since(0)))
    assert (outs[0][0] - outs[1][0]).abs().max().item() < 1e-3
    # the statistic atomics' order may flip a borderline sample or two of the 19 x 50
    assert abs(outs[0][1]["accuracy"] - outs[1][1]["accuracy"]) <= 3 / (19 * 50) + 1e-9
    assert abs(outs[0][1]["loss"] - outs[1][1]["loss"]) < 1e-3 * max(1.0, abs(outs[0][1]["loss"]))


def test_run_steps_groups_equal_single_steps(monkeypatch):
    """run_steps(n) replays CSA_GRAPH_STEPS-step graphs where a group fits in a half of the
    batch row table and single steps elsewhere: exactly n steps run, with the same batches
    (cursor, step counter) and numerics as n step() calls — across half boundaries."""
    ds = synthetic_mnist(700, seed=29)
    cfg = _cfg(CASES["sample"], optimizer="GradientDescentOptimizer", lr=0.001)
    monkeypatch.setenv("CSA_GRAPH_STEPS", "4")
    a = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=True, stream_chunk=6)
    b = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=True, stream_chunk=6)
    a.step()
    a.prepare_group_graph()
    assert a.graph_k is not None
    a.run_steps(17)
    for _ in range(18):
        b.step()
    torch.cuda.synchronize()
    assert a.host_step == b.host_step == 18
    assert int(a.dstep.item()) == int(b.dstep.item()) == 18
    assert int(a.stream.cursor.item()) == int(b.stream.cursor.item())
    assert (a.flat - b.flat).abs().max().item() < 1e-3
    ma, mb = a.metrics_since(0), b.metrics_since(0)
    assert abs(ma["loss"] - mb["loss"]) < 1e-3 * max(1.0, mb["loss"])


@pytest.mark.parametrize("name", ["sample", "dense3_act"])
def test_horizontal_fusion_matches_fused_program(monkeypatch, name):
    """Round-4 program: every dense layer's weight gradient + update is deferred into the
    pair backward launch (conv_pair_bwd_upd_kernel), the input gradients run alone, and the
    last dense layer's input gradient rides in the head launch (csa_head_dgrad).  Several
    Adam / Adagrad steps (graph-captured) match the round-3 fused program and the metric
    ring agrees."""
    ds = synthetic_mnist(600, seed=17)
    for opt in ("AdamOptimizer", "AdagradOptimizer"):
        cfg = _cfg(CASES[name], optimizer=opt, lr=1e-3)
        monkeypatch.setenv("CSA_HFUSE", "1")
        a = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=True)
        monkeypatch.setenv("CSA_HFUSE", "0")
        b = TrainEngine(cfg, ds, device="cuda", backend="hip", use_graph=True)
        assert a.program.hfuse and a.program.head_dgrad and not b.program.hfuse
        for _ in range(5):
            a.step()
            b.step()
        torch.cuda.synchronize()
        d = (a.flat - b.flat).abs().max().item()
        assert d < 2e-4, f"{name}/{opt}: horizontal-fusion vs fused params differ by {d}"
        ma, mb = a.metrics_since(0), b.metrics_since(0)
        assert abs(ma["loss"] - mb["loss"]) < 1e-3 * max(1.0, mb["loss"])
        assert ma["accuracy"] == mb["accuracy"]
        assert int(a.dstep.item()) == int(b.dstep.item()) == 5
