"""CSA_DETERMINISTIC=1 (SURVEY §5.2 "deterministic mode for kernel tests"): two runs of
the same job are bitwise identical (CPU here; the GPU variant is in the @gpu test)."""
import copy

import pytest
import torch

from cloud_server_amd.data.datasets import synthetic_mnist
from cloud_server_amd.models.dsl import SAMPLE_CONFIG, parse_train_config
from cloud_server_amd.runtime.engine import TrainEngine


def _run(device, steps=6):
    c = copy.deepcopy(SAMPLE_CONFIG)
    c["net_config"]["middle_layer"] = [
        {"layer": "conv", "filter": [3, 3, 6], "isBias": "True"}, {"layer": "active", "active_func": "relu"},
        {"layer": "pool", "kernel": [3, 3], "stride": [2, 2]}, {"layer": "norm"},
        {"layer": "connect", "hidden": 32}]
    c.update(optimizer_name="AdamOptimizer", learning_rate=1e-3)
    c["options"] = dict(batch_size=16)
    eng = TrainEngine(parse_train_config(c), synthetic_mnist(200, seed=1), device=device)
    for _ in range(steps):
        eng.step()
    eng.sync_device()
    return eng


def test_deterministic_mode_bitwise_cpu(monkeypatch):
    monkeypatch.setenv("CSA_DETERMINISTIC", "1")
    try:
        a, b = _run("cpu"), _run("cpu")
        assert a.deterministic and a.backend == "torch"
        assert torch.equal(a.flat, b.flat) and torch.equal(a.slots, b.slots)
    finally:
        torch.use_deterministic_algorithms(False)


def test_deterministic_pool_matches_max_pool():
    """The gather-form pool used in deterministic mode == F.max_pool2d (values and grads)."""
    x = torch.randn(4, 9, 9, 3, dtype=torch.float64, requires_grad=True)
    c = copy.deepcopy(SAMPLE_CONFIG)
    c["net_config"]["middle_layer"] = [{"layer": "conv", "filter": [3, 3, 3]},
                                       {"layer": "pool", "kernel": [3, 3], "stride": [2, 2]}]
    eng = TrainEngine(parse_train_config(c), synthetic_mnist(50, seed=1), device="cpu")
    lp = eng.model.plan.layers[1]
    outs = []
    for det in (False, True):
        eng.model.deterministic = det
        y = eng.model._layer(lp, x, True)
        g, = torch.autograd.grad((y * torch.arange(y.numel(), dtype=y.dtype).view_as(y)).sum(), x)
        outs.append((y.detach(), g))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=0, atol=0)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=0, atol=0)


@pytest.mark.gpu
def test_deterministic_mode_bitwise_gpu(monkeypatch):
    monkeypatch.setenv("CSA_DETERMINISTIC", "1")
    try:
        a, b = _run("cuda:0", steps=20), _run("cuda:0", steps=20)
        # conv + relu + overlapping 3x3/2 pool (a standalone gather-form unit in this mode)
        # + norm + dense: on the HIP kernels since round 4
        assert a.backend == "hip" and a.program.det and a.use_graph, a.fallback_reason
        assert torch.equal(a.flat, b.flat) and torch.equal(a.slots, b.slots)
    finally:
        torch.use_deterministic_algorithms(False)


def _sample_engine(device, use_graph=True, opt="AdagradOptimizer", lr=0.01, n=600, seed=7):
    c = copy.deepcopy(SAMPLE_CONFIG)
    c.update(optimizer_name=opt, learning_rate=lr)
    c["options"] = dict(batch_size=50)
    return TrainEngine(parse_train_config(c), synthetic_mnist(n, seed=seed), device=device,
                       backend="hip", use_graph=use_graph)


@pytest.mark.gpu
def test_deterministic_hip_kernels_bitwise_gpu(monkeypatch):
    """The sample config keeps the HIP program in deterministic mode (exclusive statistic
    rows / weight-gradient stripes per workgroup, fixed-order folds, no split-K): two
    graph runs of 20 steps, an eager run, and a run of 8-step graphs are bitwise equal."""
    monkeypatch.setenv("CSA_DETERMINISTIC", "1")
    runs = []
    for mode in ("graph", "graph", "eager", "group"):
        eng = _sample_engine("cuda:0", use_graph=mode != "eager")
        assert eng.backend == "hip" and eng.program.det, eng.fallback_reason
        if mode == "group":
            eng.step()
            eng.run_steps(19)
        else:
            for _ in range(20):
                eng.step()
        eng.sync_device()
        assert int(eng.dstep.item()) == 20
        runs.append((eng.flat.clone(), eng.slots.clone(), eng.metrics_since(0)["loss"]))
    for i in range(1, len(runs)):
        assert torch.equal(runs[0][0], runs[i][0]), f"run {i}: params differ"
        assert torch.equal(runs[0][1], runs[i][1]), f"run {i}: optimizer slots differ"
        assert runs[0][2] == runs[i][2]


@pytest.mark.gpu
def test_deterministic_hip_matches_torch_and_fast_path(monkeypatch):
    """Deterministic-mode gradients (one SGD step) agree with the fp32 eager reference and
    with the atomic fast path to fp32 reassociation noise."""
    def grads(det, backend):
        monkeypatch.setenv("CSA_DETERMINISTIC", "1" if det else "0")
        c = copy.deepcopy(SAMPLE_CONFIG)
        c.update(optimizer_name="GradientDescentOptimizer", learning_rate=0.5)
        c["options"] = dict(batch_size=50)
        cfg = parse_train_config(c)
        eng = TrainEngine(cfg, synthetic_mnist(300, seed=13), device="cuda:0", backend=backend, use_graph=False)
        if backend == "hip":
            assert eng.backend == "hip" and eng.program.det == det
        w0 = eng.flat.clone()
        eng.step()
        eng.sync_device()
        return eng, (w0 - eng.flat) / cfg.effective_lr
    try:
        e_det, g_det = grads(True, "hip")
        _, g_fast = grads(False, "hip")
        _, g_ref = grads(False, "torch")
    finally:
        torch.use_deterministic_algorithms(False)
    for k in e_det.model.state.shapes:
        a = e_det.model.state.view(k, g_det)
        for other, tol in ((g_ref, 3e-3), (g_fast, 3e-3)):
            b = e_det.model.state.view(k, other)
            scale = b.abs().max().item() + 1e-6
            assert (a - b).abs().max().item() <= tol * scale + 1e-6, k


def test_launch_profile_flags_are_per_thread():
    """The deterministic / packed launch-profile flags are host state of the calling thread:
    a job planned or warmed up on the packed host's builder thread never changes the launch
    shapes of the jobs stepping on the main thread (runs on CPU: host-only library calls)."""
    import threading
    from cloud_server_amd.ops import fused as K

    lib = K.load(required=False)
    if lib is None:
        pytest.skip("kernel library not built")
    lib.csa_set_deterministic(0)
    lib.csa_set_packed(0)
    seen = {}

    def other():
        lib.csa_set_deterministic(1)
        lib.csa_set_packed(1)
        seen["other"] = (lib.csa_deterministic(), lib.csa_packed())

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen["other"] == (1, 1)
    assert (lib.csa_deterministic(), lib.csa_packed()) == (0, 0)


DET_CASES = ("five_biased_convs", "wide_conv_192", "dense_norm_head", "pool_after_norm_act")


@pytest.mark.gpu
@pytest.mark.parametrize("name", DET_CASES)
def test_deterministic_hip_every_lowering_bitwise(monkeypatch, name):
    """deterministic mode on the conv units (exclusive statistic rows and
    weight-gradient stripes per workgroup, folded in row order), standalone BatchNorm
    units, gconv units, gather-form pools and the partial-row head — the HIP program stays
    on (no eager fallback), two graph runs and an eager run are bitwise equal, and one
    step's gradients match the fp32 eager reference."""
    from test_hip_step import CASES, _cfg

    monkeypatch.setenv("CSA_DETERMINISTIC", "1")
    try:
        runs = []
        for mode in ("graph", "graph", "eager"):
            cfg = _cfg(CASES[name], optimizer="AdamOptimizer", lr=1e-3)
            eng = TrainEngine(cfg, synthetic_mnist(400, seed=5), device="cuda:0", backend="hip",
                              use_graph=mode == "graph")
            assert eng.backend == "hip" and eng.program.det, eng.fallback_reason
            for _ in range(8):
                eng.step()
            eng.sync_device()
            runs.append((eng.flat.clone(), eng.slots.clone(), eng.metrics_since(0)["loss"]))
        for i in (1, 2):
            assert torch.equal(runs[0][0], runs[i][0]), f"run {i}: params differ"
            assert torch.equal(runs[0][1], runs[i][1]), f"run {i}: optimizer slots differ"
            assert runs[0][2] == runs[i][2]

        def grads(backend):
            cfg = _cfg(CASES[name])
            eng = TrainEngine(cfg, synthetic_mnist(300, seed=13), device="cuda:0", backend=backend,
                              use_graph=False)
            w0 = eng.flat.clone()
            eng.step()
            eng.sync_device()
            return eng, (w0 - eng.flat) / cfg.effective_lr

        e_det, g_det = grads("hip")
        assert e_det.program.det
        _, g_ref = grads("torch")
    finally:
        torch.use_deterministic_algorithms(False)
    # (a gradient that is 0 in exact arithmetic — a conv bias feeding a BatchNorm — is fp32
    # summation noise in both programs: bounded against the model's largest gradient, as in
    # test_hip_step.py)
    gmax = g_ref.abs().max().item()
    for k in e_det.model.state.shapes:
        a, b = e_det.model.state.view(k, g_det), e_det.model.state.view(k, g_ref)
        scale = b.abs().max().item() + 1e-6
        assert (a - b).abs().max().item() <= 3e-3 * scale + 1e-6 + 1e-5 * gmax, k


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [80, 300])
def test_deterministic_hip_large_batch_bitwise(monkeypatch, batch):
    """the last two eager fallbacks of deterministic mode are gone.
    Batch 80: the dense layers take the materialised-gradient GEMMs (the fused backward +
    update covers M <= 64), fc1 reading a BatchNorm'd input — its backward statistics go to
    exclusive slab rows, folded in order (gemm.hip).  Batch 300: beyond the partial-row head
    (M <= 256), the single-workgroup generic head.  The HIP program stays on, two graph runs
    and an eager run are bitwise equal, and one step's gradients match the fp32 reference."""
    from test_hip_step import CASES, _cfg

    monkeypatch.setenv("CSA_DETERMINISTIC", "1")
    try:
        runs = []
        for mode in ("graph", "graph", "eager"):
            cfg = _cfg(CASES["sample"], optimizer="AdamOptimizer", lr=1e-3, batch=batch)
            eng = TrainEngine(cfg, synthetic_mnist(700, seed=5), device="cuda:0", backend="hip",
                              use_graph=mode == "graph")
            assert eng.backend == "hip" and eng.program.det, eng.fallback_reason
            if batch == 80:
                assert any(u.kind == "dense" and not u.fused and u.in_tf.has_bn for u in eng.program.units)
            else:
                assert not (eng.program.head_row or eng.program.head_rg)
            for _ in range(6):
                eng.step()
            eng.sync_device()
            runs.append((eng.flat.clone(), eng.slots.clone(), eng.metrics_since(0)["loss"]))
        for i in (1, 2):
            assert torch.equal(runs[0][0], runs[i][0]), f"run {i}: params differ"
            assert torch.equal(runs[0][1], runs[i][1]), f"run {i}: optimizer slots differ"
            assert runs[0][2] == runs[i][2]

        def grads(backend):
            cfg = _cfg(CASES["sample"], batch=batch)
            eng = TrainEngine(cfg, synthetic_mnist(600, seed=13), device="cuda:0", backend=backend,
                              use_graph=False)
            w0 = eng.flat.clone()
            eng.step()
            eng.sync_device()
            return eng, (w0 - eng.flat) / cfg.effective_lr

        e_det, g_det = grads("hip")
        assert e_det.program.det
        _, g_ref = grads("torch")
    finally:
        torch.use_deterministic_algorithms(False)
    gmax = g_ref.abs().max().item()
    for k in e_det.model.state.shapes:
        a, b = e_det.model.state.view(k, g_det), e_det.model.state.view(k, g_ref)
        scale = b.abs().max().item() + 1e-6
        assert (a - b).abs().max().item() <= 3e-3 * scale + 1e-6 + 1e-5 * gmax, k
