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
        assert a.backend == "torch" and a.use_graph
        assert torch.equal(a.flat, b.flat) and torch.equal(a.slots, b.slots)
    finally:
        torch.use_deterministic_algorithms(False)
