"""DSL parsing / shape inference / eager model (CPU).

Reference: construct_distribute.py:57-298 (layer builders, defaults, loss) and the
sample config of API.md:306-332 (2,276,218 parameters)."""
import copy
import math

import pytest
import torch

from cloud_server_amd.models.cnn import DigitNet, FlatState, build_model, loss_fn
from cloud_server_amd.models.dsl import (SAMPLE_CONFIG, ConfigError, ConvSpec, DenseSpec, PoolSpec,
                                         parse_train_config, plan_network, same_pads)
from cloud_server_amd.models.options import CATALOG, DSL_TOKENS, get_options
from cloud_server_amd.ops import optim_ref


def test_sample_config_param_count():
    cfg = parse_train_config(SAMPLE_CONFIG)
    plan = cfg.plan()
    assert plan.num_params() == 2_276_218
    assert plan.head_in == 512
    # conv(2x2x10) SAME keeps 28x28; conv(2x2x20) -> 28x28x20; pool -> 14x14x20 = 3920
    assert plan.layers[2].out_shape.hw == (14, 14) and plan.layers[2].out_shape.c == 20


def test_same_padding_even_kernel_pads_after():
    out, before, after = same_pads(28, 2, 1)
    assert (out, before, after) == (28, 0, 1)
    assert same_pads(28, 3, 2) == (14, 0, 1)
    assert same_pads(7, 2, 2) == (4, 0, 1)


def test_numbers_as_strings_and_quirks():
    cfg = copy.deepcopy(SAMPLE_CONFIG)
    cfg["iter"] = "20"
    cfg["learning_rate"] = "0.5"
    cfg["optimizer_name"] = "SomethingElse"          # -> Adagrad, as in the reference
    cfg["net_config"]["middle_layer"][0]["isBias"] = "False"
    cfg["net_config"]["middle_layer"].append({"layer": "unknown_layer"})   # skipped
    tc = parse_train_config(cfg)
    assert tc.iter == 20 and tc.learning_rate == 0.5
    assert tc.optimizer_name == "AdagradOptimizer"
    assert tc.layers[0].bias is False
    assert len(tc.layers) == 7
    tc2 = parse_train_config(dict(cfg, options={"compat_adagrad": True}))
    assert tc2.effective_optimizer == "AdagradOptimizer" and tc2.effective_lr == 1e-4


@pytest.mark.parametrize("bad", [
    {"net_config": {"middle_layer": [{"layer": "conv"}]}},
    {"net_config": {"middle_layer": [{"layer": "conv", "filter": [0, 2, 3]}]}},
    {"net_config": {"middle_layer": [{"layer": "pool", "padding": "FULL"}]}},
    {"net_config": {"middle_layer": [{"layer": "active", "active_func": "tanh"}]}},
    {"net_config": {"middle_layer": [{"layer": "connect", "hidden": -1}]}},
    {"loss_name": "hinge", "net_config": {"middle_layer": []}},
    {"ratio": 1.5, "net_config": {"middle_layer": []}},
    {"net_config": {"middle_layer": "conv"}},
    "not json",
])
def test_config_errors(bad):
    with pytest.raises(ConfigError):
        parse_train_config(bad)


def test_valid_padding_shape_error():
    with pytest.raises(ConfigError):
        parse_train_config({"net_config": {"middle_layer": [
            {"layer": "conv", "filter": [5, 5, 4], "padding": "VALID"},
            {"layer": "pool", "kernel": [2, 2], "stride": [2, 2], "padding": "VALID"},
            {"layer": "conv", "filter": [20, 20, 4], "padding": "VALID"}]}})


def test_options_catalog():
    for name, entry in CATALOG.items():
        o = get_options(name)
        assert o["default"] in o["options"]
        assert all(opt in DSL_TOKENS for opt in o["options"])
    with pytest.raises(KeyError):
        get_options("nope")


def test_flat_state_alignment_and_views():
    st = FlatState({"a": (3, 5), "b": (7,)}, pad_multiple=4)
    assert st.offsets["a"] % 64 == 0 and st.offsets["b"] % 64 == 0
    assert st.buffer.numel() % 4 == 0
    st.view("a").fill_(2.0)
    assert st.buffer[st.offsets["a"]:st.offsets["a"] + 15].eq(2).all()


def _ref_forward(net: DigitNet, x):
    """Independent NCHW re-implementation of the same net (torch.nn.functional)."""
    import torch.nn.functional as F
    h = x.view(-1, 1, 28, 28)
    for lp in net.plan.layers:
        sp = lp.spec
        if isinstance(sp, ConvSpec):
            pt, pb, pl, pr = lp.pads
            h = F.pad(h, (pl, pr, pt, pb))
            h = F.conv2d(h, net.p(f"{lp.name}.weight").permute(3, 2, 0, 1), stride=sp.stride)
            if sp.bias:
                h = h + net.p(f"{lp.name}.bias").view(1, -1, 1, 1)
        elif isinstance(sp, PoolSpec):
            pt, pb, pl, pr = lp.pads
            h = F.max_pool2d(F.pad(h, (pl, pr, pt, pb), value=-1e30), sp.kernel, sp.stride)
        elif isinstance(sp, DenseSpec):
            if h.dim() == 4:
                h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)
            h = h @ net.p(f"{lp.name}.weight") + net.p(f"{lp.name}.bias")
        elif sp.kind == "active":
            h = torch.relu(h) if sp.func == "relu" else torch.sigmoid(h)
        elif sp.kind == "norm":
            dims = (0, 2, 3) if h.dim() == 4 else (0,)
            m, v = h.mean(dims, keepdim=True), h.var(dims, unbiased=False, keepdim=True)
            c = h.shape[1]
            shp = (1, c, 1, 1) if h.dim() == 4 else (1, c)
            h = (h - m) / torch.sqrt(v + sp.epsilon) * net.p(f"{lp.name}.scale").view(shp) + \
                net.p(f"{lp.name}.offset").view(shp)
    if h.dim() == 4:
        h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)
    return h @ net.p("head.weight") + net.p("head.bias")


def test_model_matches_independent_reference():
    cfg = parse_train_config(SAMPLE_CONFIG)
    net = build_model(cfg)
    net.train()
    x = torch.rand(6, 784)
    with torch.no_grad():
        a = net(x)
        b = _ref_forward(net, x)
    assert a.shape == (6, 10)
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)


def test_init_distributions():
    cfg = parse_train_config({"net_config": {"middle_layer": [
        {"layer": "conv", "filter": [3, 3, 64], "init": "norm", "stddev_norm": 0.1, "isBias": "True"},
        {"layer": "connect", "hidden": 256}]}})
    net = build_model(cfg)
    w = net.p("layers.0.weight")
    assert w.abs().max() <= 0.2 + 1e-6          # truncated at 2 sigma
    assert 0.05 < w.std() < 0.1
    assert torch.allclose(net.p("layers.0.bias"), torch.full((64,), 0.1))
    assert torch.allclose(net.p("layers.1.bias"), torch.full((256,), 0.1))


def test_export_import_roundtrip():
    cfg = parse_train_config(SAMPLE_CONFIG)
    a, b = build_model(cfg), build_model(parse_train_config(dict(SAMPLE_CONFIG, options={"seed": 7})))
    assert not torch.equal(a.flat, b.flat)
    b.import_state(a.export_state())
    x = torch.rand(3, 784)
    a.eval(); b.eval()
    torch.testing.assert_close(a(x), b(x))


def test_losses():
    logits = torch.randn(5, 10)
    y = torch.tensor([0, 3, 9, 2, 2])
    onehot = torch.nn.functional.one_hot(y, 10).float()
    assert torch.allclose(loss_fn("mse", logits, y), ((onehot - logits) ** 2).mean())
    ref = -(torch.log_softmax(logits, 1) * onehot).sum(1).mean()
    assert torch.allclose(loss_fn("entropy", logits, y), ref)


@pytest.mark.parametrize("opt", [optim_ref.OPT_SGD, optim_ref.OPT_ADAGRAD, optim_ref.OPT_ADAM,
                                 optim_ref.OPT_ADADELTA])
def test_optimizer_reference_formulas(opt):
    torch.manual_seed(0)
    w0 = torch.randn(100)
    g = torch.randn(100)
    w = w0.clone()
    slots = optim_ref.init_slots(opt, 100, "cpu")
    optim_ref.step_ref(opt, w, g, slots, 0.1, 1)
    if opt == optim_ref.OPT_SGD:
        exp = w0 - 0.1 * g
    elif opt == optim_ref.OPT_ADAGRAD:
        exp = w0 - 0.1 * g / torch.sqrt(0.1 + g * g)            # TF initial accumulator 0.1
    elif opt == optim_ref.OPT_ADAM:
        lr_t = 0.1 * math.sqrt(1 - 0.999) / (1 - 0.9)
        m, v = 0.1 * g, 0.001 * g * g
        exp = w0 - lr_t * m / (torch.sqrt(v) + 1e-8)
    else:
        rho, eps = 0.95, 1e-8
        acc = (1 - rho) * g * g
        upd = math.sqrt(eps) / torch.sqrt(acc + eps) * g
        exp = w0 - 0.1 * upd
    torch.testing.assert_close(w, exp, rtol=1e-5, atol=1e-6)


def test_training_reduces_loss_cpu():
    from cloud_server_amd.data.datasets import synthetic_mnist
    from cloud_server_amd.runtime.engine import TrainEngine
    cfg = parse_train_config({"learning_rate": 0.05, "optimizer_name": "AdamOptimizer",
                              "options": {"batch_size": 32},
                              "net_config": {"middle_layer": [
                                  {"layer": "conv", "filter": [3, 3, 8]}, {"layer": "active", "active_func": "relu"},
                                  {"layer": "pool"}, {"layer": "norm"}, {"layer": "connect", "hidden": 32},
                                  {"layer": "active", "active_func": "relu"}]}})
    ds = synthetic_mnist(2000, seed=1)
    eng = TrainEngine(cfg, ds, device="cpu")
    for _ in range(120):
        eng.step()
    early = eng.ring_loss[:10].mean().item()
    late = eng.ring_loss[110:120].mean().item()
    assert late < 0.5 * early
    assert eng.evaluate(synthetic_mnist(500, seed=2)) > 0.8


def test_dense_last_layout_same_params_by_name():
    """The "lowrank" DP strategy lays the flat buffer out dense-last (conv/BN/head first)
    so its all-reduced remainder is one range; values are identical by name."""
    cfg = parse_train_config(SAMPLE_CONFIG)
    a = build_model(cfg)
    b = build_model(cfg, dense_last=True)
    assert a.state.shapes.keys() == b.state.shapes.keys()
    names = list(b.state.offsets)
    dense = [lp.name for lp in cfg.plan().layers if isinstance(lp.spec, DenseSpec)]
    assert dense
    head_end = b.state.offsets["head.bias"]
    assert all(b.state.offsets[f"{n}.weight"] > head_end for n in dense)
    for n in names:
        assert torch.equal(a.state.view(n), b.state.view(n)), n
    x = torch.rand(4, 784)
    torch.testing.assert_close(a(x), b(x))
