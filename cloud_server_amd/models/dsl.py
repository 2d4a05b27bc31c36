"""Network-config DSL: the reference's ``model.json`` schema, validated and shape-inferred.

The reference accepts a JSON object (API.md:306-332) and walks ``net_config.middle_layer``
inside ``cnn()`` (apps/construction/util/construct_distribute.py:208-265) with per-layer
defaults read via ``key in every_inner.keys()`` checks.  Here the same JSON is parsed
once, on submit, into typed layer specs with explicit defaults, and the whole network is
shape-inferred so a bad config is rejected by the API instead of crashing a worker.

Reference quirks and how they are handled:

* quirk 1 – optimizer / learning rate ignored (construct_distribute.py:372): honoured
  here; ``compat_adagrad`` restores the hard-coded ``Adagrad(1e-4)``.
* quirk 2 – head flattens ``x`` instead of ``last`` (construct_distribute.py:257): fixed,
  the head flattens the last hidden tensor.
* quirk 3 – BN uses batch statistics at inference (construct_distribute.py:164):
  ``bn_mode="running"`` (default) keeps running stats for eval; ``"batch"`` is the compat mode.
* ``isBias`` is a string compare against ``"False"`` (construct_distribute.py:228): kept.
* unknown layer names are skipped silently in the reference; we keep them in the parsed
  config (so ``model.json`` round-trips) but they produce no layer.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field, asdict
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

INPUT_HW = 28          # construct_distribute.py:216 — input fixed 28x28x1
INPUT_C = 1
NUM_CLASSES = 10       # construct_distribute.py:261 — fixed 10-way head

LOSSES = ("entropy", "mse")
OPTIMIZERS = ("GradientDescentOptimizer", "AdagradOptimizer", "AdamOptimizer", "AdadeltaOptimizer")
ACTIVATIONS = ("sigmoid", "relu", "leaky_relu")
INITS = ("norm", "zero", "xavier")
PADDINGS = ("SAME", "VALID")


class ConfigError(ValueError):
    """Raised when a net config is invalid (API turns it into a 400)."""


def _as_int(v: Any, name: str) -> int:
    try:
        return int(v)
    except (TypeError, ValueError):
        raise ConfigError(f"{name}: expected int, got {v!r}")


def _as_float(v: Any, name: str) -> float:
    try:
        return float(v)
    except (TypeError, ValueError):
        raise ConfigError(f"{name}: expected float, got {v!r}")


def _pair(v: Any, name: str) -> Tuple[int, int]:
    if isinstance(v, (list, tuple)) and len(v) >= 2:
        return _as_int(v[0], name), _as_int(v[1], name)
    if isinstance(v, (int, float, str)):
        i = _as_int(v, name)
        return i, i
    raise ConfigError(f"{name}: expected [h, w], got {v!r}")


def same_pads(size: int, k: int, s: int) -> Tuple[int, int, int]:
    """TF 'SAME' padding: returns (out, pad_before, pad_after). Even kernels pad after."""
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return out, total // 2, total - total // 2


def valid_out(size: int, k: int, s: int) -> int:
    return (size - k) // s + 1


@dataclass
class ConvSpec:
    kh: int
    kw: int
    cout: int
    stride: Tuple[int, int] = (1, 1)
    padding: str = "SAME"
    init: str = "norm"
    bias: bool = False
    bias_constant: float = 0.1
    stddev: float = 0.1
    kind: str = "conv"


@dataclass
class PoolSpec:
    kernel: Tuple[int, int] = (2, 2)
    stride: Tuple[int, int] = (2, 2)
    padding: str = "SAME"
    kind: str = "pool"


@dataclass
class ActSpec:
    func: str = "sigmoid"
    alpha: float = 0.2
    kind: str = "active"


@dataclass
class DenseSpec:
    hidden: int = 512
    kind: str = "connect"


@dataclass
class NormSpec:
    epsilon: float = 1e-3
    kind: str = "norm"


LayerSpec = Union[ConvSpec, PoolSpec, ActSpec, DenseSpec, NormSpec]


def parse_layer(d: Dict[str, Any], idx: int) -> Optional[LayerSpec]:
    """One ``middle_layer`` entry -> spec (defaults from construct_distribute.py:219-250)."""
    if not isinstance(d, dict):
        raise ConfigError(f"middle_layer[{idx}] must be an object")
    name = d.get("layer")
    where = f"middle_layer[{idx}]"
    if name == "conv":
        if "filter" not in d:
            raise ConfigError(f"{where}: conv needs 'filter': [kh, kw, cout]")
        f = d["filter"]
        if not isinstance(f, (list, tuple)) or len(f) != 3:
            raise ConfigError(f"{where}: filter must be [kh, kw, cout]")
        kh, kw, cout = (_as_int(x, where + ".filter") for x in f)
        if min(kh, kw, cout) <= 0:
            raise ConfigError(f"{where}: filter dims must be positive")
        pad = str(d.get("padding", "SAME")).upper()
        init = str(d.get("init", "norm"))
        if pad not in PADDINGS:
            raise ConfigError(f"{where}: padding must be SAME or VALID")
        if init not in INITS:
            raise ConfigError(f"{where}: init must be one of {INITS}")
        stride = _pair(d.get("stride", [1, 1]), where + ".stride")
        if min(stride) <= 0:
            raise ConfigError(f"{where}: stride must be positive")
        # reference: isBias = every_inner["isBias"] != "False"  (string compare, :228)
        bias = ("isBias" in d) and (d["isBias"] != "False") and (d["isBias"] is not False)
        return ConvSpec(kh, kw, cout, stride, pad, init, bias,
                        _as_float(d.get("bias_constant", 0.1), where),
                        _as_float(d.get("stddev_norm", 0.1), where))
    if name == "pool":
        pad = str(d.get("padding", "SAME")).upper()
        if pad not in PADDINGS:
            raise ConfigError(f"{where}: padding must be SAME or VALID")
        k = _pair(d.get("kernel", [2, 2]), where + ".kernel")
        s = _pair(d.get("stride", [2, 2]), where + ".stride")
        if min(k) <= 0 or min(s) <= 0:
            raise ConfigError(f"{where}: kernel/stride must be positive")
        return PoolSpec(k, s, pad)
    if name == "active":
        func = str(d.get("active_func", "sigmoid"))
        if func not in ACTIVATIONS:
            raise ConfigError(f"{where}: active_func must be one of {ACTIVATIONS}")
        p = d.get("param", [0.2])
        alpha = _as_float(p[0], where + ".param") if isinstance(p, (list, tuple)) and p else 0.2
        return ActSpec(func, alpha)
    if name == "connect":
        h = _as_int(d.get("hidden", 512), where + ".hidden")
        if h <= 0:
            raise ConfigError(f"{where}: hidden must be positive")
        return DenseSpec(h)
    if name == "norm":
        return NormSpec(_as_float(d.get("epsilon", 1e-3), where + ".epsilon"))
    return None  # unknown layers are skipped, as in the reference (:208-250)


@dataclass
class TensorShape:
    """Per-sample activation shape. ``hw`` is None once flattened to a vector."""
    c: int
    hw: Optional[Tuple[int, int]] = None

    @property
    def numel(self) -> int:
        return self.c * (self.hw[0] * self.hw[1] if self.hw else 1)

    @property
    def is_spatial(self) -> bool:
        return self.hw is not None


@dataclass
class LayerPlan:
    """A spec bound to concrete input/output shapes and padding."""
    index: int
    spec: LayerSpec
    in_shape: TensorShape
    out_shape: TensorShape
    pads: Tuple[int, int, int, int] = (0, 0, 0, 0)   # top, bottom, left, right
    params: Dict[str, Tuple[int, ...]] = field(default_factory=dict)

    @property
    def name(self) -> str:
        return f"layers.{self.index}"


@dataclass
class NetPlan:
    layers: List[LayerPlan]
    head_in: int
    num_classes: int = NUM_CLASSES

    def param_shapes(self, dense_last: bool = False) -> Dict[str, Tuple[int, ...]]:
        """Named parameter shapes in flat-buffer order: DSL order, head last — or, with
        ``dense_last``, every non-dense parameter and the head first and the dense layers
        after them (the "lowrank" DP strategy all-reduces exactly that leading range)."""
        out: Dict[str, Tuple[int, ...]] = {}
        dense: Dict[str, Tuple[int, ...]] = {}
        for lp in self.layers:
            for k, s in lp.params.items():
                (dense if dense_last and isinstance(lp.spec, DenseSpec) else out)[f"{lp.name}.{k}"] = s
        out["head.weight"] = (self.head_in, self.num_classes)
        out["head.bias"] = (self.num_classes,)
        out.update(dense)
        return out

    def num_params(self) -> int:
        return sum(math.prod(s) for s in self.param_shapes().values())

    def flops_per_sample(self) -> int:
        """Forward multiply-add FLOPs (2/MAC) per sample for the matmul-like layers."""
        f = 0
        for lp in self.layers:
            sp = lp.spec
            if isinstance(sp, ConvSpec):
                oh, ow = lp.out_shape.hw
                f += 2 * oh * ow * sp.cout * sp.kh * sp.kw * lp.in_shape.c
            elif isinstance(sp, DenseSpec):
                f += 2 * lp.in_shape.numel * sp.hidden
        f += 2 * self.head_in * self.num_classes
        return f


def plan_network(layers: Sequence[LayerSpec], in_hw: int = INPUT_HW, in_c: int = INPUT_C,
                 num_classes: int = NUM_CLASSES) -> NetPlan:
    """Shape inference (replaces TF's graph-build-time shape checks)."""
    shape = TensorShape(in_c, (in_hw, in_hw))
    plans: List[LayerPlan] = []
    for i, sp in enumerate(layers):
        if isinstance(sp, ConvSpec):
            if not shape.is_spatial:
                raise ConfigError(f"layer {i}: conv after a connect layer (input is flat)")
            (h, w), (sh, sw) = shape.hw, sp.stride
            if sp.padding == "SAME":
                oh, pt, pb = same_pads(h, sp.kh, sh)
                ow, pl, pr = same_pads(w, sp.kw, sw)
            else:
                oh, ow, pt, pb, pl, pr = valid_out(h, sp.kh, sh), valid_out(w, sp.kw, sw), 0, 0, 0, 0
            if oh <= 0 or ow <= 0:
                raise ConfigError(f"layer {i}: conv kernel larger than its {h}x{w} input")
            params = {"weight": (sp.kh, sp.kw, shape.c, sp.cout)}
            if sp.bias:
                params["bias"] = (sp.cout,)
            out = TensorShape(sp.cout, (oh, ow))
            plans.append(LayerPlan(i, sp, shape, out, (pt, pb, pl, pr), params))
        elif isinstance(sp, PoolSpec):
            if not shape.is_spatial:
                raise ConfigError(f"layer {i}: pool after a connect layer (input is flat)")
            (h, w), (kh, kw), (sh, sw) = shape.hw, sp.kernel, sp.stride
            if sp.padding == "SAME":
                oh, pt, pb = same_pads(h, kh, sh)
                ow, pl, pr = same_pads(w, kw, sw)
            else:
                oh, ow, pt, pb, pl, pr = valid_out(h, kh, sh), valid_out(w, kw, sw), 0, 0, 0, 0
            if oh <= 0 or ow <= 0:
                raise ConfigError(f"layer {i}: pool window larger than its {h}x{w} input")
            plans.append(LayerPlan(i, sp, shape, TensorShape(shape.c, (oh, ow)), (pt, pb, pl, pr)))
        elif isinstance(sp, ActSpec):
            plans.append(LayerPlan(i, sp, shape, shape))
        elif isinstance(sp, NormSpec):
            plans.append(LayerPlan(i, sp, shape, shape, params={"scale": (shape.c,), "offset": (shape.c,)}))
        elif isinstance(sp, DenseSpec):
            fan_in = shape.numel
            out = TensorShape(sp.hidden, None)
            plans.append(LayerPlan(i, sp, shape, out,
                                   params={"weight": (fan_in, sp.hidden), "bias": (sp.hidden,)}))
        else:  # pragma: no cover
            raise ConfigError(f"layer {i}: unsupported spec {sp!r}")
        shape = plans[-1].out_shape
    return NetPlan(plans, shape.numel, num_classes)


@dataclass
class TrainConfig:
    """The whole ``model.json`` (API.md:306-332) in typed form."""
    iter: int = 1000
    learning_rate: float = 0.01
    ratio: float = 0.8
    loss_name: str = "entropy"
    optimizer_name: str = "GradientDescentOptimizer"
    net_type: str = "CNN"
    layers: List[LayerSpec] = field(default_factory=list)
    raw: Dict[str, Any] = field(default_factory=dict)
    # --- new-framework knobs (not in the reference JSON; all optional) ---
    batch_size: int = 50                   # construct_distribute.py:403 hard-codes 50
    log_every: int = 100                   # :405 — accuracy line every 100 global steps
    ckpt_every: int = 0                    # optional step-based checkpoints (0 = off)
    ckpt_secs: float = 60.0                # Supervisor(save_model_secs=60) (:391)
    bn_mode: str = "running"               # "batch" = reference quirk 3
    compat_adagrad: bool = False           # True = reference quirk 1 (Adagrad 1e-4)
    sync_bn: bool = False                  # DP: BatchNorm statistics over the GLOBAL batch
    seed: int = 0

    @property
    def effective_optimizer(self) -> str:
        return "AdagradOptimizer" if self.compat_adagrad else self.optimizer_name

    @property
    def effective_lr(self) -> float:
        return 1e-4 if self.compat_adagrad else self.learning_rate

    def plan(self) -> NetPlan:
        return plan_network(self.layers)

    def to_json(self) -> Dict[str, Any]:
        return dict(self.raw)


def parse_train_config(cfg: Union[str, bytes, Dict[str, Any]]) -> TrainConfig:
    """Parse the reference JSON verbatim (numbers may be strings, cf. cmd.py:63-69)."""
    if isinstance(cfg, (str, bytes)):
        try:
            cfg = json.loads(cfg)
        except json.JSONDecodeError as e:
            raise ConfigError(f"config is not valid JSON: {e}")
    if not isinstance(cfg, dict):
        raise ConfigError("config must be a JSON object")
    net = cfg.get("net_config")
    if not isinstance(net, dict) or not isinstance(net.get("middle_layer", []), list):
        raise ConfigError("net_config.middle_layer must be a list")
    layers = []
    for i, d in enumerate(net.get("middle_layer", [])):
        sp = parse_layer(d, i)
        if sp is not None:
            layers.append(sp)
    loss = str(cfg.get("loss_name", "entropy"))
    if loss not in LOSSES:
        raise ConfigError(f"loss_name must be one of {LOSSES}")
    opt = str(cfg.get("optimizer_name", "GradientDescentOptimizer"))
    if opt not in OPTIMIZERS:
        # reference: anything that is not GD falls back to Adagrad (construct_distribute.py:308-311)
        opt = "AdagradOptimizer"
    ext = cfg.get("options", {}) if isinstance(cfg.get("options", {}), dict) else {}
    tc = TrainConfig(
        iter=_as_int(cfg.get("iter", 1000), "iter"),
        learning_rate=_as_float(cfg.get("learning_rate", 0.01), "learning_rate"),
        ratio=_as_float(cfg.get("ratio", 0.8), "ratio"),
        loss_name=loss, optimizer_name=opt,
        net_type=str(cfg.get("net_type", "CNN")),
        layers=layers, raw=dict(cfg),
        batch_size=_as_int(ext.get("batch_size", 50), "batch_size"),
        log_every=_as_int(ext.get("log_every", 100), "log_every"),
        ckpt_every=_as_int(ext.get("ckpt_every", 0), "ckpt_every"),
        ckpt_secs=_as_float(ext.get("ckpt_secs", 60.0), "ckpt_secs"),
        bn_mode=str(ext.get("bn_mode", "running")),
        compat_adagrad=bool(ext.get("compat_adagrad", False)),
        sync_bn=str(ext.get("sync_bn", False)).lower() in ("1", "true", "yes"),
        seed=_as_int(ext.get("seed", 0), "seed"),
    )
    if tc.iter < 0:
        raise ConfigError("iter must be >= 0")
    if not (0.0 < tc.ratio <= 1.0):
        raise ConfigError("ratio must be in (0, 1]")
    if tc.learning_rate <= 0:
        raise ConfigError("learning_rate must be > 0")
    if tc.batch_size <= 0:
        raise ConfigError("batch_size must be > 0")
    if tc.bn_mode not in ("running", "batch"):
        raise ConfigError("bn_mode must be 'running' or 'batch'")
    tc.plan()  # shape-check now
    return tc


# The canonical sample config: API.md:306-332 (== a.sh:8 == cmd.py:89-93).
SAMPLE_CONFIG: Dict[str, Any] = {
    "iter": 1000,
    "learning_rate": 0.01,
    "ratio": 0.8,
    "loss_name": "entropy",
    "optimizer_name": "GradientDescentOptimizer",
    "net_type": "CNN",
    "net_config": {
        "middle_layer": [
            {"layer": "conv", "filter": [2, 2, 10]},
            {"layer": "conv", "filter": [2, 2, 20]},
            {"layer": "pool"},
            {"layer": "norm"},
            {"layer": "active"},
            {"layer": "connect"},
            {"layer": "connect"},
        ],
        "output_layer": {},
    },
}


def spec_to_dict(sp: LayerSpec) -> Dict[str, Any]:
    return asdict(sp)
