"""The DSL-built digit CNN (reference ``cnn()``, construct_distribute.py:208-265).

Parameters live in ONE flat fp32 buffer (``FlatState``) with every named tensor a view
into it.  That layout is what the MI355X path is built around:

* the fused optimizer kernel updates all 2.28 M parameters in one launch,
* data-parallel gradient sync is one (or a few) large RCCL collectives over the flat
  gradient buffer instead of one call per tensor,
* checkpoints are a single contiguous copy.

Tensors use the reference's layouts: activations NHWC, conv weights HWIO
(``[kh, kw, cin, cout]``), dense weights ``[in, out]`` so the flatten order (H, W, C)
matches construct_distribute.py:176-178.

``DigitNet.forward`` here is the eager PyTorch implementation — the numerics oracle
for the HIP kernels and the CPU path used by tests.  The MI355X training step lives in
``cloud_server_amd.runtime.engine`` and calls the fused kernels in ``ops``.
"""
from __future__ import annotations

import math
from typing import Dict, Iterator, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .dsl import (ActSpec, ConvSpec, DenseSpec, LayerPlan, NetPlan, NormSpec, PoolSpec,
                  TrainConfig)


def trunc_normal_(t: torch.Tensor, std: float, gen: Optional[torch.Generator] = None) -> torch.Tensor:
    """tf.truncated_normal: N(0, std) redrawn outside ±2 std (construct_distribute.py:72-78)."""
    with torch.no_grad():
        t.normal_(0.0, 1.0, generator=gen)
        for _ in range(8):
            bad = t.abs() > 2.0
            if not bool(bad.any()):
                break
            t[bad] = torch.randn(int(bad.sum()), generator=gen, dtype=t.dtype, device=t.device)
        t.clamp_(-2.0, 2.0).mul_(std)
    return t


class FlatState:
    """Contiguous storage for named tensors, with named views (params, grads, optimizer slots)."""

    ALIGN = 64  # elements (256 B): every tensor starts 256-B aligned for dwordx4 access

    def __init__(self, shapes: Dict[str, Tuple[int, ...]], device="cpu", dtype=torch.float32,
                 pad_multiple: int = 1):
        self.shapes = dict(shapes)
        self.offsets: Dict[str, int] = {}
        off = 0
        for k, s in self.shapes.items():
            self.offsets[k] = off
            n = math.prod(s)
            off += -(-n // self.ALIGN) * self.ALIGN
        m = self.ALIGN * max(1, pad_multiple)   # sharded ("ps") mode needs numel % world == 0
        self.numel = -(-off // m) * m
        self.buffer = torch.zeros(self.numel, device=device, dtype=dtype)

    def view(self, name: str, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        buf = self.buffer if buf is None else buf
        o, s = self.offsets[name], self.shapes[name]
        return buf[o:o + math.prod(s)].view(s)

    def views(self, buf: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        return {k: self.view(k, buf) for k in self.shapes}

    def like(self) -> torch.Tensor:
        return torch.zeros_like(self.buffer)


def init_params(plan: NetPlan, state: FlatState, seed: int = 0) -> None:
    """Reference initialisers: trunc-normal σ / zeros / 'xavier' (σ/fan_in), bias 0.1,
    BN scale 1 offset 0 (construct_distribute.py:57-87, 155-165, 180-181, 262-263)."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    host = torch.zeros(state.numel, dtype=torch.float32)
    for lp in plan.layers:
        sp = lp.spec
        if isinstance(sp, ConvSpec):
            w = state.view(f"{lp.name}.weight", host)
            if sp.init == "zero":
                w.zero_()
            elif sp.init == "xavier":
                kh, kw, cin, _ = w.shape
                trunc_normal_(w, sp.stddev / float(kw * cin * w.shape[3]), gen)  # shape[1]*[2]*[3] (:80)
            else:
                trunc_normal_(w, sp.stddev, gen)
            if sp.bias:
                state.view(f"{lp.name}.bias", host).fill_(sp.bias_constant)
        elif isinstance(sp, DenseSpec):
            trunc_normal_(state.view(f"{lp.name}.weight", host), 0.1, gen)
            state.view(f"{lp.name}.bias", host).fill_(0.1)
        elif isinstance(sp, NormSpec):
            state.view(f"{lp.name}.scale", host).fill_(1.0)
            state.view(f"{lp.name}.offset", host).zero_()
    trunc_normal_(state.view("head.weight", host), 0.1, gen)
    state.view("head.bias", host).fill_(0.1)
    state.buffer.copy_(host)


def act_fwd(x: torch.Tensor, sp: ActSpec) -> torch.Tensor:
    if sp.func == "relu":
        return torch.relu(x)
    if sp.func == "leaky_relu":
        return torch.maximum(x, sp.alpha * x)   # tf.maximum(x, a*x) (:148-151)
    return torch.sigmoid(x)


def _global_moments(h: torch.Tensor, dims) -> "tuple[torch.Tensor, torch.Tensor]":
    """Biased mean / variance of ``h`` over ``dims`` AND over every rank of the default
    process group: one all-reduce of [sum, sum of squares, count] (2C + 1 floats)."""
    import torch.distributed as dist
    from torch.distributed.nn.functional import all_reduce
    C = h.shape[-1]
    n = torch.full((1,), float(h.numel() // C), dtype=h.dtype, device=h.device)
    st = torch.cat([h.sum(dim=dims), (h * h).sum(dim=dims), n])
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        st = all_reduce(st)
    cnt = st[2 * C]
    mean = st[:C] / cnt
    var = (st[C:2 * C] / cnt - mean * mean).clamp_min(0.0)
    return mean, var


class DigitNet(nn.Module):
    """Eager model over a ``FlatState``.  ``forward(x)`` takes NHWC [B,28,28,1] or [B,784]."""

    def __init__(self, plan: NetPlan, device="cpu", seed: int = 0, bn_mode: str = "running",
                 bn_momentum: float = 0.1, pad_multiple: int = 1, dense_last: bool = False):
        super().__init__()
        self.plan = plan
        self.bn_mode = bn_mode
        self.bn_momentum = bn_momentum
        # SyncBN: under data parallelism the reference's single worker
        # normalised over its whole batch; with sync_bn the per-channel {sum, sum of
        # squares, count} are all-reduced (autograd-aware, so the backward statistics are
        # global too) and every replica normalises with the GLOBAL batch statistics
        self.sync_bn = False
        self.deterministic = False          # CSA_DETERMINISTIC: atomics-free op choices
        self.state = FlatState(plan.param_shapes(dense_last), device=device, pad_multiple=pad_multiple)
        init_params(plan, self.state, seed)
        self.flat = nn.Parameter(self.state.buffer)
        self.state.buffer = self.flat.data
        # running BN statistics (fix for quirk 3); NOT part of the optimised flat buffer
        for lp in plan.layers:
            if isinstance(lp.spec, NormSpec):
                c = lp.in_shape.c
                self.register_buffer(f"bn{lp.index}_mean", torch.zeros(c, device=device))
                self.register_buffer(f"bn{lp.index}_var", torch.ones(c, device=device))

    # ---- named parameter views (grad flows to self.flat) ----
    def p(self, name: str) -> torch.Tensor:
        o, s = self.state.offsets[name], self.state.shapes[name]
        return self.flat[o:o + math.prod(s)].view(s)

    def named_tensors(self) -> Dict[str, torch.Tensor]:
        return {k: self.p(k) for k in self.state.shapes}

    def forward(self, x: torch.Tensor, use_batch_stats: Optional[bool] = None) -> torch.Tensor:
        if use_batch_stats is None:
            use_batch_stats = self.training or self.bn_mode == "batch"
        B = x.shape[0]
        h = x.reshape(B, 28, 28, 1) if x.dim() == 2 else x
        for lp in self.plan.layers:
            h = self._layer(lp, h, use_batch_stats)
        if h.dim() != 2:
            h = h.reshape(B, -1)  # quirk 2 fixed: flatten the LAST hidden tensor
        return h @ self.p("head.weight") + self.p("head.bias")

    def _layer(self, lp: LayerPlan, h: torch.Tensor, use_batch_stats: bool) -> torch.Tensor:
        sp = lp.spec
        if isinstance(sp, ConvSpec):
            pt, pb, pl, pr = lp.pads
            t = h.permute(0, 3, 1, 2)
            if any(lp.pads):
                t = F.pad(t, (pl, pr, pt, pb))
            w = self.p(f"{lp.name}.weight").permute(3, 2, 0, 1)
            b = self.p(f"{lp.name}.bias") if sp.bias else None
            return F.conv2d(t, w, b, stride=sp.stride).permute(0, 2, 3, 1)
        if isinstance(sp, PoolSpec):
            pt, pb, pl, pr = lp.pads
            t = h.permute(0, 3, 1, 2)
            if any(lp.pads):
                t = F.pad(t, (pl, pr, pt, pb), value=float("-inf"))
            if self.deterministic:
                # gather-form max pool: unfold + max (backward = one scatter per window +
                # col2im, both free of atomics) instead of max_pool2d's atomic backward
                Bn, Cn, Hn, Wn = t.shape
                kh, kw = sp.kernel
                oh, ow = (Hn - kh) // sp.stride[0] + 1, (Wn - kw) // sp.stride[1] + 1
                cols = F.unfold(t, (kh, kw), stride=sp.stride).view(Bn, Cn, kh * kw, oh * ow)
                return cols.max(dim=2).values.view(Bn, Cn, oh, ow).permute(0, 2, 3, 1)
            return F.max_pool2d(t, sp.kernel, sp.stride).permute(0, 2, 3, 1)
        if isinstance(sp, ActSpec):
            return act_fwd(h, sp)
        if isinstance(sp, NormSpec):
            dims = tuple(range(h.dim() - 1))
            scale, offset = self.p(f"{lp.name}.scale"), self.p(f"{lp.name}.offset")
            rm, rv = getattr(self, f"bn{lp.index}_mean"), getattr(self, f"bn{lp.index}_var")
            if use_batch_stats and self.sync_bn and self.training:
                mean, var = _global_moments(h, dims)
                with torch.no_grad():
                    m = self.bn_momentum
                    rm.mul_(1 - m).add_(mean.detach(), alpha=m)
                    rv.mul_(1 - m).add_(var.detach(), alpha=m)
            elif use_batch_stats:
                mean = h.mean(dim=dims)
                var = h.var(dim=dims, unbiased=False)   # tf.nn.moments: biased
                if self.training:
                    with torch.no_grad():
                        m = self.bn_momentum
                        rm.mul_(1 - m).add_(mean.detach(), alpha=m)
                        rv.mul_(1 - m).add_(var.detach(), alpha=m)
            else:
                mean, var = rm, rv
            return (h - mean) * torch.rsqrt(var + sp.epsilon) * scale + offset
        if isinstance(sp, DenseSpec):
            if h.dim() != 2:
                h = h.reshape(h.shape[0], -1)
            return h @ self.p(f"{lp.name}.weight") + self.p(f"{lp.name}.bias")
        raise TypeError(sp)

    # ---- checkpoint helpers: named keys derived from layer index (quirk 14 fixed) ----
    def export_state(self) -> Dict[str, torch.Tensor]:
        out = {k: v.detach().clone().cpu() for k, v in self.named_tensors().items()}
        for name, buf in self.named_buffers():
            out["buffers." + name] = buf.detach().clone().cpu()
        return out

    def import_state(self, sd: Dict[str, torch.Tensor]) -> None:
        with torch.no_grad():
            for k, v in self.named_tensors().items():
                if k not in sd:
                    raise KeyError(f"checkpoint missing {k}")
                v.copy_(sd[k].to(v.device).view(v.shape))
            for name, buf in self.named_buffers():
                key = "buffers." + name
                if key in sd:
                    buf.copy_(sd[key].to(buf.device))


def loss_fn(name: str, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """construct_distribute.py:285-298.  ``labels`` are int class ids; one-hot is implicit."""
    if name == "mse":
        onehot = F.one_hot(labels.long(), logits.shape[1]).to(logits.dtype)
        return ((onehot - logits) ** 2).mean()
    return F.cross_entropy(logits, labels.long())


def build_model(cfg: TrainConfig, device="cpu", pad_multiple: int = 1,
                dense_last: bool = False) -> DigitNet:
    return DigitNet(cfg.plan(), device=device, seed=cfg.seed, bn_mode=cfg.bn_mode,
                    pad_multiple=pad_multiple, dense_last=dense_last)
